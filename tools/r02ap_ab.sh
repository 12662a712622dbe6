#!/bin/bash
# Batch SSSP: 512-thread workgroups (8 waves per CU, 256 VGPRs per lane: no spills) vs 1024.
set -u
mkdir -p gpurun_out/r02ap
bash tools/ab_probe.sh gpurun_out/r02ap "base|-|--rows 10000 --reps 2" "b512rb4|b512rb4|--rows 10000 --reps 2" "b512rb2|b512rb2|--rows 10000 --reps 2" "b512rb8|b512rb8|--rows 10000 --reps 2" "base|-|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1" gpurun_out/r02ap/ab.log
