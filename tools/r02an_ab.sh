#!/bin/bash
# Batch SSSP (pair rounds, RB 2): sweep loads in flight (SU) and hub speculation depth.
set -u
mkdir -p gpurun_out/r02an
bash tools/ab_probe.sh gpurun_out/r02an "base|-|--rows 10000 --reps 2" "su4|su4|--rows 10000 --reps 2" "su16|su16|--rows 10000 --reps 2" "spec0|spec0|--rows 10000 --reps 2" "spec2|spec2|--rows 10000 --reps 2" "base|-|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1|split ms" gpurun_out/r02an/ab.log
