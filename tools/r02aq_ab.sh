#!/bin/bash
# Batch SSSP (pair rounds, RB 2): bucket width around the default 0.2 x mean latency (~10 ms).
set -u
mkdir -p gpurun_out/r02aq
bash tools/ab_probe.sh gpurun_out/r02aq "d10|-|--rows 10000 --reps 2" "d6|-|--rows 10000 --reps 2 --delta 6" "d8|-|--rows 10000 --reps 2 --delta 8" "d13|-|--rows 10000 --reps 2 --delta 13" "d16|-|--rows 10000 --reps 2 --delta 16" "d10|-|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1|per-source ms" gpurun_out/r02aq/ab.log
