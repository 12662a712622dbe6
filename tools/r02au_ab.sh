#!/bin/bash
# Batch SSSP: sweep rounds load the next pending-bitmap word ahead.
set -u
mkdir -p gpurun_out/r02au
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02au/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02au/tests.log; exit 1; }
tail -1 gpurun_out/r02au/tests.log
bash tools/ab_probe.sh gpurun_out/r02au "new|-|--rows 10000 --reps 2" "prev|prev|--rows 10000 --reps 2" "new|-|--rows 10000 --reps 2" "prev|prev|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1|split ms" gpurun_out/r02au/ab.log
