#!/bin/bash
# Batch SSSP: 8 kappa probes per vertex (binary search only past position 127) vs 4 (past 7).
set -u
mkdir -p gpurun_out/r02at
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02at/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02at/tests.log; exit 1; }
tail -1 gpurun_out/r02at/tests.log
bash tools/ab_probe.sh gpurun_out/r02at "kp8|-|--rows 10000 --reps 2" "kp4|kp4|--rows 10000 --reps 2" "kp8|-|--rows 10000 --reps 2" "kp4|kp4|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1|per-source ms" gpurun_out/r02at/ab.log
