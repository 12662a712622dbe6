#!/bin/bash
# C4-int exact table with the reworked replay (1 step), after the replay/parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_multi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02w_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02w_tests.log; exit 1; }
tail -1 gpurun_out/r02w_tests.log
timeout -k 10 500 python -u bench.py --integer --steps 1 --warmup 0 --no-cpu-baseline --no-complete --no-graphml > gpurun_out/r02w_bench_int.json 2> gpurun_out/r02w_bench_int.log || { echo bench failed; tail -20 gpurun_out/r02w_bench_int.log; exit 1; }
cat gpurun_out/r02w_bench_int.json
