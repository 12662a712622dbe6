#!/bin/bash
# Heap replay, restored best variant: parity tests + one 5120-row probe.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ah_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02ah_tests.log; exit 1; }
tail -1 gpurun_out/r02ah_tests.log
timeout -k 10 200 python -u tools/replay_probe.py 5120 0 all || { echo probe failed; exit 1; }
