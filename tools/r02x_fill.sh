#!/bin/bash
# Batch fill: parity tests, then the strong-scaling probe (shard sizes of N = 1, 2, 4, 8).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02x_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02x_tests.log; exit 1; }
tail -1 gpurun_out/r02x_tests.log
timeout -k 10 300 python -u tools/scale_probe.py || { echo scale probe failed; exit 1; }
