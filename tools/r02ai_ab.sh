#!/bin/bash
# Heap replay landmark skip: replay tests, then 5120 C4-int rows with the skip on / off (x2).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ai_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02ai_tests.log; exit 1; }
tail -1 gpurun_out/r02ai_tests.log
for lm in 1 0 1 0; do
  echo "== landmark $lm"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 0 all $lm || { echo probe failed; exit 1; }
done
