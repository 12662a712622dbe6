#!/bin/bash
# Rows re-sorted by the target-aware key: every GPU parity test, then an interleaved A/B of the
# full C4 table and the 8-GPU shard size (target_resort 0 / 1).
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02m_gpu_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r02m_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02m_gpu_tests.log
for v in 1 0 1 0; do
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 --opt target_resort=$v > gpurun_out/r02m_full_$v.log 2>&1 || { echo probe failed; tail -20 gpurun_out/r02m_full_$v.log; exit 1; }
  echo "resort=$v"; grep -h -A1 "^rep 1" gpurun_out/r02m_full_$v.log; grep -h "prep\|parent phases\|split ms" gpurun_out/r02m_full_$v.log | tail -3
done
for v in 1 0; do
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 1250 --reps 3 --opt target_resort=$v > gpurun_out/r02m_1250_$v.log 2>&1 || { echo probe failed; exit 1; }
  echo "1250 resort=$v"; grep -A1 "^rep 2" gpurun_out/r02m_1250_$v.log
done
