#!/bin/bash
# Target-aware kappa fixpoint: every GPU parity test (default iterations), then an interleaved
# A/B of the full C4 table and the 8-GPU shard size over the iteration cap (0 = kappa0).
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02j_gpu_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r02j_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02j_gpu_tests.log
for v in 0 32 2 8 0 32; do
  SHD_KFIX_LOG=1 timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 --opt target_kappa=$v > gpurun_out/r02j_full_$v.log 2>&1 || { echo probe failed; tail -20 gpurun_out/r02j_full_$v.log; exit 1; }
  echo "kappa iters=$v"; grep -h "kappa fixpoint\|^rep" gpurun_out/r02j_full_$v.log; grep -A1 "^rep 1" gpurun_out/r02j_full_$v.log | tail -1
done
for v in 0 32; do
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 1250 --reps 3 --opt target_kappa=$v > gpurun_out/r02j_1250_$v.log 2>&1 || { echo probe failed; exit 1; }
  echo "1250 kappa iters=$v"; grep -A1 "^rep 2" gpurun_out/r02j_1250_$v.log
done
