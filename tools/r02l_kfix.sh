#!/bin/bash
# Kappa fixpoint iterations (prep time vs kernel time): full C4 table, interleaved.
set -u
mkdir -p gpurun_out
for v in 6 12 6; do
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 --opt target_kappa=$v > gpurun_out/r02l_full_$v.log 2>&1 || { echo probe failed; tail -20 gpurun_out/r02l_full_$v.log; exit 1; }
  echo "kappa iters=$v"; grep -h "^rep 1\|prep" gpurun_out/r02l_full_$v.log
done
