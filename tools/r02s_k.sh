#!/bin/bash
# Batch width after the target-aware steps: K = 8 / 16 / 4 on the full C4 table, interleaved;
# then every shard of the 1/2/4/8-GPU splits (tools/scale_probe2.py).
set -u
mkdir -p gpurun_out
for k in 8 16 4 8 16; do
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 --opt batch=$k > gpurun_out/r02s_k$k.log 2>&1 || { echo probe failed; tail -20 gpurun_out/r02s_k$k.log; exit 1; }
  echo "K=$k"; grep -h -A1 "^rep 1" gpurun_out/r02s_k$k.log
done
timeout -k 10 400 python -u tools/scale_probe2.py > gpurun_out/r02r_scale.log 2>&1 || { echo scale failed; tail -20 gpurun_out/r02r_scale.log; exit 1; }
tail -6 gpurun_out/r02r_scale.log
