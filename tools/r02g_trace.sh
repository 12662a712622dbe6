#!/bin/bash
# Per-batch timing of sssp_batch_kernel (SHD_BATCH_TRACE) on the full C4 table and on the
# 8-GPU shard size (1,250 rows): how long the slots idle at the kernel's end.
set -u
mkdir -p gpurun_out
rm -f gpurun_out/bt_full.bin gpurun_out/bt_1250.bin
SHD_BATCH_TRACE=gpurun_out/bt_full.bin timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 > gpurun_out/bt_full.log 2>&1 || { echo full failed; tail -20 gpurun_out/bt_full.log; exit 1; }
SHD_BATCH_TRACE=gpurun_out/bt_1250.bin timeout -k 10 300 python -u tools/gpu_probe.py --rows 1250 --reps 3 > gpurun_out/bt_1250.log 2>&1 || { echo 1250 failed; tail -20 gpurun_out/bt_1250.log; exit 1; }
grep -h "^rep" gpurun_out/bt_full.log gpurun_out/bt_1250.log
python tools/batch_trace.py gpurun_out/bt_full.bin
python tools/batch_trace.py gpurun_out/bt_1250.bin
