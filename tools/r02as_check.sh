#!/bin/bash
# Fresh-process shard builds after the slot-sizing fix (a slot per source for short shards) +
# the batch-kernel GPU tests.
set -u
mkdir -p gpurun_out/r02as
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_replay.py tests/test_multi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02as/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02as/tests.log; exit 1; }
tail -1 gpurun_out/r02as/tests.log
for r in 1250 2500 5000; do
  echo "== rows $r" >> gpurun_out/r02as/ab.log
  timeout -k 10 150 python3 -u tools/gpu_probe.py --rows $r --reps 2 >> gpurun_out/r02as/ab.log 2>&1 || { echo failed; exit 1; }
done
grep -E "^==|^rep 1|slots" gpurun_out/r02as/ab.log
