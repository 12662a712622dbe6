#!/bin/bash
# Heap replay: next root row bounds prefetched after the sink (default) vs not (rp_head).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ac_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02ac_tests.log; exit 1; }
tail -1 gpurun_out/r02ac_tests.log
for v in default rp_head default rp_head; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 5120 all || { echo probe failed; exit 1; }
done
export SHDTOPO_LIB=abtest/rp_time/libshdtopo.so
timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
