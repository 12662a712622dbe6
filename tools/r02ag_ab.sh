#!/bin/bash
# Heap replay: keys-only LDS levels 10 (default) / 9 / 11 vs HEAD (keys + vertices, 9 levels).
set -u
mkdir -p gpurun_out
for v in default rp_k11; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ag_tests_$v.log 2>&1 || { echo tests failed $v; tail -30 gpurun_out/r02ag_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r02ag_tests_$v.log
done
for v in default rp_head rp_k9 rp_k11 default rp_head; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 0 all || { echo probe failed; exit 1; }
done
export SHDTOPO_LIB=abtest/rp_time/libshdtopo.so
timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
