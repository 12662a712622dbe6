#!/bin/bash
# Heap replay A/B: replay tests with the new layout, then 256 C4-int rows per variant.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02r_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02r_tests.log; exit 1; }
for v in rp_old default rp_la4 rp_la3; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 240 python -u tools/replay_probe.py 256 || { echo probe failed; exit 1; }
done
unset SHDTOPO_LIB
timeout -k 10 300 python -u tools/scale_probe.py || { echo scale probe failed; exit 1; }
