#!/bin/bash
# Heap replay: HBM-level sink lookahead 5 (default) / 4 / 3 / 2 at 20 wavefronts per CU, then
# the line counts of 4 and 3.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02y_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02y_tests.log; exit 1; }
for v in default rp_h4 rp_h3 rp_h2 default; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 5120 all || { echo probe failed; exit 1; }
done
for v in rp_h4_lines rp_h3_lines; do
  export SHDTOPO_LIB=abtest/$v/libshdtopo.so
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
done
