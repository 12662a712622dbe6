#!/bin/bash
# Heap replay A/B at full occupancy: loads issued together at each pop (default), vs the previous
# build (rp_prev_la4), lookahead 4, 10 LDS levels; then the full C4-int table at 4096 / 5000 slots.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02u_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02u_tests.log; exit 1; }
tail -1 gpurun_out/r02u_tests.log
for v in default rp_prev_la4 rp_pf_la4 rp_pf_lds10; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 4096 4096 all || { echo probe failed; exit 1; }
done
export SHDTOPO_LIB=abtest/rp_lines/libshdtopo.so
timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
