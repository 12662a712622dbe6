#!/bin/bash
# Heap replay: HBM sink rounds of 5 (default) / 6 / 4 levels; rp_head = without the root prefetch.
set -u
mkdir -p gpurun_out
for v in default rp_hl6 rp_hl4; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ad_tests_$v.log 2>&1 || { echo tests failed $v; tail -30 gpurun_out/r02ad_tests_$v.log; exit 1; }
done
for v in default rp_hl6 rp_hl4 rp_head default rp_hl6; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 5120 all || { echo probe failed; exit 1; }
done
export SHDTOPO_LIB=abtest/rp_time6/libshdtopo.so
timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
