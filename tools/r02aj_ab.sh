#!/bin/bash
# Heap replay: relaxation records read during the sink (SHD_RP_EARLY) vs not; 5120 C4-int rows.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02aj_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02aj_tests.log; exit 1; }
tail -1 gpurun_out/r02aj_tests.log
for v in default rp_noearly default rp_noearly; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 0 all || { echo probe failed; exit 1; }
done
