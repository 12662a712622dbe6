#!/bin/bash
# Heap replay: path-first sink (default) vs round-by-round sink (rp_old_sink), timing builds.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02aa_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02aa_tests.log; exit 1; }
tail -1 gpurun_out/r02aa_tests.log
for v in default rp_old_sink default rp_old_sink; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 5120 5120 all || { echo probe failed; exit 1; }
done
for v in rp_time rp_time_old; do
  export SHDTOPO_LIB=abtest/$v/libshdtopo.so
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
done
