#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02t_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02t_tests.log; exit 1; }
tail -2 gpurun_out/r02t_tests.log
for v in rp_lines rp_lines_old; do
  export SHDTOPO_LIB=abtest/$v/libshdtopo.so
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 256 256 all || { echo probe failed; exit 1; }
done
