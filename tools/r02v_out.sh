#!/bin/bash
# Nontemporal table stores: every GPU parity test, then an interleaved A/B against the
# previous walk loop (abtest/noout: -DSHD_OUT_NT=0) on the full C4 table.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v_gpu_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r02v_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02v_gpu_tests.log
bash tools/ab_probe.sh gpurun_out/ab_r02v "fast|-|--rows 10000 --reps 2" "old|noout|--rows 10000 --reps 2" "fast|-|--rows 10000 --reps 2" "old|noout|--rows 10000 --reps 2"
grep -E "^==|^rep 1|per-source ms" gpurun_out/ab_r02v/ab.log
