#!/bin/bash
# Batch SSSP phase B over compacted (edge, source) pairs (default) vs edge rounds: parity tests,
# then the full C4 table interleaved, the timing build, and the 1250-row (8-GPU shard) case.
set -u
mkdir -p gpurun_out/r02ak
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ak/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02ak/tests.log; exit 1; }
tail -1 gpurun_out/r02ak/tests.log
bash tools/ab_probe.sh gpurun_out/r02ak "pairs|-|--rows 10000 --reps 2" "edges|edges|--rows 10000 --reps 2" "pairs_bt|pairs_bt|--rows 10000 --reps 1" "pairs1250|-|--rows 1250 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep|wave ms" gpurun_out/r02ak/ab.log
