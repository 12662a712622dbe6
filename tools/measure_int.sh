#!/bin/bash
# The C4-int line on the GPU box (run from the repo root): rocprofv3 passes of the integer-latency
# bench (heap replay), their summary + PMC JSON under profiles/<TAG>int_*, then the bench line.
#   tools/measure_int.sh TAG
set -u
TAG=$1
OUT=gpurun_out/meas_${TAG}int
mkdir -p "$OUT"
tools/profile_bench.sh "$OUT/prof_int" --integer || exit $?
python3 tools/summarize_prof.py "$OUT/prof_int" "${TAG}int" > "$OUT/summary_int.log" 2>&1 || exit $?
cp profiles/${TAG}int_* "$OUT/" || exit $?
timeout -k 10 900 python3 -u bench.py --integer --pmc-tag "${TAG}int" --no-complete --getter-queries 0 \
    > "$OUT/bench_int.json" 2> "$OUT/bench_int.log" || exit $?
echo "measure_int $TAG done"
