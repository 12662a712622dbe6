#!/bin/bash
# The C4-int line (every row through the heap replay) on the current code: rocprofv3 trace + PMC
# passes, their summary (profiles/<TAG>int_*), then the bench line (run from the repo root on the
# GPU box).   tools/measure_int.sh TAG
set -u
TAG=$1
OUT=gpurun_out/meas_${TAG}int
mkdir -p "$OUT"
tools/profile_bench.sh "$OUT/prof_int" --integer || exit $?
python3 tools/summarize_prof.py "$OUT/prof_int" "${TAG}int" > "$OUT/summary_int.log" 2>&1 || exit $?
cp profiles/${TAG}int_* "$OUT/" || exit $?
timeout -k 10 700 python3 -u bench.py --integer --pmc-tag "${TAG}int" --no-complete \
    > "$OUT/bench_int.json" 2> "$OUT/bench_int.log" || exit $?
echo "measure_int $TAG done"
