#!/bin/bash
# One measurement session on the GPU box (run from the repo root): rocprofv3 evidence for the C4
# bench configuration (tools/profile_bench.sh), its summary + the per-launch PMC JSONs the bench
# reads for its roofline (tools/summarize_prof.py, written to profiles/ and copied to the output
# directory, which gpurun brings back), then the bench line itself.
#   tools/measure_round.sh TAG [int]     (int: the C4-int line -- heap replay -- as well)
set -u
TAG=$1
OUT=gpurun_out/meas_$TAG
mkdir -p "$OUT"
tools/profile_bench.sh "$OUT/prof" || exit $?
python3 tools/summarize_prof.py "$OUT/prof" "$TAG" > "$OUT/summary.log" 2>&1 || exit $?
cp profiles/${TAG}_* "$OUT/" || exit $?
timeout -k 10 600 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
if [ "${2:-}" = "int" ]; then
  tools/profile_bench.sh "$OUT/prof_int" --integer || exit $?
  python3 tools/summarize_prof.py "$OUT/prof_int" "${TAG}int" > "$OUT/summary_int.log" 2>&1 || exit $?
  cp profiles/${TAG}int_* "$OUT/" || exit $?
  timeout -k 10 900 python3 -u bench.py --integer --pmc-tag "${TAG}int" --no-complete \
      > "$OUT/bench_int.json" 2> "$OUT/bench_int.log" || exit $?
fi
echo "measure_round $TAG done"
