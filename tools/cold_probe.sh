#!/bin/bash
# Cold-build probe (GPU box, repo root): the bench's cold build and two warm steps, then a
# kernel trace of one more run for the target preparation's timeline.  Output under $1.
#   tools/cold_probe.sh gpurun_out/cold
set -u
OUT=$1
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS=(--no-cpu-baseline --no-complete --no-directed --route-steps 1 --getter-queries 0)
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 "${ARGS[@]}" > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/prof" -o cold -- \
    python3 -u "$ROOT/bench.py" --steps 1 --warmup 0 "${ARGS[@]}" > "$ROOT/$OUT/trace.log" 2>&1
