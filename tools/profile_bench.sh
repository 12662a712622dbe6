#!/bin/bash
# rocprofv3 evidence for the bench configuration (run on the GPU box from the repo root):
#   one kernel-trace + stats pass, then one PMC pass per counter group (rocprofv3 does not split
#   counters over passes), each its own process under a hard time limit.  Output under $1
#   (e.g. gpurun_out/prof_r03); summarise with `python tools/summarize_prof.py $1 <tag>`.
#   Extra arguments go to bench.py (e.g. --integer for the heap-replay line).
set -u
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
# (--no-directed: the C4-dir line's kernels would add their dispatches to the same kernel names)
BENCH_ARGS=(--steps 1 --warmup 0 --no-cpu-baseline --no-graphml --no-complete --no-directed --route-steps 3 --getter-queries 0 "$@")
LIMIT=${PROF_LIMIT:-240}
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL "$LIMIT" rocprofv3 "$@" --output-format csv -d "$ROOT/$OUT/$name" -o "$name" -- \
      python3 -u "$ROOT/bench.py" "${BENCH_ARGS[@]}" > "$ROOT/$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass trace --kernel-trace --stats &&
pass fetch --pmc FETCH_SIZE &&
pass write --pmc WRITE_SIZE &&
pass req --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum &&
pass sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE
