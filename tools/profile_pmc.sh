#!/bin/bash
# Counter passes over one command (each pass its own process, as rocprofv3 does not split
# counters over passes).  Usage: tools/profile_pmc.sh <outdir> <python args...>
# Run from the repo root on the GPU box.
set -u
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --output-format csv -d "$ROOT/$OUT/$name" -o "$name" -- \
      python3 -u "$ROOT/$PYSCRIPT" "${ARGS[@]}" > "$ROOT/$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
PYSCRIPT=$1; shift
ARGS=("$@")
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run req --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum &&
run hit --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum &&
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES
