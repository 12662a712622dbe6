#!/bin/bash
# SQ instruction-mix / stall counters of one probe command (two passes; run from the repo root).
#   tools/pmc_sq.sh OUTDIR probe-args...     (PROBE=tools/replay_probe.py for the heap replay)
set -u
PROBE=${PROBE:-tools/gpu_probe.py}
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU \
  --output-format csv -d "$ROOT/$OUT/sq1" -o sq1 -- python3 -u "$ROOT/$PROBE" "$@" > "$ROOT/$OUT/sq1.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$ROOT/$OUT/sq2" -o sq2 -- python3 -u "$ROOT/$PROBE" "$@" > "$ROOT/$OUT/sq2.log" 2>&1
