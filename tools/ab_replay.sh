#!/bin/bash
# A/B timing of heap-replay variants on C4-int (run on the GPU box from the repo root).
#   tools/ab_replay.sh OUTDIR ROWS "name|lib[|probe args]" ...    (lib "-" = the in-tree library;
#   probe args after "all": LANDMARK INT_KEYS, see tools/replay_probe.py)
set -u
OUT=$1; ROWS=$2; shift 2
mkdir -p "$OUT"
for spec in "$@"; do
  IFS='|' read -r name lib extra <<< "$spec"
  if [ "$lib" = "-" ]; then L=""; else L="$(pwd)/abtest/$lib/libshdtopo.so"; fi
  echo "== $name ($lib) rows $ROWS" | tee -a "$OUT/ab.log"
  SHDTOPO_LIB="$L" timeout -k 10 200 python3 -u tools/replay_probe.py "$ROWS" 0 all ${extra:-} >> "$OUT/ab.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "probe $name failed rc=$rc" | tee -a "$OUT/ab.log"; exit $rc; fi
  grep -E "^replay_all" "$OUT/ab.log" | tail -1
done
