#!/bin/bash
# A/B timing of kernel variants on the C4 graph (run on the GPU box from the repo root).
#   tools/ab_probe.sh OUTDIR "name|lib|probe args" ...
# lib "-" = the in-tree shadow_amd/libshdtopo.so, else abtest/<lib>/libshdtopo.so.
# Stops at the first failing probe (a fault or time limit ends the call).
set -u
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  IFS='|' read -r name lib args <<< "$spec"
  if [ "$lib" = "-" ]; then L=""; else L="$(pwd)/abtest/$lib/libshdtopo.so"; fi
  echo "== $name ($lib) $args" | tee -a "$OUT/ab.log"
  SHDTOPO_LIB="$L" timeout -k 10 150 python3 -u tools/gpu_probe.py $args >> "$OUT/ab.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "probe $name failed rc=$rc" | tee -a "$OUT/ab.log"; exit $rc; fi
  grep -E "^rep|per-source|split ms" "$OUT/ab.log" | tail -3
done
