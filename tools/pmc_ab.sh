#!/bin/bash
# Request-count comparison of kernel variants (run on the GPU box from the repo root):
#   tools/pmc_ab.sh OUTDIR "name|lib|probe args" ...
# One rocprofv3 pass per variant with the DRAM request counters; PMC="..." picks other counters
# (one block's limits per pass, e.g. PMC=WRITE_SIZE), TAG a suffix for the output names and
# PROBE the probe script.
set -u
PMC=${PMC:-"TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum"}
TAG=${TAG:-}
PROBE=${PROBE:-tools/gpu_probe.py}  # e.g. PROBE=tools/replay_probe.py "name|lib|1024 0 all"
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name lib args <<< "$spec"
  if [ "$lib" = "-" ]; then L=""; else L="$ROOT/abtest/$lib/libshdtopo.so"; fi
  export SHDTOPO_LIB="$L"
  timeout -s KILL 150 rocprofv3 --pmc $PMC \
      --output-format csv -d "$ROOT/$OUT/$name$TAG" -o "$name$TAG" -- \
      python3 -u "$ROOT/$PROBE" $args > "$ROOT/$OUT/$name$TAG.log" 2>&1 || exit $?
  echo "pmc $name$TAG ok"
done
