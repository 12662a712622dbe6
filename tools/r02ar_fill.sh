#!/bin/bash
# Sources per batch (batch_fill) for the N-GPU shards with pair rounds: rows 2500 / 5000 / 1250.
set -u
mkdir -p gpurun_out/r02ar
for spec in "2500 8" "2500 7" "2500 6" "2500 5" "5000 8" "5000 7" "5000 6" "1250 5" "1250 6" "1250 4"; do
  set -- $spec
  echo "== rows $1 fill $2" >> gpurun_out/r02ar/ab.log
  timeout -k 10 150 python3 -u tools/gpu_probe.py --rows $1 --reps 2 --opt batch_fill=$2 >> gpurun_out/r02ar/ab.log 2>&1 || { echo failed; exit 1; }
done
grep -E "^==|^rep 1" gpurun_out/r02ar/ab.log
