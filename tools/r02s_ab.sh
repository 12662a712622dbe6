#!/bin/bash
# Heap replay A/B at full occupancy (4096 C4-int rows on 4096 wavefronts, replay only).
set -u
for v in default rp_old rp_np rp_la4 rp_la3 rp_np3; do
  if [ $v = default ]; then unset SHDTOPO_LIB; else export SHDTOPO_LIB=abtest/$v/libshdtopo.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/replay_probe.py 4096 4096 all || { echo probe failed; exit 1; }
done
