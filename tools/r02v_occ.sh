#!/bin/bash
# Heap replay occupancy: wavefronts per CU vs replay throughput (C4-int, replay only).
set -u
for cfg in "4096 4096" "5120 5120" "5120 4096" "5376 5376"; do
  echo "== rows/slots $cfg"
  timeout -k 10 200 python -u tools/replay_probe.py $cfg all || { echo probe failed; exit 1; }
done
