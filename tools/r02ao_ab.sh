#!/bin/bash
# Batch SSSP: tail sub-chunk loads (mask, row bounds, kappa probes, distances) in one round trip.
set -u
mkdir -p gpurun_out/r02ao
bash tools/ab_probe.sh gpurun_out/r02ao "new|-|--rows 10000 --reps 2" "prev|prev|--rows 10000 --reps 2" "new|-|--rows 10000 --reps 2" "prev|prev|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1" gpurun_out/r02ao/ab.log
