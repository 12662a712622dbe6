#!/bin/bash
# Batch SSSP with pair rounds: RB (rounds in flight) and UA (phase-A edges per lane) re-tuned.
set -u
mkdir -p gpurun_out/r02al
bash tools/ab_probe.sh gpurun_out/r02al "base|-|--rows 10000 --reps 2" "rb2|rb2|--rows 10000 --reps 2" "rb8|rb8|--rows 10000 --reps 2" "ua4|ua4|--rows 10000 --reps 2" "ua1|ua1|--rows 10000 --reps 2" "base|-|--rows 10000 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep" gpurun_out/r02al/ab.log
