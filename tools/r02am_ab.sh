#!/bin/bash
# Batch SSSP with pair rounds: RB / UA combinations around RB 2 (best of r02al).
set -u
mkdir -p gpurun_out/r02am
bash tools/ab_probe.sh gpurun_out/r02am "rb2|rb2|--rows 10000 --reps 2" "rb2ua1|rb2ua1|--rows 10000 --reps 2" "rb1|rb1|--rows 10000 --reps 2" "rb3|rb3|--rows 10000 --reps 2" "rb1ua1|rb1ua1|--rows 10000 --reps 2" "rb2|rb2|--rows 10000 --reps 2" "rb2ua1|rb2ua1|--rows 10000 --reps 2" "base|-|--rows 10000 --reps 2" "rb2_1250|rb2|--rows 1250 --reps 2" "rb2ua1_1250|rb2ua1|--rows 1250 --reps 2" > /dev/null || exit 1
grep -E "^==|^rep 1" gpurun_out/r02am/ab.log
