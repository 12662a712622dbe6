#!/bin/bash
# Re-tune after the target-aware steps: bucket width (delta, ms) and LDS hubs, full C4 table.
set -u
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python -u tools/gpu_probe.py --rows 10000 --reps 2 "$@" > gpurun_out/r02x.log 2>&1 || { echo probe failed; tail -20 gpurun_out/r02x.log; exit 1; }
  echo "$*"; grep -h "^rep 1" gpurun_out/r02x.log
}
run
run --delta 6
run --delta 15
run --delta 25
run --opt lds_hubs=1024
run --opt lds_hubs=512
run
