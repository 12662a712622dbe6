#!/bin/bash
# Round-2 (f) evidence for the current code: every GPU test, the rocprofv3 passes of the bench,
# the bench line with the new PMC numbers, then the C4-int bench.  Summaries are copied to
# gpurun_out/r02f_profiles.
set -u
T=${1:-r02f}
mkdir -p gpurun_out/${T}_profiles
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 900 bash tools/profile_bench.sh gpurun_out/prof_${T} > gpurun_out/${T}_prof.log 2>&1 || { echo profile failed; cat gpurun_out/${T}_prof.log; exit 1; }
python tools/summarize_prof.py gpurun_out/prof_${T} ${T} && cp profiles/${T}_* gpurun_out/${T}_profiles/ && cp gpurun_out/prof_${T}/trace/trace_kernel_stats.csv gpurun_out/${T}_profiles/${T}_kernel_stats.csv
timeout -k 10 600 python -u bench.py --pmc-json profiles/${T}_sssp_pmc.json --route-pmc-json profiles/${T}_route_pmc.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo bench failed; tail -20 gpurun_out/${T}_bench.log; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 600 python -u bench.py --integer --steps 1 --warmup 1 --no-cpu-baseline --no-complete --no-graphml > gpurun_out/${T}_bench_int.json 2> gpurun_out/${T}_bench_int.log || { echo int bench failed; tail -20 gpurun_out/${T}_bench_int.log; exit 1; }
echo done
