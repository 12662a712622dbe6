#!/bin/bash
# Round-2 (e) evidence: every GPU test, the rocprofv3 passes of the bench, the bench line with
# the new PMC numbers, then the C4-int bench.  Summaries are copied to gpurun_out/r02e_profiles.
set -u
mkdir -p gpurun_out/r02e_profiles
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02e_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02e_gpu_tests.log
timeout -k 10 900 bash tools/profile_bench.sh gpurun_out/prof_r02e > gpurun_out/r02e_prof.log 2>&1 || { echo profile failed; cat gpurun_out/r02e_prof.log; exit 1; }
python tools/summarize_prof.py gpurun_out/prof_r02e r02e && cp profiles/r02e_* gpurun_out/r02e_profiles/ && cp gpurun_out/prof_r02e/trace/trace_kernel_stats.csv gpurun_out/r02e_profiles/r02e_kernel_stats.csv
timeout -k 10 600 python -u bench.py --pmc-json profiles/r02e_sssp_pmc.json --route-pmc-json profiles/r02e_route_pmc.json > gpurun_out/r02e_bench.json 2> gpurun_out/r02e_bench.log || { echo bench failed; tail -20 gpurun_out/r02e_bench.log; exit 1; }
cat gpurun_out/r02e_bench.json
timeout -k 10 600 python -u bench.py --integer --steps 1 --warmup 1 --no-cpu-baseline --no-complete --no-graphml > gpurun_out/r02e_bench_int.json 2> gpurun_out/r02e_bench_int.log || { echo int bench failed; tail -20 gpurun_out/r02e_bench_int.log; exit 1; }
echo done
