set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02q_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r02q_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r02q_bench.json 2> gpurun_out/r02q_bench.log || { echo bench failed; exit 1; }
timeout -k 10 700 bash tools/profile_bench.sh gpurun_out/prof_r02b > gpurun_out/r02q_prof.log 2>&1
echo done $?
