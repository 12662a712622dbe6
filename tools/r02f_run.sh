set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r02f_bench.json 2> gpurun_out/r02f_bench.log && \
timeout -k 10 700 bash tools/profile_bench.sh gpurun_out/prof_r02 > gpurun_out/r02f_prof.log 2>&1
echo done $?
