# round-5 measured batch layout: full GPU suite, then the 1-GPU bench and the 8-engine rehearsal
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/tests
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/bal5_gputests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bal5_bench.json 2> gpurun_out/bal5_bench.err
timeout -k 10 400 python -u bench.py --no-directed --opt devices=8 > gpurun_out/bal5_dev8.json 2> gpurun_out/bal5_dev8.err
