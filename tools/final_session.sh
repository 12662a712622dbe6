# final round-5 session: GPU tests, measurement (PMC + bench + C4-int), shard probe, 8-engine rehearsal
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/tests
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/fin_gputests.log 2>&1
tools/measure_round.sh r05n int
bash tools/shard_probe.sh
timeout -k 10 400 python -u bench.py --no-directed --opt devices=8 > gpurun_out/fin_dev8.json 2> gpurun_out/fin_dev8.err
