# final round-5 session: GPU tests, smoke, measurement (PMC + bench + C4-int), shard probe
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/tests
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/fo_gputests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fo_smoke.log 2>&1
tools/measure_round.sh r05o int
bash tools/shard_probe.sh
