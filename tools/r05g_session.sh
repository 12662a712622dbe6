set -u
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py -x -q --timeout 200 --timeout-method thread > $O/mgpu.log 2>&1; tail -2 $O/mgpu.log
for cfg in "1250 1" "1250 0" "10000 1" "10000 0"; do
  set -- $cfg
  SHD_BATCH_TRACE=$O/trace_$1_$2.bin timeout -k 10 200 python3 -u tools/gpu_probe.py --rows $1 --reps 1 --opt share=$2 > $O/probe_$1_$2.log 2>&1 || exit 1
  python3 tools/batch_trace.py $O/trace_$1_$2.bin > $O/trace_$1_$2.txt 2>&1
  rm -f $O/trace_$1_$2.bin
done
timeout -k 10 500 python -u bench.py --opt devices=8 --no-cpu-baseline --steps 2 --route-steps 5 > $O/bench_dev8.json 2> $O/bench_dev8.log
