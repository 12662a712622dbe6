# shard kernel times of the 8/4/2/1-GPU splits (the first shard of each, one GPU), 6 builds each
set -e
mkdir -p gpurun_out
for R in 10000 5000 2500 1250; do
  timeout -k 10 200 python -u tools/gpu_probe.py --rows $R --reps 6 > gpurun_out/shard_$R.log 2>&1
done
