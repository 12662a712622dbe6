set -u
mkdir -p gpurun_out
bash tools/ab_probe.sh gpurun_out/ab_k2 "k8|-|--rows 10000 --reps 2" "k16|-|--rows 10000 --reps 2 --opt batch=16" "k8r|-|--rows 10000 --reps 2" "k16r|-|--rows 10000 --reps 2 --opt batch=16"
