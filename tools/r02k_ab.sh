set -u
mkdir -p gpurun_out
bash tools/ab_probe.sh gpurun_out/ab_ord2 "hub|-|--rows 10000 --reps 2" "dfs|-|--rows 10000 --reps 2 --opt source_order=2" "hub2|-|--rows 10000 --reps 2" "dfs2|-|--rows 10000 --reps 2 --opt source_order=2"
