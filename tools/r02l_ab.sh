set -u
mkdir -p gpurun_out
O="--rows 10000 --reps 2 --opt source_order=2"
bash tools/ab_probe.sh gpurun_out/ab_bo "b0|-|$O" "b1|-|$O --opt batch_order=1" "b2|-|$O --opt batch_order=2" "b3|-|$O --opt batch_order=3" "b0r|-|$O" "b1r|-|$O --opt batch_order=1" "b2r|-|$O --opt batch_order=2" "b3r|-|$O --opt batch_order=3"
