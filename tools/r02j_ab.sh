set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_replay.py -x -q --timeout 200 --timeout-method thread -k "synthetic or full_size or landmark or widths or integer" > gpurun_out/r02j_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_probe.sh gpurun_out/ab_ord "hubord|-|--rows 10000 --reps 2" "roword|-|--rows 10000 --reps 2 --opt source_order=0" "hubord2|-|--rows 10000 --reps 2" "roword2|-|--rows 10000 --reps 2 --opt source_order=0"
