set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "synthetic or full_size or landmark or widths" > gpurun_out/r02i_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_probe.sh gpurun_out/ab_kap "new|-|--rows 10000 --reps 2" "old|kapold|--rows 10000 --reps 2" "new2|-|--rows 10000 --reps 2" "old2|kapold|--rows 10000 --reps 2"
