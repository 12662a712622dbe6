set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_replay.py -x -q --timeout 200 --timeout-method thread -k "synthetic or full_size or landmark or widths or integer" > gpurun_out/r02n_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_probe.sh gpurun_out/ab_hint "hint|-|--rows 10000 --reps 2" "nohint|nohint|--rows 10000 --reps 2" "hint2|-|--rows 10000 --reps 2" "nohint2|nohint|--rows 10000 --reps 2"
