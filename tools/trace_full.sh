# batch trace of the full table with the measured layout, then smoke()
set -e
mkdir -p gpurun_out
rm -f gpurun_out/tf_trace.bin
SHD_BATCH_TRACE=gpurun_out/tf_trace.bin timeout -k 10 200 python -u tools/gpu_probe.py --rows 10000 --reps 4 > gpurun_out/tf.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/tf_smoke.log 2>&1
