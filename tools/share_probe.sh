set -e
mkdir -p gpurun_out
for O in share=0 share=-1 share=0 share=-1; do
  timeout -k 10 200 python -u tools/gpu_probe.py --rows 1250 --reps 6 --opt $O > gpurun_out/sh_$O.log 2>&1
  grep -E "^rep" gpurun_out/sh_$O.log | awk -v o=$O '{printf "%s ", $7} END {print o}'
done
