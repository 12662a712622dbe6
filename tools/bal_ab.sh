# A/B of the measured layout's cost model (abtest/ variants: fixed part, EMA weight), 1,250 rows
set -e
mkdir -p gpurun_out
for V in base a2 a6 e1 e25 base a2 a6 e1 e25; do
  SHDTOPO_LIB=abtest/$V/libshdtopo.so timeout -k 10 200 python -u tools/gpu_probe.py --rows 1250 --reps 8 > gpurun_out/balab_$V.log 2>&1
  grep -E "^rep" gpurun_out/balab_$V.log | awk -v v=$V '{printf "%s ", $7} END {print v}'
done
