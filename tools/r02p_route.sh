set -u
mkdir -p gpurun_out
for v in 8 1 2 4 8 1 2 4; do
  if [ $v = 8 ]; then L=""; else L="$(pwd)/abtest/route$v/libshdtopo.so"; fi
  echo "U=$v" >> gpurun_out/r02p_route.log
  SHDTOPO_LIB="$L" timeout -k 10 120 python3 -u tools/route_probe.py >> gpurun_out/r02p_route.log 2>&1 || exit 1
done
