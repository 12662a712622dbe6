#!/bin/bash
# Build an A/B variant of libshdtopo.so with extra compile-time defines (kernel experiments).
#   tools/build_variant.sh NAME -DSHD_BATCH_RB=3 ...   ->  abtest/NAME/libshdtopo.so
# Load it with SHDTOPO_LIB=abtest/NAME/libshdtopo.so (shadow_amd/_lib.py); time it on the GPU box
# with tools/ab_probe.sh.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
shift
OUT=$ROOT/abtest/$NAME
mkdir -p "$OUT/obj"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result $*"
cd "$ROOT/shadow_amd/csrc"
for f in topo_core.cpp topo_graph.cpp topo_window.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $f -o "$OUT/obj/${f%.cpp}.o" &
done
for f in topo_kernels.hip topo_sssp_batch.hip topo_replay.hip topo_prep.hip; do
  /opt/rocm/bin/hipcc $FLAGS -c $f -o "$OUT/obj/${f%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libshdtopo.so" "$OUT"/obj/*.o -lpthread
echo "$OUT/libshdtopo.so"
