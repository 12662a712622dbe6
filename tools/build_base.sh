#!/bin/bash
# Build the committed HEAD (or REV) library as abtest/base/libshdtopo.so: the "base" side of a
# same-box A/B against the working tree (tools/ab_probe.sh, tools/ab_replay.sh).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" shadow_amd/csrc include | tar -x -C "$TMP"
OUT=$ROOT/abtest/base
mkdir -p "$OUT/obj"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result"
cd "$TMP/shadow_amd/csrc"
for f in topo_core.cpp topo_graph.cpp topo_window.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $f -o "$OUT/obj/${f%.cpp}.o" &
done
for f in topo_kernels.hip topo_sssp_batch.hip topo_replay.hip topo_prep.hip; do
  /opt/rocm/bin/hipcc $FLAGS -c $f -o "$OUT/obj/${f%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libshdtopo.so" "$OUT"/obj/*.o -lpthread
rm -rf "$OUT/obj" "$TMP"
echo "$OUT/libshdtopo.so ($REV)"
