#!/bin/bash
# Build a variant of libmignn.so for same-box A/B timing: the product objects
# (build/obj, from `make`) with ONE source replaced.
#   scripts/build_variant.sh NAME SOURCE.hip [extra hipcc flags...]
# -> variants/libmignn_NAME.so (loaded by scripts only: win_bench WB_LIBS,
#    MIGNN_LIB_VARIANT for gpu_ab.sh)
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
base=$(basename "$src"); stem=${base%.hip}
# the replaced file keeps its product name so the object list matches
tmp=$(mktemp -d)
cp "$src" "gnn-bfs-rans_amd/csrc/.variant_$stem.hip"
trap 'rm -rf "$tmp" "gnn-bfs-rans_amd/csrc/.variant_$stem.hip"' EXIT
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude \
    -munsafe-fp-atomics "$@" -c "gnn-bfs-rans_amd/csrc/.variant_$stem.hip" -o "$tmp/$stem.o"
objs=()
for o in build/obj/*.o; do
  [ "$(basename "$o")" = "$stem.o" ] && objs+=("$tmp/$stem.o") || objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "variants/libmignn_$name.so" "${objs[@]}"
echo "variants/libmignn_$name.so"
