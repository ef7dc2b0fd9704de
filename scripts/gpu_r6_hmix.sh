#!/bin/bash
# round 6: the output head's split through mixed-precision FMAs (hmix1), + the
# float abs-max of x and opaque per-layer LDS bases (hmixlb), + ldexp seeds
# (hmixe) vs the product, same box, H = 128 and 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for h in 128 64; do
  HA_H=$h HA_LIBS=hmix1=variants/libmignn_hmix1.so,hmixlb=variants/libmignn_hmixlb.so,hmixe=variants/libmignn_hmixe.so \
    timeout -k 10 300 python -u scripts/head_ab.py 2>> gpurun_out/r6_hmix.err | tee -a gpurun_out/r6_hmix.jsonl \
    || { tail -20 gpurun_out/r6_hmix.err; exit 1; }
done
