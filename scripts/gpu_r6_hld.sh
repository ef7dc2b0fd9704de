#!/bin/bash
# round 6: the head's W-fragment loads pinned ahead of each step's MFMAs
# (MIGNN_HEAD_LDFIRST, prefetch depth 1 / 2) vs the product, H = 128 / 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for h in 128 64; do
  HA_H=$h HA_LIBS=hld1=variants/libmignn_hld1.so,hld2=variants/libmignn_hld2.so \
    timeout -k 10 300 python -u scripts/head_ab.py 2>> gpurun_out/r6_hld.err | tee -a gpurun_out/r6_hld.jsonl \
    || { tail -20 gpurun_out/r6_hld.err; exit 1; }
done
