#!/bin/bash
# round 6: MFMA order experiments -- the window kernel's groups product-major
# (wmj, WB A/B) and the H = 128 head k-step-outer (hilv, head A/B), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
WB_H=128 WB_REPS=9 WB_LIBS=wmj=variants/libmignn_wmj.so AB_OUT=gpurun_out/r6_ab_mj.json bash scripts/gpu_r6_ab.sh || exit 1
HA_H=128 HA_LIBS=hilv=variants/libmignn_hilv.so timeout -k 10 300 python -u scripts/head_ab.py \
    2>> gpurun_out/r6_mj.err | tee -a gpurun_out/r6_mj.jsonl || { tail -20 gpurun_out/r6_mj.err; exit 1; }
