#!/bin/bash
# round 6: GIN H256 layer A/B (agg_gemm_kernel, AB_LIBS) and the H = 256 head A/B (HA_LIBS), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB_MODE=gin AB_REPS=${AB_REPS:-5} timeout -k 10 400 python -u scripts/ab_lib.py 2>> gpurun_out/r6_gin.err \
    | tee -a gpurun_out/r6_gin.jsonl || { tail -20 gpurun_out/r6_gin.err; exit 1; }
HA_H=256 HA_N=12600000 timeout -k 10 300 python -u scripts/head_ab.py 2>> gpurun_out/r6_gin.err \
    | tee -a gpurun_out/r6_gin.jsonl || { tail -20 gpurun_out/r6_gin.err; exit 1; }
