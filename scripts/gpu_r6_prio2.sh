#!/bin/bash
# round 6: asymmetric wave priority in tf_fused_kernel (aprio2) and gemm_f16x3_kernel (apriog), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB_MODE=tf AB_GRID=250,200,200 AB_REPS=5 AB_LIBS=aprio2=variants/libmignn_aprio2.so,apriog=variants/libmignn_apriog.so \
    timeout -k 10 500 python -u scripts/ab_lib.py 2>> gpurun_out/r6_prio2.err | tee -a gpurun_out/r6_prio2.jsonl \
    || { tail -20 gpurun_out/r6_prio2.err; exit 1; }
AB_MODE=gemm AB_GRID=250,200,200 AB_REPS=5 AB_LIBS=apriog=variants/libmignn_apriog.so \
    timeout -k 10 300 python -u scripts/ab_lib.py 2>> gpurun_out/r6_prio2.err | tee -a gpurun_out/r6_prio2.jsonl \
    || { tail -20 gpurun_out/r6_prio2.err; exit 1; }
