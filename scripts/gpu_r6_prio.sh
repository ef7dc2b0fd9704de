#!/bin/bash
# round 6: asymmetric wave priority in the GIN layer, the H = 256 head and the H = 128 head (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB_MODE=gin AB_REPS=5 AB_LIBS=aprio=variants/libmignn_aprioagg.so timeout -k 10 400 python -u scripts/ab_lib.py \
    2>> gpurun_out/r6_prio.err | tee -a gpurun_out/r6_prio.jsonl || { tail -20 gpurun_out/r6_prio.err; exit 1; }
HA_H=256 HA_N=12600000 HA_LIBS=aprio=variants/libmignn_aprioagg.so timeout -k 10 300 python -u scripts/head_ab.py \
    2>> gpurun_out/r6_prio.err | tee -a gpurun_out/r6_prio.jsonl || { tail -20 gpurun_out/r6_prio.err; exit 1; }
HA_H=128 HA_LIBS=aprio=variants/libmignn_apriohead.so timeout -k 10 300 python -u scripts/head_ab.py \
    2>> gpurun_out/r6_prio.err | tee -a gpurun_out/r6_prio.jsonl || { tail -20 gpurun_out/r6_prio.err; exit 1; }
