#!/bin/bash
# round 6: split_pair (mixed-precision FMA split) in agg_gemm.hip's kernels --
# GIN H256 layer, H = 256 head, GAT fused layers, TF fused layer -- vs the
# in-tree library, same box, outputs compared
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=variants/libmignn_amix.so
AB_LIBS=amix=$V AB_MODE=gin AB_REPS=5 timeout -k 10 400 python -u scripts/ab_lib.py 2>> gpurun_out/r6_amix.err \
    | tee -a gpurun_out/r6_amix.jsonl || { tail -20 gpurun_out/r6_amix.err; exit 1; }
HA_LIBS=amix=$V HA_H=256 HA_N=12600000 timeout -k 10 300 python -u scripts/head_ab.py 2>> gpurun_out/r6_amix.err \
    | tee -a gpurun_out/r6_amix.jsonl || { tail -20 gpurun_out/r6_amix.err; exit 1; }
for cfg in "100,100,100 128" "100,100,100 64"; do
  set -- $cfg
  AB_LIBS=amix=$V AB_MODE=gat AB_GRID=$1 AB_H=$2 AB_REPS=7 timeout -k 10 300 python -u scripts/ab_lib.py \
      2>> gpurun_out/r6_amix.err | tee -a gpurun_out/r6_amix.jsonl || { tail -20 gpurun_out/r6_amix.err; exit 1; }
done
AB_LIBS=amix=$V AB_MODE=tf AB_REPS=3 timeout -k 10 400 python -u scripts/ab_lib.py 2>> gpurun_out/r6_amix.err \
    | tee -a gpurun_out/r6_amix.jsonl || { tail -20 gpurun_out/r6_amix.err; exit 1; }
