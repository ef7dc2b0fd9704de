#!/bin/bash
# round 6: GAT fused-layer A/B (AB_LIBS variants vs the in-tree library), 1M and 10M nodes, H = 128 / 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "100,100,100 128" "100,100,100 64" "250,200,200 128"; do
  set -- $cfg
  AB_MODE=gat AB_GRID=$1 AB_H=$2 AB_REPS=${AB_REPS:-7} timeout -k 10 300 python -u scripts/ab_lib.py \
      2>> gpurun_out/r6_gat.err | tee -a gpurun_out/r6_gat.jsonl || { tail -20 gpurun_out/r6_gat.err; exit 1; }
done
