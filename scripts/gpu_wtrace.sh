#!/bin/bash
# window kernel timelines (diag build): WT_H in WT_HS, modes in WT_MODES
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for h in ${WT_HS:-64}; do
  for m in ${WT_MODES:-0 32}; do
    WT_H=$h WT_MODE=$m timeout -k 10 200 python -u scripts/win_trace.py >> gpurun_out/wtrace.json 2> gpurun_out/wtrace.err \
        || { tail -20 gpurun_out/wtrace.err; exit 1; }
  done
done
cat gpurun_out/wtrace.json
