#!/bin/bash
# GAT leg (1M nodes: below the auto-reorder threshold) with and without the locality order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in auto 1 auto 1; do
  MIGNN_REORDER=$r timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-bfs --no-train --no-graph --layers 1 --grid 40,40,40 --legs gat > gpurun_out/gatord_$r.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then tail -3 gpurun_out/gatord_$r.log; exit $rc; fi
  echo "reorder=$r $(grep -o '"gat": {[^}]*' gpurun_out/gatord_$r.log | grep -o '"ms_per_forward": [0-9.]*')"
done
