#!/bin/bash
# aggregation timing with alternative library builds (AGG_LIB), natural order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 AGG_REPS=20
for lib in gnn-bfs-rans_amd/mignn/libmignn.so ${VARIANTS}; do
  AGG_LIB=$lib timeout -k 10 200 python -u scripts/agg_bench.py > gpurun_out/aggvar.json 2> gpurun_out/aggvar.err
  rc=$?; echo "$lib: $(cat gpurun_out/aggvar.json)"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/aggvar.err; exit $rc; fi
done
