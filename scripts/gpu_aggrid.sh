#!/bin/bash
# aggregation grid-size sweep in the locality order (MIGNN_AGG_GRID caps the block count)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 AGG_LOCAL=1
for g in ${GRIDS:-2048 1024 512 256}; do
  MIGNN_AGG_GRID=$g timeout -k 10 200 python -u scripts/agg_bench.py > gpurun_out/aggrid_$g.json 2> gpurun_out/aggrid_$g.err
  rc=$?; echo "grid $g: $(cat gpurun_out/aggrid_$g.json)"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/aggrid_$g.err; exit $rc; fi
done
