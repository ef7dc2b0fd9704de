#!/bin/bash
# Locality-order x tile-schedule experiment for the f16x3 GCN layer kernel
# (kbench cases gcn16_full / gcn16_chunks on one tile-aligned 10M-node grid).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KB_GRID=${KB_GRID:-256,192,200} KB_ONLY=${KB_ONLY:-gcn16_full,gcn16_chunks,copy}
run() {
  name=$1; shift
  env "$@" timeout -k 10 240 python -u scripts/kbench.py > gpurun_out/exp/$name.json 2> gpurun_out/exp/$name.err
  rc=$?; echo "$name rc=$rc $(cat gpurun_out/exp/$name.json)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/exp/$name.err; exit $rc; fi
}
run pencil44 KB_PERM=4,4
run panel84 KB_PANEL=8,4
run panel48 KB_PANEL=4,8
run panel44 KB_PANEL=4,4
run panel88 KB_PANEL=8,8
