#!/bin/bash
# Ablations of the f16x3 GCN layer kernel (kbench diagnostic flags) on one
# locality order / schedule: KB_PANEL / KB_PERM and KB_XFLAGS from the caller.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KB_GRID=${KB_GRID:-256,192,200}
export KB_ONLY=${KB_ONLY:-gcn16,diag_copy}
name=${EXP_NAME:-ablate}
timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/exp/$name.json 2> gpurun_out/exp/$name.err
rc=$?; echo "$name rc=$rc $(cat gpurun_out/exp/$name.json)"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/exp/$name.err; fi
exit $rc
