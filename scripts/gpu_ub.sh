#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_ub3,gcn16_dec KB_CHECK=1 KB_CHECK_FLAGS=8388608 timeout -k 10 200 python -u scripts/kbench.py > gpurun_out/kb_ub.json 2> gpurun_out/kb_ub.err
rc=$?; cat gpurun_out/kb_ub.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_ub.err; fi; exit $rc
