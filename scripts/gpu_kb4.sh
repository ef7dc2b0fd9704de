#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_plain,gcn16_dma_late,gcn16_dma_late_plain KB_CHECK=1 KB_CHECK_FLAGS=524288 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb4.json 2> gpurun_out/kb4.err
rc=$?; cat gpurun_out/kb4.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb4.err; fi
exit $rc
