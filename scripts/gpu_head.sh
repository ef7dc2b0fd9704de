#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=head16,head16_w12 KB_CHECK_HEAD=1 KB_CHECK_HEAD_MODE=5 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_head.json 2> gpurun_out/kb_head.err
rc=$?; cat gpurun_out/kb_head.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_head.err; fi; exit $rc
