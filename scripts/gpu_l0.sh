#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_l0.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_l0.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_l0.log | head; exit $rc; fi
KB_PERM=4,4 KB_ONLY=layer0,layer0_onerole,layer0_no_gather,head16 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_l0.json 2> gpurun_out/kb_l0.err
rc=$?; cat gpurun_out/kb_l0.json; exit $rc
