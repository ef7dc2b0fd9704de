#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_plain,gcn16_prio_cons,gcn16_prio_prod,head16,head16_prio KB_CHECK_HEAD=1 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb3.json 2> gpurun_out/kb3.err
rc=$?; cat gpurun_out/kb3.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb3.err; fi
exit $rc
