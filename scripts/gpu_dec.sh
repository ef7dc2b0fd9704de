#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_dec,gcn16_ub4 KB_CHECK=1 KB_CHECK_FLAGS=4194304 timeout -k 10 200 python -u scripts/kbench.py > gpurun_out/kb_dec.json 2> gpurun_out/kb_dec.err
rc=$?; cat gpurun_out/kb_dec.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_dec.err; exit $rc; fi
KB_H=64 KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_dec,gcn16_ub4 KB_CHECK=1 KB_CHECK_FLAGS=4194304 timeout -k 10 200 python -u scripts/kbench.py > gpurun_out/kb_dec64.json 2> gpurun_out/kb_dec64.err
rc=$?; cat gpurun_out/kb_dec64.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_dec64.err; fi; exit $rc
