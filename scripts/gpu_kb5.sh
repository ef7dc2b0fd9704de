#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_staged,gcn16_plain KB_CHECK=1 KB_CHECK_FLAGS=1048576 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb5.json 2> gpurun_out/kb5.err
rc=$?; cat gpurun_out/kb5.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb5.err; exit $rc; fi
KB_H=64 KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_staged KB_CHECK=1 KB_CHECK_FLAGS=1048576 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb5_64.json 2> gpurun_out/kb5_64.err
rc=$?; cat gpurun_out/kb5_64.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb5_64.err; fi
exit $rc
