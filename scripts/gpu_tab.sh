#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_no_ext,gcn16_no_tables_ext,gcn16_no_produce timeout -k 10 200 python -u scripts/kbench.py > gpurun_out/kb_tab.json 2> gpurun_out/kb_tab.err
rc=$?; cat gpurun_out/kb_tab.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_tab.err; fi; exit $rc
