#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_ONLY=diag_copy,diag_tilecopy,copy timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_copy.json 2> gpurun_out/kb_copy.err
rc=$?; cat gpurun_out/kb_copy.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_copy.err; exit $rc; fi
KB_PERM=4,4 KB_ONLY=gcn16_full,gcn16_no_produce,gcn16_no_ext,gcn16_no_local,gcn16_chunks KB_TRACE=1 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_perm.json 2> gpurun_out/kb_perm.err
rc=$?; cat gpurun_out/kb_perm.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_perm.err; fi
exit $rc
