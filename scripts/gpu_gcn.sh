#!/bin/bash
# GCN kernels: window + ring GPU tests, then the window timing study
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win.py tests/test_gpu_ring.py \
    > gpurun_out/gcn_tests.log 2>&1 || { tail -40 gpurun_out/gcn_tests.log; exit 1; }
tail -3 gpurun_out/gcn_tests.log
WB_H=${WB_H:-64,128} WB_MODES=${WB_MODES:-4,32} timeout -k 10 400 python -u scripts/win_bench.py \
    > gpurun_out/win_bench.json 2> gpurun_out/win_bench.err || { tail -20 gpurun_out/win_bench.err; exit 1; }
cat gpurun_out/win_bench.json
