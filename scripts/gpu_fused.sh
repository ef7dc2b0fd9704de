#!/bin/bash
# fused H = 256 layers: GPU tests, then timing (scripts/fused_bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused256.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -15 gpurun_out/fused_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/fused_bench.py > gpurun_out/fused_gin.json 2> gpurun_out/fused_gin.err
rc=$?; cat gpurun_out/fused_gin.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/fused_gin.err; exit $rc; fi
FB_MODE=gcn FB_GRID=250,200,200 timeout -k 10 300 python -u scripts/fused_bench.py > gpurun_out/fused_gcn.json 2> gpurun_out/fused_gcn.err
rc=$?; cat gpurun_out/fused_gcn.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/fused_gcn.err; exit $rc; fi
FB_MODE=gat FB_GRID=100,100,100 timeout -k 10 300 python -u scripts/fused_bench.py > gpurun_out/fused_gat.json 2> gpurun_out/fused_gat.err
rc=$?; cat gpurun_out/fused_gat.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/fused_gat.err; exit $rc; fi
