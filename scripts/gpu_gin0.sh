#!/bin/bash
# Round-3 GIN layer-0 composition check: tests, then the GIN leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fused256.py tests/test_gpu_large.py tests/test_gpu_dist.py -k "gin or GIN" \
    > gpurun_out/gin0_tests.log 2>&1
rc=$?; tail -14 gpurun_out/gin0_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-train --no-graph \
    --legs gin > gpurun_out/bench_gin.json 2> gpurun_out/bench_gin.err
rc=$?; grep "leg gin" gpurun_out/bench_gin.err; exit $rc
