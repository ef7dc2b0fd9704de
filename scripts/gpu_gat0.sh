#!/bin/bash
# Round-3 GAT layer-0 composition check: tests, then the GAT leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fused256.py tests/test_gpu_large.py tests/test_gpu_parity.py tests/test_gpu_dist.py \
    -k "gat or GAT" > gpurun_out/gat0_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gat0_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-bfs --no-train --no-graph \
    --legs gat > gpurun_out/bench_gat.json 2> gpurun_out/bench_gat.err
rc=$?; grep "leg gat" gpurun_out/bench_gat.err; exit $rc
