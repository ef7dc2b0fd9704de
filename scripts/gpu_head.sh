#!/bin/bash
# Round-3 head256 check: H=256 head tests, then the head timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "mlp_head" > gpurun_out/head_tests.log 2>&1
rc=$?; tail -3 gpurun_out/head_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/head_bench.py > gpurun_out/head256.json 2> gpurun_out/head256.err
rc=$?; cat gpurun_out/head256.json; tail -3 gpurun_out/head256.err; exit $rc
