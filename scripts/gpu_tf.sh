#!/bin/bash
# Round-3 fused TransformerConv check: tests, then the layer timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_fused256.py -k "transformer" > gpurun_out/tf_tests.log 2>&1
rc=$?; tail -8 gpurun_out/tf_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/tf_bench.py > gpurun_out/tf_bench.json 2> gpurun_out/tf_bench.err
rc=$?; cat gpurun_out/tf_bench.json; tail -3 gpurun_out/tf_bench.err; exit $rc
