#!/bin/bash
# Round-3 fused TransformerConv check: tests, then the layer timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fused256.py tests/test_gpu_large.py -k "transformer or Transformer" \
    > gpurun_out/tf_tests.log 2>&1
rc=$?; tail -12 gpurun_out/tf_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/tf_bench.py > gpurun_out/tf_bench.json 2> gpurun_out/tf_bench.err
rc=$?; cat gpurun_out/tf_bench.json; tail -3 gpurun_out/tf_bench.err; exit $rc
