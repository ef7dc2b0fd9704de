#!/bin/bash
# round 6: A/B of the window kernels against the round-5 build on one box,
# the H = 128 timeline, window / ring tests, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win.py tests/test_gpu_ring.py \
    > gpurun_out/r6_c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6_c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
WB_OLD=0 WB_H=${WB_H:-128,64} WB_REPS=7 WB_MODES=${WB_MODES:-} WB_LIBS=${WB_LIBS:-r05=variants/libmignn_r05.so} \
    timeout -k 10 500 python -u scripts/win_bench.py > gpurun_out/r6_c_bench.json 2> gpurun_out/r6_c_bench.err \
    || { tail -20 gpurun_out/r6_c_bench.err; exit 1; }
cat gpurun_out/r6_c_bench.json
WT_H=128 WT_MODE=0 timeout -k 10 200 python -u scripts/win_trace.py 2> gpurun_out/wtrace.err | tee gpurun_out/r6_c_trace.json
