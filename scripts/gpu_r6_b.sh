#!/bin/bash
# round 6: window / ring / parity tests after the pipelined H = 128 step,
# then the window timing (H = 128 and 64) and the H = 128 timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_win.py tests/test_gpu_ring.py tests/test_gpu_pkfma.py \
    > gpurun_out/r6_b_tests.log 2>&1; rc=$?; tail -6 gpurun_out/r6_b_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
WB_OLD=0 WB_H=128,64 WB_REPS=5 WB_MODES=4,32 timeout -k 10 400 python -u scripts/win_bench.py \
    > gpurun_out/r6_b_bench.json 2> gpurun_out/r6_b_bench.err || { tail -20 gpurun_out/r6_b_bench.err; exit 1; }
cat gpurun_out/r6_b_bench.json
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3
