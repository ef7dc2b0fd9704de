#!/bin/bash
# round 6: window / ring / pk_fma tests + smoke, then the window A/B (WB_LIBS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win.py tests/test_gpu_ring.py tests/test_gpu_pkfma.py tests/test_gpu_dist_mp.py \
    > gpurun_out/r6_d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6_d_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash scripts/gpu_r6_ab.sh
