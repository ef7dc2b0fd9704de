#!/bin/bash
# round 6 baseline: the multi-process shard test, then window kernel
# ablations at H = 64 / 128 on the bench mesh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist_mp.py \
    > gpurun_out/r6_mp.log 2>&1; rc=$?; tail -15 gpurun_out/r6_mp.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
WB_OLD=0 WB_H=64,128 WB_REPS=5 WB_MODES=1,2,3,4,32,33 timeout -k 10 500 python -u scripts/win_bench.py \
    > gpurun_out/r6_base.json 2> gpurun_out/r6_base.err || { tail -20 gpurun_out/r6_base.err; exit 1; }
cat gpurun_out/r6_base.json
