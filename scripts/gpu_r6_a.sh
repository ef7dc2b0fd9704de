#!/bin/bash
# round 6: window tests + pk_fma test after the prune, then window timelines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pkfma.py tests/test_gpu_win.py \
    > gpurun_out/r6_a_tests.log 2>&1; rc=$?; tail -8 gpurun_out/r6_a_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
rm -f gpurun_out/wtrace.json
for h in 64 128; do
  for m in 0 32 3; do
    WT_H=$h WT_MODE=$m timeout -k 10 200 python -u scripts/win_trace.py >> gpurun_out/wtrace.json 2> gpurun_out/wtrace.err \
        || { tail -20 gpurun_out/wtrace.err; exit 1; }
  done
done
cat gpurun_out/wtrace.json
