#!/bin/bash
# window GCN kernel: parity tests, timing study, timelines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/win_tests.log 2>&1 || { tail -30 gpurun_out/win_tests.log; exit 1; }
tail -2 gpurun_out/win_tests.log
WB_MODES=${WB_MODES:-1,4,33} timeout -k 10 400 python -u scripts/win_bench.py \
    > gpurun_out/win_bench.json 2> gpurun_out/win_bench.err || { tail -20 gpurun_out/win_bench.err; exit 1; }
cat gpurun_out/win_bench.json
rm -f gpurun_out/win_trace.jsonl
for cfg in "128 0" "64 0"; do
  set -- $cfg
  WT_H=$1 WT_MODE=$2 timeout -k 10 120 python -u scripts/win_trace.py >> gpurun_out/win_trace.jsonl 2>> gpurun_out/win_trace.err || exit 1
done
cat gpurun_out/win_trace.jsonl
