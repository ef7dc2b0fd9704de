#!/bin/bash
# aggregation A/B: parity tests, natural-order timing, then the GIN /
# Transformer / GAT legs (locality order) under rocprofv3 --stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/agg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/agg_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/agg_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u scripts/agg_bench.py > gpurun_out/agg_bench.json 2> gpurun_out/agg_bench.err
rc=$?; cat gpurun_out/agg_bench.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/agg_bench.err; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/aprof -o legs --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-bfs --no-train --no-graph --legs ${LEGS:-gin,transformer,gat} > gpurun_out/aprof.log 2>&1
rc=$?; tail -1 gpurun_out/aprof.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print({k:v['ms_per_forward'] for k,v in d['legs'].items()})"
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/aprof/legs_kernel_stats.csv')):
    n=r['Name']
    if any(k in n for k in ('sum_rows','tf_rows','gat_rows','gemm_f16x3')): print(n[:70], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
exit $rc
