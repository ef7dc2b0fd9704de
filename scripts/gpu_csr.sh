#!/bin/bash
# GPU tests, then the headline bench (no legs) under rocprofv3 --stats: CSR build kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_csr.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_csr.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_csr.log | head; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof -o b --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-bfs --no-train --no-graph --no-legs > gpurun_out/cprof.log 2>&1
rc=$?; tail -1 gpurun_out/cprof.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'cached',d['ms_per_step_graph_cached'])"
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/cprof/b_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('csr_', 'rows_gather', 'order_', 'bbox', 'spacing', 'inverse', 'trampoline')):
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 3))
PY
exit $rc
