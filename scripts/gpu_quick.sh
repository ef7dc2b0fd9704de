#!/bin/bash
# quick check: GPU tests selected by QK_TESTS (pytest -k), then the headline's
# kernel stats (rocprof) and two bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu -k "${QK_TESTS:-codes}" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -2 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o b --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-bfs --no-train --no-legs --no-config4 > gpurun_out/qprof.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-bfs --no-train --no-legs --no-config4 > gpurun_out/q.json 2> gpurun_out/q.err || exit $?
  echo "bench $(python -c "import json;d=json.load(open('gpurun_out/q.json'));print(round(d['ms_per_step'],3),round(d['ms_per_step_graph_cached'],3),d['roofline']['avg_launch_ms'],d['roofline'].get('layers01_codes',{}).get('avg_ms'))")"
done
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/qprof/b_kernel_stats.csv')):
    n = r['Name']
    if any(k in n for k in ('gcn_', 'csr_', 'mlp_head', 'win_plan', 'rows_gather', 'order_', 'inverse', 'bbox', 'spacing')):
        print('  %-60s %4s %9.1f' % (n[:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
