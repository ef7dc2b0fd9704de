#!/bin/bash
# codes form: tests, kernel stats, headline A/B (codes on / off, alternating)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_win.py -k "codes or csr" -m gpu > gpurun_out/codes_tests.log 2>&1
rc=$?; tail -2 gpurun_out/codes_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof1 -o b --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-bfs --no-train --no-legs --no-config4 > gpurun_out/cprof1.log 2>&1 || exit $?
for c in 1 0 1 0; do
  MIGNN_GCN_CODES=$c timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-bfs --no-train --no-legs --no-config4 > gpurun_out/bench_codes$c.json 2> gpurun_out/bench_codes$c.err || exit $?
  echo "codes=$c $(python -c "import json;d=json.load(open('gpurun_out/bench_codes$c.json'));print(d['value'],d['ms_per_step'],d['ms_per_step_graph_cached'])")"
done
