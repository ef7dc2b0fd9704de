#!/bin/bash
# selected GPU tests (PYTEST_K) + a short headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_sel.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_sel.log | head; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-bfs --no-train --no-graph --legs ${LEGS:-gcn_h64,shuffled} > gpurun_out/bench_sel.log 2>&1
rc=$?; tail -1 gpurun_out/bench_sel.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'cached',d['ms_per_step_graph_cached'],'frac',d['roofline']['frac'],'launch_ms',d['roofline']['avg_launch_ms']); print({k:(v['ms_per_forward'],v['roofline']['frac']) for k,v in d['legs'].items()})"
exit $rc
