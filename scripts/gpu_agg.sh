#!/bin/bash
# Aggregation kernels: GPU parity tests, A/B timing at the leg sizes, then
# the SQ-side PMC passes (MFMA busy etc.) over a short bench with the legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -v --timeout 120 --timeout-method thread > gpurun_out/agg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/agg_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/agg_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u scripts/agg_bench.py > gpurun_out/agg_bench.json 2> gpurun_out/agg_bench.err
rc=$?; tail -5 gpurun_out/agg_bench.err; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${PMC:-}" ]; then
  BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-bfs --no-train --no-graph" bash scripts/pmc_sq.sh
fi
