#!/bin/bash
# One GPU-box session: smoke -> GPU tests -> bench (-> rocprof kernel stats).
# Stops at the first abort / fault / timeout (exit >1); a plain test failure
# (exit 1) still lets the bench run so the numbers are collected.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${PROFILE:-}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench \
      --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-bfs --no-train \
      > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
fi
exit $rc
