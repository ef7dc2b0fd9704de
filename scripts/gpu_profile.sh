#!/bin/bash
# round profile set: kernel stats of the bench, PMC traffic of the hot kernel,
# SQ (MFMA/VALU) passes over the bench with the legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
[ -n "${SKIP_STATS:-}" ] || timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv \
    -- python bench.py --steps 5 --warmup 2 --no-cpu --no-bfs --no-train > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof.log; exit $rc; fi
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-bfs --no-legs --no-train --no-graph --no-config4" bash scripts/pmc.sh
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "${SKIP_SQ:-}" ] || BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-bfs --no-train --no-graph" bash scripts/pmc_sq.sh
