#!/bin/bash
# round 6: head A/B (HA_LIBS), then bench + rocprof kernel stats (no tests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "${HA_LIBS:-}" ]; then
  timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/r6_head_ab.json 2> gpurun_out/r6_head_ab.err \
      || { tail -20 gpurun_out/r6_head_ab.err; exit 1; }
  cat gpurun_out/r6_head_ab.json
fi
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o bench \
    --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu --no-bfs --no-train --no-legs --no-config4 --no-graph \
    > gpurun_out/prof_e.log 2>&1 || { tail -20 gpurun_out/prof_e.log; exit 1; }
grep '^{' gpurun_out/prof_e.log | tail -1 | cut -c1-400
