#!/bin/bash
# round 6 combined: the -m gpu suite + smoke, the GIN / H = 256 head A/B
# (AB_LIBS / HA_LIBS), then the bench (+ legs) and its rocprof kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${TAG:-i}
TAG=$tag bash scripts/gpu_r6_tests.sh || exit $?
if [ -n "${AB_LIBS:-}" ]; then bash scripts/gpu_r6_gin.sh || exit $?; fi
TAG=$tag bash scripts/gpu_r6_bench.sh
