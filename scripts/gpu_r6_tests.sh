#!/bin/bash
# round 6: the whole -m gpu suite (one process) and smoke(), as the driver runs them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${TAG:-g}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r6_pytest_gpu_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/r6_pytest_gpu_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
