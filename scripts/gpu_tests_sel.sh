#!/bin/bash
# Run a selection of GPU tests (PYTEST_SEL) under a time limit; log to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
name=${LOG_NAME:-pytest_sel}
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -v --timeout 300 --timeout-method thread --maxfail=${MAXFAIL:-20} -s ${PYTEST_ARGS:-} > gpurun_out/$name.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|max\|gpu" gpurun_out/$name.log | tail -${TAILN:-60}
exit $rc
