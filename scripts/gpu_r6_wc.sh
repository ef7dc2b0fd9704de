#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_win.py -k "weight_classes or codes" > gpurun_out/r6_wc.log 2>&1; rc=$?; tail -5 gpurun_out/r6_wc.log; exit $rc
