#!/bin/bash
# GEMM parity tests, then timing of the default build against VARIANTS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gemm_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gemm_tests.log | head -20; exit $rc; fi
bash scripts/gpu_gemmvar.sh
