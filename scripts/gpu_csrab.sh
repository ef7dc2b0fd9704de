#!/bin/bash
# CSR build A/B: CSR tests, then csr_bench for the product and CSR_VARIANTS, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_win.py -k "csr or codes or natural" -m gpu > gpurun_out/csr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/csr_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in product ${CSR_VARIANTS:-}; do
    if [ "$v" = product ]; then unset CB_LIB; else export CB_LIB=variants/libmignn_$v.so; fi
    timeout -k 10 200 python scripts/csr_bench.py > gpurun_out/csr_$v.json 2> gpurun_out/csr_$v.err || exit $?
    echo "$v $(cat gpurun_out/csr_$v.json)"
  done
done
