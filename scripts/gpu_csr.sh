#!/bin/bash
# graph-setup A/B: CSR tests, csr_bench for the product and variants/libmignn_old.so,
# kernel stats of the product's setup kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "csr or order" -m gpu > gpurun_out/csr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/csr_tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${CSR_VARIANTS:-old}; do
  CB_LIB=variants/libmignn_$v.so timeout -k 10 200 python scripts/csr_bench.py > gpurun_out/csr_$v.json 2> gpurun_out/csr_$v.err || exit $?
  echo "$v $(cat gpurun_out/csr_$v.json)"
done
timeout -k 10 200 python scripts/csr_bench.py > gpurun_out/csr_new.json 2> gpurun_out/csr_new.err || exit $?
echo "new $(cat gpurun_out/csr_new.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/csrprof -o csr --output-format csv -- python scripts/csr_bench.py > gpurun_out/csrprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
