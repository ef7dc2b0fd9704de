#!/bin/bash
# round 6: CSR build A/B (product vs CB_LIB variant, alternating, same box), hashes compared
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python -u scripts/csr_bench.py 2>> gpurun_out/r6_csr.err | sed 's/^/product /' | tee -a gpurun_out/r6_csr.txt || exit 1
  CB_LIB=${CB:-variants/libmignn_runpos.so} timeout -k 10 200 python -u scripts/csr_bench.py 2>> gpurun_out/r6_csr.err | sed 's/^/variant /' | tee -a gpurun_out/r6_csr.txt || exit 1
done
