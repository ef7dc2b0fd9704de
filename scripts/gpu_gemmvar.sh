#!/bin/bash
# split-fp16 GEMM timing with alternative library builds (GB_LIB)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in gnn-bfs-rans_amd/mignn/libmignn.so ${VARIANTS}; do
  GB_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/gemm_bench.py > gpurun_out/gemmvar.out 2>&1
  rc=$?; echo "== $lib"; grep -E "f16x3|ms" gpurun_out/gemmvar.out | tail -8; if [ $rc -ne 0 ]; then tail -3 gpurun_out/gemmvar.out; exit $rc; fi
done
