#!/bin/bash
# round 6 records: bench (N = 1, default legs) -> r6_bench.json; the headline
# under rocprofv3 --kernel-trace --stats; window-kernel PMC passes (H = 64, 128)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-g}
timeout -k 10 600 python -u bench.py > gpurun_out/r6_bench_$tag.log 2>&1 || { tail -20 gpurun_out/r6_bench_$tag.log; exit 1; }
grep '^{' gpurun_out/r6_bench_$tag.log | tail -1 > gpurun_out/r6_bench_$tag.json
cut -c1-300 gpurun_out/r6_bench_$tag.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o bench \
    --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu --no-bfs --no-train --no-legs --no-config4 --no-graph \
    > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
grep '^{' gpurun_out/prof_$tag.log | tail -1 | cut -c1-200
if [ -n "${PMC:-}" ]; then
  for h in 64 128; do
    KP_H=$h KP_KINDS=win,winagg KP_GROUPS="FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" bash scripts/gpu_kpmc.sh
    python scripts/kpmc_report.py gpurun_out/kpmc > gpurun_out/r6_kpmc_h$h.json
    rm -rf gpurun_out/kpmc
  done
fi
