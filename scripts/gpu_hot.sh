#!/bin/bash
# hot kernel: timing + correctness (scripts/hot_bench.py) with the diagnostic
# flag sets of HB_DIAGFLAGS, then PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 240 python -u scripts/hot_bench.py > gpurun_out/hot128.json 2> gpurun_out/hot128.err
rc=$?; cat gpurun_out/hot128.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/hot128.err; exit $rc; fi
HB_H=64 timeout -k 10 240 python -u scripts/hot_bench.py > gpurun_out/hot64.json 2> gpurun_out/hot64.err
rc=$?; cat gpurun_out/hot64.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/hot64.err; exit $rc; fi
[ -n "${HB_NO_PMC:-}" ] && exit 0
mkdir -p gpurun_out/hotpmc
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  HB_PMC=1 timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/hotpmc/p$i -o run --output-format csv \
      -- python scripts/hot_bench.py > gpurun_out/hotpmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/hotpmc/p$i.log; fi
done
exit 0
