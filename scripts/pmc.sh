#!/bin/bash
# PMC passes for the bench workload (one counter group per rocprofv3 run, no
# tracing domains combined with --pmc).  Output: gpurun_out/pmc/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --no-bfs}"
mkdir -p gpurun_out/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv \
      -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
