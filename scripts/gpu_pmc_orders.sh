#!/bin/bash
# fabric traffic of the hot kernel under two tile orders (PMC, one counter group per run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmco
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
i=0
for cfg in "KB_PERM=4,4 KB_ONLY=gcn16_full" "KB_PANEL=4 KB_ONLY=gcn16_chunks" "KB_PANEL=4 KB_ONLY=gcn16_full"; do
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    env $cfg timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmco/p$i -o run --output-format csv -- python scripts/kbench.py > gpurun_out/pmco/p$i.json 2> gpurun_out/pmco/p$i.err
    rc=$?; echo "pass $i ($cfg | $grp) rc=$rc $(cat gpurun_out/pmco/p$i.json | head -c 300)"
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmco/p$i.err; exit $rc; fi
  done
done
