#!/bin/bash
# PMC passes (memory side) over the eval legs only: FETCH/WRITE/TCC hit-miss
# of the aggregation and GEMM kernels.  Output: gpurun_out/pmcl/p<i>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="--steps 1 --warmup 1 --no-cpu --no-bfs --no-train --no-graph --layers 1 --grid 40,40,40 --legs ${LEGS:-gin}"
mkdir -p gpurun_out/pmcl
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmcl/p$i -o run --output-format csv \
      -- python bench.py $ARGS > gpurun_out/pmcl/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcl/p$i.log; exit $rc; fi
done
python - <<'PY'
import csv, glob, collections, statistics
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcl/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in ("sum_rows_kernel", "tf_rows_kernel", "gat_rows_kernel", "gemm_f16x3_kernel",
                  "agg_gemm_kernel", "gat_fused_kernel", "tf_fused_kernel", "head256_kernel",
                  "gin0_fused_kernel", "tf0_kernel"):
            if k in n:
                vals[(k, r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(vals.items()):
    m = {c: statistics.mean(v) for c, v in d.items()}
    rd = 2 * m.get("FETCH_SIZE", 0) * 1024 / 1e9
    wr = m.get("WRITE_SIZE", 0) * 1024 / 1e9
    h, mi = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
    print(k, f"read {rd:.2f} GB write {wr:.2f} GB l2_hit {h / max(h + mi, 1):.3f}")
PY
