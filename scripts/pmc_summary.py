"""Per-kernel summary of the PMC passes of scripts/gpu_hot.sh (gpurun_out/hotpmc)."""
import csv
import collections
import glob
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hotpmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gcn" not in n and "diag" not in n:
            continue
        key = n.replace("(anonymous namespace)::", "").split("(")[0][:90]
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    m = {c: statistics.mean(v) for c, v in d.items()}
    print(k)
    for c, v in sorted(m.items()):
        print(f"   {c:32s} {v:.4g}")
    if "FETCH_SIZE" in m:
        print("   fabric read GB", round(2 * m["FETCH_SIZE"] * 1024 / 1e9, 3))
    if "TCC_HIT_sum" in m:
        print("   L2 hit", round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3))
