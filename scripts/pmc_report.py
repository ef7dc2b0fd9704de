"""Summarise rocprofv3 counter CSVs per kernel (mean over dispatches)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcsq"
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/p*/*counter_collection.csv") + glob.glob(f"{root}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        m = re.search(r"(\w+_kernel)<([^>]*)>", name)
        k = f"{m.group(1)}<{m.group(2)}>" if m else re.sub(r"\(.*", "", name).split("::")[-1]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = collections.defaultdict(dict)
for (k, c), v in agg.items():
    kern[k][c] = sum(v) / len(v)
for k, d in sorted(kern.items()):
    if "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"] < 1e5:
        continue
    print(k)
    for c in sorted(d):
        print(f"   {c:32s} {d[c]:.4g}")
