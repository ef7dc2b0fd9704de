"""Summarise scripts/gpu_kpmc.sh output: per kernel (name prefix), the mean
of each counter per dispatch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kpmc"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        import re
        m = re.search(r"(gcn_\w+_kernel|agg_gemm_kernel|tf_fused_kernel|gat_fused_kernel|"
                      r"gemm_f16x3_kernel|gin0_fused_kernel|mlp_head_kernel)(<[^>]*>)?", k)
        if not m:
            continue
        short = m.group(1) + (m.group(2) or "")
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
print(json.dumps(out, indent=1))
