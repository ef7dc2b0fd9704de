"""Per-launch memory-side traffic of the fused GCN layer kernel from the
rocprofv3 --pmc passes of scripts/pmc.sh (bench.py workload), corrected as
MI355X_MICROARCH.md §HBM prescribes for gfx950:
  read  bytes = 2 x FETCH_SIZE   (FETCH_SIZE tallies 128-B requests at 64 B)
  write bytes = WRITE_SIZE       (exact for 16-B-per-lane stores)
FETCH/WRITE count the L2's fabric requests, so Infinity-Cache hits are
included: the figure is an upper bound of HBM bytes.  Writes
profiles/gcn_layer_traffic.json (read by bench.py's roofline object)."""
import csv
import glob
import json
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
config = sys.argv[2] if len(sys.argv) > 2 else "GCN_L4_H128_250x200x200"
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "gcn_f16x3_kernel<128"
vals = {}
for f in glob.glob(f"{root}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
if not vals.get("FETCH_SIZE"):
    sys.exit(f"no FETCH_SIZE records for {KERNEL!r} under {root}; nothing written")
mean = {k: statistics.mean(v) for k, v in vals.items()}
out = {
    "config": config, "kernel": KERNEL, "launches_sampled": len(vals.get("FETCH_SIZE", [])),
    "fetch_size_bytes": mean.get("FETCH_SIZE", 0) * 1024,
    "write_size_bytes": mean.get("WRITE_SIZE", 0) * 1024,
}
if "TCC_HIT_sum" in mean:
    out["l2_hit_rate"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
if "TCC_EA0_RDREQ_sum" in mean:   # cross-check: 128-B requests (+ 32-B ones)
    r32 = mean.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    out["rdreq_bytes"] = (mean["TCC_EA0_RDREQ_sum"] - r32) * 128 + r32 * 32
out["read_bytes_per_launch"] = 2 * out["fetch_size_bytes"]
out["hbm_bytes_per_launch"] = out["read_bytes_per_launch"] + out["write_size_bytes"]
out["note"] = ("fabric-side bytes (L2 misses, Infinity-Cache hits included): 2 x FETCH_SIZE "
               "+ WRITE_SIZE per launch, gfx950 FETCH_SIZE correction per MI355X_MICROARCH.md")
print(json.dumps(out, indent=1))
os.makedirs("profiles", exist_ok=True)
with open("profiles/gcn_layer_traffic.json", "w") as fh:
    json.dump(out, fh, indent=1)
