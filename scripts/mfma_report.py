"""MFMA / VALU utilisation per kernel from the SQ PMC passes of scripts/pmc_sq.sh.

  cycles     = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs' GRBMs: checked
               against the kernel durations, ~2 GHz)
  mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 4 SIMDs * CUs)
               (MFMA_BUSY counts matrix-pipe cycles summed over all SIMDs --
               32 x N for the exact-f32 16x16x4 kernel, whose N is known:
               5.12e9 cycles for 160M MFMAs)
  cu_busy    = SQ_BUSY_CU_CYCLES / (cycles * CUs)
Prints a JSON object keyed "kernel [grid]": means over the dispatches of one
kernel at one grid size that ran longer than 100k GPU cycles."""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcsq"
cus = int(sys.argv[2]) if len(sys.argv) > 2 else 256
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
        k = (m.group(1) + (m.group(2) or "")) if m else re.sub(r"\(.*", "", name).split("::")[-1]
        k = f"{k} [{r['Grid_Size']}]"
        # one dispatch = one (file, dispatch id); counters of a pass are per dispatch
        per[k][(f, r["Dispatch_Id"])].append((r["Counter_Name"], float(r["Counter_Value"])))
        per[k][(f, r["Dispatch_Id"])].append(
            ("_ns", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 4.0))
out = {}
for k, disp in per.items():
    acc = collections.defaultdict(list)
    for _, cv in disp.items():
        d = collections.defaultdict(float)
        for c, v in cv:
            d[c] += v
        d["_ns"] /= sum(1 for c, _ in cv if c == "_ns") / 4.0
        for c, v in d.items():
            acc[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in acc.items()}
    if mean.get("GRBM_GUI_ACTIVE", 0) < 8e5 and "GRBM_GUI_ACTIVE" in mean:
        continue
    row = {"dispatches_per_pass": max(len(v) for v in acc.values())}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        cyc = mean["GRBM_GUI_ACTIVE"] / 8.0
        row["gpu_cycles"] = round(cyc)
        row["ms"] = round(mean["_ns"] / 1e6, 4)
        row["clock_GHz"] = round(cyc / mean["_ns"], 3)
        row["mfma_util"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 4 * cus), 4)
        if "SQ_BUSY_CU_CYCLES" in mean:
            row["cu_busy"] = round(mean["SQ_BUSY_CU_CYCLES"] / (cyc * cus), 4)
    for c in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
        if c in mean:
            row[c] = mean[c]
    if "SQ_WAVE_CYCLES" in mean and mean["SQ_WAVE_CYCLES"] > 0:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in mean:
                row[c.replace("SQ_", "").lower() + "_frac"] = round(mean[c] / mean["SQ_WAVE_CYCLES"], 4)
    out[k] = row
def ours(k):
    name = k.split(" [")[0]
    return not name.startswith(("index_elementwise", "elementwise", "vectorized", "reduce_kernel",
                                "trampoline", "init_lookback", "rocblas", "Cijk", "__amd"))


keep = {k: v for k, v in out.items() if ours(k)}
print(json.dumps(dict(sorted(keep.items())), indent=1))
