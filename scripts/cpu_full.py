#!/usr/bin/env python3
"""The CPU baseline at the configurations' own sizes: the
torch-CPU oracle (oracle/flowgnn_oracle.py, the reference forward's op
pattern) timed on this host's cores at the headline 10M-node size and at
>= 0.5M nodes for the other configurations, median of the timed runs.
Writes gpurun_out/cpu_full.json (copied to profiles/ and reported by
bench.py's cpu_baseline as `full_size`).  CPU only: no GPU is touched.

  python scripts/cpu_full.py [--only name,...]
"""

import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnn-bfs-rans_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

# name: (layer type, hidden, layers, mesh, timed runs, what it stands for)
RUNS = {
    "headline": ("GCN", 128, 4, (250, 200, 200), 1, "configs[1] model at the bench headline size (10M)"),
    "gcn_h64": ("GCN", 64, 4, (250, 200, 200), 1, "SURVEY 8d H=64 layer model at 10M"),
    "gat": ("GAT", 128, 4, (100, 100, 100), 3, "configs[2] at its own size (1M)"),
    "gin": ("GIN", 256, 8, (100, 100, 100), 3, "configs[4] model at 1M (of 12.6M per GPU)"),
    "transformer": ("Transformer", 256, 6, (80, 80, 80), 3,
                    "configs[3] model at 512k (of 10M: the oracle's per-edge [E, heads, C] "
                    "tensors of the full size exceed host memory)"),
}


def log(msg):
    print(f"[cpu_full {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def graph(dims):
    """The periodic hex mesh on the host (built by mignn_grid_graph on the GPU
    when there is one, else by its numpy restatement tests/helpers.py)."""
    if torch.cuda.is_available():
        from mignn.synthetic import grid_graph
        x, ei = grid_graph(*dims, device="cuda")
        return x.cpu(), ei.cpu()
    from helpers import grid_graph_np
    x, ei = grid_graph_np(*dims)
    return torch.from_numpy(x), torch.from_numpy(ei)


def thread_sweep(orc, sd, cfg):
    """bench.cpu_thread_sweep's rule: the fastest thread count of a sweep up
    to this process's CPU affinity, on the 40^3 mesh."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    xs, eis = graph((40, 40, 40))
    sweep = {}
    for nt in sorted({c for c in (8, 16, 32, 64, 128, avail) if c <= avail}):
        torch.set_num_threads(nt)
        orc.flowgnn_forward(sd, cfg, xs, eis, None, dtype=torch.float32)
        t0 = time.perf_counter()
        orc.flowgnn_forward(sd, cfg, xs, eis, None, dtype=torch.float32)
        sweep[nt] = round(time.perf_counter() - t0, 4)
    return {"threads": min(sweep, key=sweep.get), "cpus_available": avail,
            "os_cpu_count": os.cpu_count(), "sweep_s_40x40x40": sweep}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cpu_full.json"))
    args = ap.parse_args()
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    from oracle import flowgnn_oracle as orc

    c0 = dict(hidden_dim=128, num_layers=4, layer_type="GCN")
    threads = thread_sweep(orc, seeded_state_dict(
        FlowGNN(input_dim=3, output_dim=7, **c0).state_dict(), seed=0), c0)
    log(f"threads {threads}")
    torch.set_num_threads(threads["threads"])
    cpu_model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    res = {"kind": "port", "oracle": "oracle/flowgnn_oracle.py flowgnn_forward, fp32, torch CPU",
           "threads": threads, "cpu_model": cpu_model, "runs": {}}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    names = [n for n in args.only.split(",") if n] or list(RUNS)
    for name in names:
        lt, H, L, dims, reps, what = RUNS[name]
        cfg = dict(hidden_dim=H, num_layers=L, layer_type=lt)
        sd = seeded_state_dict(FlowGNN(input_dim=3, output_dim=7, **cfg).state_dict(), seed=0)
        x, ei = graph(dims)
        times = []
        for r in range(reps):
            log(f"{name}: run {r + 1}/{reps} ({x.shape[0]} nodes, {ei.shape[1]} edges)")
            t0 = time.perf_counter()
            with torch.no_grad():
                orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float32)
            times.append(time.perf_counter() - t0)
            log(f"{name}: {times[-1]:.2f} s")
        t = statistics.median(times)
        res["runs"][name] = {
            "what": what, "workload": f"{lt.lower()}_L{L}_H{H}_periodic_hex_{dims[0]}x{dims[1]}x{dims[2]}",
            "nodes": x.shape[0], "edges": ei.shape[1], "timed_runs": reps,
            "s_per_forward": [round(v, 3) for v in times], "median_s": round(t, 3),
            "edges_per_s": L * ei.shape[1] / t, "cores": threads["threads"]}
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)
        del x, ei
    log("done")


if __name__ == "__main__":
    main()
