#!/usr/bin/env python3
"""Benchmark: edges/s of the FlowGNN forward on MI355X (BASELINE.json metric).

Workload (one "step" = one full eval-mode forward):
  4-layer GCN, hidden 128, output 7 (the model of BASELINE configs[1]) on a
  3-D periodic hex mesh of 250x200x200 = 10M nodes / 60M directed edges
  (avg degree 6) PER GPU -- the north-star size.  At N GPUs the mesh is
  250x200x(200N), k-slab partitioned, with an RCCL halo exchange of one
  50k-node plane per side per layer (weak scaling).
  value = L * E_total * K / t  (E_total = directed edges of edge_index over all
  ranks, GCN's implicit self-loops not counted), t = max over ranks.

Extra objects on the same JSON line:
  roofline     : the fused GCN layer kernel (default precision "f16x3":
                 mignn_gcn_layer_f16x3, split-fp16 MFMA with fp32 accumulation;
                 "f32": mignn_gcn_layer on the f32 MFMA), timed live with HIP
                 events on the stream it is launched on; algorithmic bytes and
                 flops per launch as in DESIGN.md §Roofline; the binding bound
                 (HBM 8.0 TB/s vs the compute time of the precision's MFMA +
                 VALU work) is reported, the other side is given too.
                 traffic = PMC-measured HBM bytes per launch from profiles/
                 (rocprofv3 --pmc passes of this command, scripts/pmc.sh).
  exact_f32    : the same forward in the exact-fp32 mode (MIGNN_PRECISION=f32),
                 graph cached, for reference.
  cpu_baseline : the CPU oracle (pure-torch restatement of the reference
                 forward, the same op pattern PyG runs on the CPU) timed on
                 this box's host cores on a bounded 1M-node sample (rank 0, N=1).
  bfs_mesh     : the reference BFS mesh (train-path graph, 12,225 nodes /
                 48,330 edges; configs[1]) -- edges/s and max-abs / mean-abs
                 error of the raw [N,7] output vs the committed reference-CPU
                 golden output.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "edges/s GNN forward (+MAE vs ref) on BFS mesh & 10M-node synthetic, 1/2/4/8 GPU"
HBM_PEAK = 8.0e12      # B/s, MI355X spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK = 157.3e12  # FLOP/s, dense f32 MFMA (= f32 vector peak)
F16_MFMA_PEAK = 2.5e15     # FLOP/s, dense f16 MFMA (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--layers", type=int, default=4)
    p.add_argument("--hidden", type=int, default=128)
    p.add_argument("--layer-type", default="GCN")
    p.add_argument("--grid", default="250,200,200", help="per-GPU nx,ny,nz")
    p.add_argument("--shuffle", action="store_true", help="seeded random node order (N=1)")
    p.add_argument("--precision", default="f16x3", choices=["f16x3", "f32"],
                   help="GCN transform / output head arithmetic (FlowGNN.precision)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-bfs", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="skip the mesh->graph builder leg")
    p.add_argument("--cpu-grid", default="100,100,100")
    p.add_argument("--no-train", action="store_true", help="skip the training-step leg")
    p.add_argument("--train-grid", default="100,100,100")
    return p.parse_args()


def gcn_layer_cost(n_rows, e_prime, H):
    """Algorithmic bytes / flops of one fused GCN layer launch over n_rows
    destination rows with e_prime CSR entries."""
    bytes_ = 4 * (2 * n_rows * H + (n_rows + 1) + e_prime + n_rows)
    flops = 2 * n_rows * H * H + 2 * e_prime * H
    return bytes_, flops


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from mignn import FlowGNN
    from mignn.dist import FlowGNNExecutor, SlabPartition, sharded_forward
    from mignn.synthetic import grid_graph, seeded_state_dict

    nx, ny, nz = (int(v) for v in args.grid.split(","))
    L, H = args.layers, args.hidden
    cfg = dict(hidden_dim=H, num_layers=L, layer_type=args.layer_type)
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    model.precision = args.precision

    part = SlabPartition(nx, ny, nz, rank, world)
    if world == 1:
        x, ei = grid_graph(nx, ny, nz, device=dev, permute_seed=0 if args.shuffle else None)
        E_local = ei.shape[1]
        N_local = x.shape[0]

        def step():
            return model(x, ei)
    else:
        x, ei_g = grid_graph(nx, ny, nz * world, device=dev, z_begin=rank * nz, z_count=nz)
        ei = part.localize(ei_g)
        del ei_g
        E_local = ei.shape[1]
        N_local = part.n_own
        ex = FlowGNNExecutor(model, part, ei)

        def step():
            if model._csr.capacity <= 0:      # graph setup inside the step (see timed_loop)
                ex.build_graph()
            return sharded_forward(ex, part, x)

    # ---- live per-launch timing of the dominant (GCN layer) kernel
    launches = []   # (start_event, end_event, n_rows)
    orig_layer = model._layer

    def timed_layer(i, layer, csr, xin, out, rb, re):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig_layer(i, layer, csr, xin, out, rb, re)
        e1.record()
        if recording[0]:
            launches.append((e0, e1, re - rb))

    recording = [False]
    model._layer = timed_layer

    def timed_loop(cache_graph):
        # cache_graph False: every forward rebuilds the CSR + GCN norm from
        # edge_index, as the reference's GCNConv(cached=False) recomputes its
        # normalisation each call; True: steady state on a fixed mesh
        model._csr.capacity = 4 if cache_graph else 0
        model._csr.entries.clear()
        with torch.no_grad():
            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            recording[0] = not cache_graph
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            recording[0] = False
        el = t1 - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        return el

    elapsed = timed_loop(cache_graph=False)
    elapsed_cached = timed_loop(cache_graph=True)

    # ---- roofline of the fused GCN layer kernel (this rank's launches)
    deg_plus_self = E_local / N_local + 1.0
    tot_ms = 0.0
    tot_bytes = tot_flops = 0.0
    for e0, e1, n in launches:
        tot_ms += e0.elapsed_time(e1)
        b, f = gcn_layer_cost(n, n * deg_plus_self, H)
        tot_bytes += b
        tot_flops += f
    roofline = None
    if launches and args.layer_type == "GCN":
        t_s = tot_ms / 1e3
        gbs = tot_bytes / t_s
        t_hbm = tot_bytes / HBM_PEAK
        n_rows = sum(n for _, _, n in launches)
        if model.precision == "f16x3":
            # 3 fp16 MFMA products per fp32 product on the transform; the
            # gather-aggregate FMAs on the fp32 VALU
            t_comp = (3 * 2 * n_rows * H * H / F16_MFMA_PEAK
                      + 2 * n_rows * deg_plus_self * H / F32_MFMA_PEAK)
            kname = "gcn_f16x3_kernel<%d> (mignn_gcn_layer_f16x3)" % H
            comp_peak, comp_note = F16_MFMA_PEAK, "f16 MFMA x3 (split fp32) + f32 VALU aggregate"
        else:
            t_comp = tot_flops / F32_MFMA_PEAK
            kname = "fused_tile_kernel<%d, %d, 0, true> (mignn_gcn_layer)" % (H, H)
            comp_peak, comp_note = F32_MFMA_PEAK, "f32 MFMA"
        per_launch_bytes = tot_bytes / len(launches)
        traffic = None
        tf = os.path.join(HERE, "profiles", "gcn_layer_traffic.json")
        if os.path.exists(tf):
            try:
                with open(tf) as fh:
                    tj = json.load(fh)
                if (tj.get("config") == f"{args.layer_type}_L{L}_H{H}_{nx}x{ny}x{nz}"
                        and tj.get("kernel", "").split("<")[0] in kname):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        bound_hbm = t_hbm >= t_comp
        t_bound = max(t_hbm, t_comp)
        roofline = {
            "kernel": kname,
            "bound": "hbm" if bound_hbm else "mfma",
            "achieved": round((gbs / 1e9) if bound_hbm else (tot_flops / t_s / 1e12), 3),
            "peak": round((HBM_PEAK / 1e9) if bound_hbm else (comp_peak / 1e12), 1),
            "unit": "GB/s" if bound_hbm else "TFLOP/s",
            "frac": round(t_bound / t_s, 4),
            "traffic": traffic,
            "avg_launch_ms": round(tot_ms / len(launches), 4),
            "launches": len(launches),
            "algorithmic_bytes_per_launch": int(per_launch_bytes),
            "algorithmic_flops_per_launch": int(tot_flops / len(launches)),
            "hbm_side": {"achieved_GBps": round(gbs / 1e9, 1), "peak_GBps": HBM_PEAK / 1e9,
                         "frac": round(gbs / HBM_PEAK, 4), "t_min_ms": round(1e3 * t_hbm / len(launches), 4)},
            "compute_side": {"model": comp_note, "t_min_ms": round(1e3 * t_comp / len(launches), 4),
                             "frac": round(t_comp / t_s, 4)},
        }

    model._layer = orig_layer
    exact = None
    if model.precision != "f32":
        model.precision = "f32"
        el32 = timed_loop(cache_graph=True) if args.steps > 0 else 0.0
        model.precision = args.precision
        exact = {"ms_per_step_graph_cached": 1e3 * el32 / args.steps,
                 "value_graph_cached": L * E_local * world * args.steps / el32}

    E_total = E_local * world
    value = L * E_total * args.steps / elapsed
    line = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
        "graph_setup_in_step": True,
        "ms_per_step_graph_cached": 1e3 * elapsed_cached / args.steps,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "arithmetic": ("f16x3: fp32 values split into fp16 hi+lo, 3 fp16 MFMA products, fp32 "
                       "accumulate (GCN transform, output head); gathers / norms / biases fp32; "
                       "max-abs error <= 1e-5 (BASELINE tolerance)")
                      if model.precision == "f16x3" else "exact fp32 (f32 MFMA / VALU)",
        "config": {
            "workload": f"{args.layer_type.lower()}_L{L}_H{H}_periodic_hex_{nx}x{ny}x{nz}_per_gpu"
                        + ("_shuffled" if args.shuffle else ""),
            "model": f"FlowGNN({args.layer_type}, layers={L}, hidden={H}, out=7), eval, "
                     "seeded random weights",
            "nodes_per_gpu": N_local, "edges_per_gpu": E_local, "global_batch": 1,
            "parallelism": "single" if world == 1 else f"kslab{world}+rccl_halo",
            "internal_node_order": ("locality (4x4-cell pencils, mignn_locality_order; part of "
                                    "the per-step graph setup)")
                                   if (world == 1 and model._use_reorder(x)) else "as given",
        },
        "roofline": roofline,
        "exact_f32": exact,
    }
    if world > 1:
        dist.barrier()

    if rank == 0 and not args.no_bfs:
        line["bfs_mesh"] = bfs_leg(dev)
    if rank == 0 and world == 1 and not args.no_graph:
        line["graph_build"] = graph_build_leg(dev, nx, ny, nz, not args.no_cpu)
    if rank == 0 and world == 1 and not args.no_train:
        line["train_step"] = train_leg(dev, args)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_leg(model, sd, cfg, args, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bfs_leg(dev):
    """configs[1]: 4-layer GCN H=128 on the reference-built BFS mesh vs the
    committed reference-CPU output."""
    import numpy as np
    from mignn import FlowGNN

    g = np.load(os.path.join(HERE, "tests", "golden", "bfs_graphs.npz"))
    m = np.load(os.path.join(HERE, "tests", "golden", "models.npz"))
    name = "c2_gcn_h128_l4"
    cfg = json.loads(str(m[f"{name}/cfg"]))
    sd = {k[len(name) + 4:]: torch.from_numpy(m[k]) for k in m.files
          if k.startswith(f"{name}/sd/")}
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    x = torch.from_numpy(g["train_x"]).to(dev)
    ei = torch.from_numpy(g["train_ei"].astype(np.int64)).to(dev)
    ea = torch.from_numpy(g["train_ea"]).to(dev)
    y32 = torch.from_numpy(m[f"{name}/train/y32"])
    times = []
    with torch.no_grad():
        for _ in range(3):
            y = model(x, ei, ea)
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y = model(x, ei, ea)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
    t = statistics.median(times)
    err = (y.cpu() - y32).abs()
    return {"config": "configs[1]: GCN L4 H128, train-path BFS mesh",
            "nodes": int(x.shape[0]), "edges": int(ei.shape[1]),
            "ms_per_forward": round(t * 1e3, 4),
            "edges_per_s": cfg["num_layers"] * ei.shape[1] / t,
            "max_abs_err_vs_ref_cpu": err.max().item(), "mae_vs_ref_cpu": err.mean().item()}


def train_leg(dev, args):
    """one train.py step (train.py:158-196: model.train()
    forward with batch-stat BN + dropout 0.1, WeightedMSELoss, backward,
    clip_grad_norm_, Adam) per layer type, L4 H128, on a periodic hex grid
    (default 1M nodes / 6M edges).  edges/s = L * E / t_step (forward +
    backward counted once, as the reference's train loop sees it)."""
    from mignn import FlowGNN
    from mignn.normalization import WeightedMSELoss
    from mignn.synthetic import grid_graph

    nx, ny, nz = (int(v) for v in args.train_grid.split(","))
    x, ei = grid_graph(nx, ny, nz, device=dev)
    n, e = x.shape[0], ei.shape[1]
    g = torch.Generator(device="cpu").manual_seed(11)
    target = torch.randn((n, 7), generator=g).to(dev)
    weights = {"U": 1.0, "p": 3.0, "k": 0.5, "epsilon": 0.5, "nut": 0.5}   # train.py:352-360
    out = {"workload": f"periodic_hex_{nx}x{ny}x{nz}", "nodes": n, "edges": e,
           "step": "train fwd + WeightedMSELoss + backward + clip_grad_norm_ + Adam"}
    for lt in ("GCN", "GIN", "GAT", "Transformer"):
        torch.manual_seed(0)
        model = FlowGNN(input_dim=3, hidden_dim=args.hidden, output_dim=7,
                        num_layers=args.layers, layer_type=lt, dropout=0.1).to(dev).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
        crit = WeightedMSELoss(field_weights=weights, use_fieldwise=True, pressure_ref_weight=0.1)
        ea = None if lt == "Transformer" else torch.zeros((e, 4), device=dev)

        def step():
            opt.zero_grad()
            loss = crit(model(x, ei, ea), target, pressure_ref_weight=0.1)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
            return loss

        for _ in range(2):
            step()
        torch.cuda.synchronize()
        k = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            loss = step()
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / k
        out[lt] = {"ms_per_step": round(t * 1e3, 3),
                   "edges_per_s": args.layers * e / t,
                   "loss_finite": bool(torch.isfinite(loss).item())}
        del model, opt
    return out


def graph_build_leg(dev, nx, ny, nz, with_cpu):
    """mesh -> graph (GraphConstructor.build_graph, train
    path: filter_internal, n_internal_cells = all cells) on a blockMesh-ordered
    polyMesh of the bench's cell count; the numpy oracle (vectorised CPU
    restatement of the reference's loops) on a bounded 1M-cell sample."""
    from mignn.graph import GraphConstructor
    from mignn.synthetic import hex_polymesh

    mesh = hex_polymesh(nx, ny, nz, device=dev)
    gc = GraphConstructor(mesh, device=dev)
    n = mesh["n_cells"]
    kw = dict(node_features=mesh["cell_centers"], filter_internal=True, n_internal_cells=n)
    g = gc.build_graph(**kw)                     # warm-up
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        g = gc.build_graph(**kw)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts)
    E = g.num_edges
    out = {"cells": n, "faces": int(mesh["owner"].numel()), "edges": E,
           "ms": round(1e3 * t, 3), "edges_per_s": E / t,
           "note": "includes the one host read of the edge count and the output allocation"}
    del g, gc, mesh
    if with_cpu:
        from oracle import graph_oracle as go
        m = hex_polymesh(100, 100, 100, device="cpu")
        mc = {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in m.items()}
        t0 = time.perf_counter()
        _, ei, _, _ = go.build_graph(mc, node_features=mc["cell_centers"], filter_internal=True,
                                     n_internal_cells=mc["n_cells"])
        tc = time.perf_counter() - t0
        out["cpu_oracle"] = {"edges_per_s": ei.shape[1] / tc, "s": round(tc, 3), "cores": 1,
                             "sample": "100x100x100 cells, vectorised numpy oracle"}
    return out


def cpu_leg(model, sd, cfg, args, dev):
    """The CPU oracle on a bounded sample of the same workload (1M-node mesh)."""
    from oracle import flowgnn_oracle as orc
    from mignn.synthetic import grid_graph

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cx, cy, cz = (int(v) for v in args.cpu_grid.split(","))
    xg, eig = grid_graph(cx, cy, cz, device=dev)
    with torch.no_grad():
        yg = model(xg, eig).cpu()
    x, ei = xg.cpu(), eig.cpu()
    times = []
    y = None
    for it in range(3):          # 1 warm-up + 2 timed
        t0 = time.perf_counter()
        y = orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float32)
        dt = time.perf_counter() - t0
        if it > 0:
            times.append(dt)
    t = statistics.median(times)
    cpu_model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": cfg["num_layers"] * ei.shape[1] / t, "unit": "edges/s", "cores": threads,
            "kind": "port",
            "sample": f"{cfg['layer_type']} L{cfg['num_layers']} H{cfg['hidden_dim']} forward on "
                      f"the {cx}x{cy}x{cz} periodic mesh ({x.shape[0]} nodes, {ei.shape[1]} edges), "
                      f"torch-CPU oracle fp32, median of 2 after 1 warm-up",
            "s_per_forward": round(t, 3), "cpu_model": cpu_model,
            "gpu_vs_cpu_max_abs_err": (yg - y).abs().max().item()}


if __name__ == "__main__":
    main()
