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
                 graph cached, with the roofline of its fused layer kernel
                 (fused_tile_kernel on the f32 MFMA).
  legs         : the other BASELINE.json configurations and SURVEY §8d legs,
                 each an eval forward at its named size with the graph cached
                 (steady state; edges/s = L*E/t) and a per-layer roofline
                 (the layer's launches timed by HIP events; MFMA-bound layers
                 against the dense f32 MFMA peak, executed flops):
                   gcn_h64   : §8d's HBM-target layer, GCN L4 H64, 10M nodes
                   shuffled  : the headline model on a seeded random node order
                               (locality stress; the locality order is rebuilt
                               inside every timed step, as in the headline)
                   gat       : configs[2], GAT L4 H128 heads 4, 1M nodes
                   transformer: configs[3], TransformerConv L6 H256, 10M nodes
                   gin       : configs[4]'s model on one GPU's shard of the 100M
                               mesh (500 x 400 x 63 = 12.6M nodes), GIN L8 H256
  config4      : configs[4] at the run's N (every N, every rank): GIN L8 H256 on
                 500 x 400 x 63 nodes PER GPU (100.8M at N = 8), k-slab ranges,
                 mignn.dist.FlowGNNShard per rank with the RCCL halo
  cpu_baseline : the CPU oracle (pure-torch restatement of the reference
                 forward, the same op pattern PyG runs on the CPU) timed on
                 this box's host cores (the fastest thread count of a sweep)
                 on the headline workload itself -- GCN L4 H128 on the
                 250x200x200 mesh, one timed forward in this run (rank 0,
                 N=1); a 1M-node sample (median of 2, with its accuracy vs
                 fp64) beside it.
  bfs_mesh     : configs[1]'s model on the reference BFS mesh (train-path
                 graph, 12,225 nodes / 48,330 edges) -- edges/s, max-abs /
                 mean-abs error of the raw [N,7] output vs the committed
                 reference-CPU golden output, and the per-field error after the
                 reference's float64 denormalisation (inference.py:76-85,
                 normalization.py:111-133, tests/golden/normalizer.json).
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
HEADS = 4


def layer_flops(lt, n_rows, e_rows, H):
    """Executed flops of one layer over n_rows destination rows with e_rows
    aggregation entries (E' incl. self-loops for GCN/GAT), as the engine runs
    it (DESIGN.md §3 kernel table); the reference formulation's count differs
    only for TransformerConv (26 N H^2 + 16 E H: Q/K/V/skip GEMMs, which the
    engine re-associates to 18 N H^2)."""
    if lt == "GCN":
        return 2 * n_rows * H * H + 2 * e_rows * H
    if lt == "GIN":
        return 4 * n_rows * H * H + e_rows * H
    if lt == "GAT":
        return 8 * n_rows * H * H + 8 * e_rows * H + 16 * n_rows * H
    return 18 * n_rows * H * H + 16 * e_rows * H          # Transformer (re-associated)


def gemm_flops(lt, n_rows, H):
    """The node-transform (MFMA GEMM) part of layer_flops; the rest is
    edge-wise aggregation on the VALU."""
    return {"GCN": 2, "GIN": 4, "GAT": 8, "Transformer": 18}[lt] * n_rows * H * H


def layer_bytes(n_rows, e_rows, H, gcn=False):
    """Algorithmic HBM bytes of one fused layer: read x rows and write the
    output rows once, the CSR arrays once."""
    return 4 * (2 * n_rows * H + (n_rows + 1) + e_rows + (n_rows if gcn else 0))


def progress(msg):
    """A progress line on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


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
    p.add_argument("--cpu-sample-only", action="store_true",
                   help="CPU baseline on the --cpu-grid sample only (not the headline mesh)")
    p.add_argument("--no-train", action="store_true", help="skip the training-step leg")
    p.add_argument("--train-grid", default="100,100,100")
    p.add_argument("--no-legs", action="store_true", help="skip the other-config legs")
    p.add_argument("--legs", default="gcn_h64,shuffled,gat,transformer,gin",
                   help="comma list of legs (see the docstring)")
    p.add_argument("--no-config4", action="store_true",
                   help="skip the configs[4] leg (GIN L8 H256, 500x400x63 per GPU, sharded)")
    p.add_argument("--oversubscribe", action="store_true",
                   help="rehearsal only: every rank on GPU 0, gloo + host-staged halo")
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
    # --oversubscribe (rehearsal of the N > 1 path on a one-GPU box only):
    # every rank on device 0, gloo with the halo staged through host memory
    # (mignn.dist.DistExchange); the driver's multi-GPU runs use one GPU per
    # rank and RCCL
    if args.oversubscribe:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.oversubscribe:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from mignn import FlowGNN
    from mignn.dist import DistExchange, DistRequests, FlowGNNShard, RangeLayout, sharded_forward
    from mignn.gnn_model import locality_order
    from mignn.synthetic import grid_graph, seeded_state_dict

    nx, ny, nz = (int(v) for v in args.grid.split(","))
    L, H = args.layers, args.hidden
    cfg = dict(hidden_dim=H, num_layers=L, layer_type=args.layer_type)
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    model.precision = args.precision

    if world == 1:
        x, ei = grid_graph(nx, ny, nz, device=dev, permute_seed=0 if args.shuffle else None)
        E_local = ei.shape[1]
        N_local = x.shape[0]

        def step():
            return model(x, ei)
    else:
        # contiguous node ranges of the 250 x 200 x (200 N) mesh (natural order:
        # k-slabs), this rank's in-edges with global ids, RCCL halo exchange.
        # Each timed step (graph cache off, as at N = 1) rebuilds the partition
        # layout (ghost lists, interior-first locality order, send lists) and
        # the rank-local CSR + GCN weights (with the ghost-degree exchange), as
        # the N = 1 step rebuilds its order and CSR from edge_index
        x, ei = grid_graph(nx, ny, nz * world, device=dev, z_begin=rank * nz, z_count=nz)
        E_local = ei.shape[1]
        N_local = x.shape[0]
        bounds = [r * N_local for r in range(world + 1)]
        exch = DistExchange()
        if not model._use_reorder(x):
            order = None
        elif model._column_order():
            # the column order, as on one GPU: its info marks the rank-local
            # CSR for the window kernel (the interior range's plan takes the
            # column schedule with the planes per column from the CSR)
            order = lambda p, e: (lambda r: (r[0], r[2]))(locality_order(p, e, cols=True))  # noqa: E731
        else:
            order = lambda p, e: locality_order(p, e)[0]  # noqa: E731
        shard_box = [None]

        def build_shard():
            # the whole per-graph setup, as FlowGNN.forward does it at N = 1
            # from edge_index: partition layout (ghost lists, interior-first
            # locality order, request lists), rank-local CSR + GCN weights,
            # ghost coordinates
            lay = RangeLayout(ei, bounds, rank, DistRequests(), pos=x, order_fn=order)
            sh = FlowGNNShard(model, lay, x)
            sh.setup(exch, [sh])
            shard_box[0] = sh

        build_shard()

        def step():
            if model._csr.capacity <= 0:      # graph setup inside the step (see timed_loop)
                build_shard()
            return sharded_forward([shard_box[0]], exch, [x])[0]

    # ---- live per-launch timing of the dominant (GCN layer) kernel
    from mignn import _lib
    dev_errors = [0]
    launches = []   # (start_event, end_event, n_rows) of the headline loop
    launches32 = []  # the same in the exact-fp32 loop
    launches01 = []  # layers 0 + 1 in the codes form (GCN H = 128, window route)
    recording = [None]
    restore = time_layers(model, recording, launches01)

    def timed_loop(cache_graph, rec_into=None):
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
            recording[0] = rec_into
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            recording[0] = None
        el = t1 - t0
        # in-kernel protocol failures during the timed steps (mignn_device_errors:
        # a launch whose bounded LDS wait ran out wrote wrong rows) fail the run
        dev_err = _lib.device_errors(clear=True)
        if world > 1:
            t = torch.tensor([el, float(dev_err)], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, dev_err = t[0].item(), int(t[1].item())
        dev_errors[0] |= dev_err
        if dev_err:
            raise SystemExit(f"bench: device error word 0x{dev_err:x} after a timed loop "
                             "(mignn_device_errors: an in-kernel bounded wait ran out): "
                             "results invalid")
        return el

    progress(f"headline workload ready: {N_local} nodes, {E_local} edges per GPU")
    elapsed = timed_loop(cache_graph=False, rec_into=launches)
    progress(f"headline: {1e3 * elapsed / max(args.steps, 1):.2f} ms per step")
    elapsed_cached = timed_loop(cache_graph=True)

    # ---- roofline of the fused GCN layer kernel (this rank's launches)
    deg_plus_self = E_local / N_local + 1.0
    traffic = None
    tf = os.path.join(HERE, "profiles", "gcn_layer_traffic.json")
    # (the PMC record is of the single-GPU launch over the whole mesh; at N > 1
    # a rank's launches cover its interior / boundary row ranges: no record)
    if os.path.exists(tf) and world == 1:
        try:
            with open(tf) as fh:
                tj = json.load(fh)
            if (tj.get("config") == f"{args.layer_type}_L{L}_H{H}_{nx}x{ny}x{nz}"
                    and tj.get("precision", "f16x3") == model.precision):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = None
    if args.layer_type == "GCN":
        route = model._gcn_kernel(H)
        if (world > 1 and route == "win" and model.gcn_kernel == "auto"
                and not (model._use_reorder(x) and model._column_order())):
            # (a shard's rows without the column order: FlowGNN._gcn_kernel's fallback)
            from mignn.gnn_model import GCN_BLOCK_ORDER
            route = GCN_BLOCK_ORDER.get(H, "pc")
        roofline = gcn_roofline(launches, H, deg_plus_self, model.precision, traffic, route)
        if roofline is not None and launches01:
            # layers 0 + 1 through the row codes (FlowGNN._gcn_layers01_codes):
            # the launches above are layers 2 .. L-1
            ms01 = sum(e0.elapsed_time(e1) for e0, e1, _ in launches01) / len(launches01)
            roofline["layers01_codes"] = {
                "kernels": "gcn_layer0_codes_kernel<3> + gcn_win_kernel<128, codes> "
                           "(mignn_gcn_layer0_codes + mignn_gcn_layer_win_codes)",
                "avg_ms": round(ms01, 4), "launches": len(launches01),
                "note": "layer 0 writes 32-B row codes, layer 1 expands the rows it "
                        "reads from them (DESIGN.md 3.16); the roofline above is "
                        "over layers 2 .. L-1"}

    exact = None
    if model.precision != "f32":
        model.precision = "f32"
        el32 = timed_loop(cache_graph=True, rec_into=launches32) if args.steps > 0 else 0.0
        model.precision = args.precision
        exact = {"ms_per_step_graph_cached": 1e3 * el32 / args.steps,
                 "value_graph_cached": L * E_local * world * args.steps / el32,
                 "roofline": (gcn_roofline(launches32, H, deg_plus_self, "f32", None)
                              if args.layer_type == "GCN" else None)}
    restore()

    E_total = E_local * world
    value = L * E_total * args.steps / elapsed
    line = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
        "graph_setup_in_step": True,
        "ms_per_step_graph_cached": 1e3 * elapsed_cached / args.steps,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "f16x3 (split fp32)" if model.precision == "f16x3" else "f32",
        "data": "synthetic",
        "arithmetic": ("f16x3: fp32 values split into fp16 hi+lo, 3 fp16 MFMA products, fp32 "
                       "accumulate (GCN transform, output head); gathers / norms / biases fp32; "
                       "max-abs error vs the fp32 CPU reference <= 1e-5 on the BFS mesh "
                       "(configs[0]/[1]); at synthetic sizes the tested bound is max(1e-5, 2x the "
                       "fp32 CPU oracle's own error vs fp64) (DESIGN.md section 5)")
                      if model.precision == "f16x3" else "exact fp32 (f32 MFMA / VALU)",
        "config": {
            "workload": f"{args.layer_type.lower()}_L{L}_H{H}_periodic_hex_{nx}x{ny}x{nz}_per_gpu"
                        + ("_shuffled" if args.shuffle else ""),
            "model": f"FlowGNN({args.layer_type}, layers={L}, hidden={H}, out=7), eval, "
                     "seeded random weights",
            "nodes_per_gpu": N_local, "edges_per_gpu": E_local, "global_batch": 1,
            "parallelism": "single" if world == 1 else f"node_range{world}+rccl_halo",
            "internal_node_order": (("locality: 8x8-cell columns, z inside "
                                     "(mignn_locality_order_cols, the window GCN kernel's order)"
                                     if model._column_order() else
                                     "locality: 4x4x4-cell blocks in panels of 4x4 block columns "
                                     "(mignn_locality_order)") + "; part of the per-step graph setup"
                                    if world == 1 else
                                    ("column order (window GCN kernel)" if model._column_order()
                                     else "block order") +
                                    " inside each rank's range, interior rows "
                                    "first; the partition layout (ghost / send lists, the "
                                    "order) and the rank-local CSR are rebuilt inside every "
                                    "timed step, as the N = 1 step rebuilds its CSR and order")
                                   if model._use_reorder(x) else "as given",
        },
        "roofline": roofline,
        "exact_f32": exact,
        "device_errors": dev_errors[0],
    }
    if world == 1 and args.layer_type == "GCN":
        line["aggregate_alone"] = aggregate_roofline(model, x, args.steps)
    if world > 1:
        dist.barrier()
    if not args.no_config4:
        # every rank takes part (the sharded forward exchanges halos)
        model._csr.entries.clear()
        shard_box = None
        torch.cuda.empty_cache()
        line["config4"] = config4_leg(dev, args, world, rank)
        progress(f"config4 leg: {line['config4']['ms_per_forward']} ms per forward")

    cpu_threads = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu_threads = cpu_thread_sweep(dev)
        progress(f"cpu thread sweep: {cpu_threads}")
    if rank == 0 and not args.no_bfs:
        line["bfs_mesh"] = bfs_leg(dev, cpu_threads)
    if rank == 0 and world == 1 and not args.no_legs:
        model._csr.entries.clear()
        del x
        ei = None
        torch.cuda.empty_cache()
        line["legs"] = {}
        for name in [v for v in args.legs.split(",") if v]:
            heavy = name in ("transformer", "gin")
            line["legs"][name] = eval_leg(name, dev, args.precision,
                                          steps=max(1, min(args.steps, 3 if heavy else 10)),
                                          warmup=1 if heavy else 2, cpu_threads=cpu_threads)
            progress(f"leg {name}: {line['legs'][name]['ms_per_forward']} ms per forward")
    if rank == 0 and world == 1 and not args.no_graph:
        line["graph_build"] = graph_build_leg(dev, nx, ny, nz, not args.no_cpu)
        progress("graph_build leg done")
    if rank == 0 and world == 1 and not args.no_train:
        line["train_step"] = train_leg(dev, args)
        progress("train_step leg done")
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_leg(model, sd, cfg, args, dev, cpu_threads)
        progress("cpu_baseline leg done")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def time_layers(model, recording, recording01=None):
    """Wrap model._layer with HIP events on the current stream (the stream the
    layer kernels are launched on); events go to recording[0] when it is a
    list -- and those of the codes form of layers 0 + 1
    (FlowGNN._gcn_layers01_codes) to recording01.  Returns the restore
    function."""
    orig_layer = model._layer
    orig01 = model._gcn_layers01_codes

    def timed01(csr, pos, n, out):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig01(csr, pos, n, out)
        e1.record()
        if recording[0] is not None and recording01 is not None:
            recording01.append((e0, e1, n))

    def timed_layer(i, layer, csr, xin, out, rb, re, **kw):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig_layer(i, layer, csr, xin, out, rb, re, **kw)
        e1.record()
        if recording[0] is not None:
            recording[0].append((e0, e1, re - rb))

    model._layer = timed_layer
    model._gcn_layers01_codes = timed01

    def restore():
        model._layer = orig_layer
        model._gcn_layers01_codes = orig01
    return restore


def aggregate_roofline(model, x, steps):
    """SURVEY 8(d) target (i): the GCN aggregate kernel alone (out = D^-1/2
    (A + I) D^-1/2 x, fp32, CSR order) at H = 128 and 64 over the bench graph,
    HIP events on the launch stream; algorithmic bytes as the layer's: read x
    and write the output once, the CSR arrays once.  The window kernel
    (mignn_gcn_aggregate_win) over the graph's CSR in the column order and the
    ring kernel (mignn_gcn_aggregate_ring) over the block order are timed;
    the faster is the entry, the other beside it."""
    from mignn import _lib
    from mignn.gnn_model import _CsrCache
    csr = None
    for c in model._csr.entries.values():
        csr = c
    if csr is None or csr.pos is None or csr.key_tensor is None:
        return None
    n = csr.num_nodes
    nnz = int(csr.row_ptr[-1].item())
    if csr.order_info is not None:
        ccsr, bcsr = csr, _CsrCache._build(csr.key_tensor, n, _lib.CSR_ONE_SELF_LOOP, csr.pos, cols=False)
    else:
        ccsr, bcsr = _CsrCache._build(csr.key_tensor, n, _lib.CSR_ONE_SELF_LOOP, csr.pos, cols=True), csr
    L = _lib.lib()
    P = _lib.ptr
    st = _lib.stream(x.device)
    k = max(5, min(steps, 20))
    res = {}
    for H in (128, 64):
        X = torch.randn((n, H), device=x.device,
                        generator=torch.Generator(device=x.device).manual_seed(3))
        Y = torch.empty_like(X)
        rplan = bcsr.ring_plan(H, 0, n)
        wplan = ccsr.win_plan(H, 0, n)
        runs = {
            "win": ("%s<32> (mignn_gcn_aggregate_win)" % ("gcn_win64_kernel" if H == 64 else
                                                           "gcn_win_kernel<128>"),
                    lambda: _lib.check(L.mignn_gcn_aggregate_win(
                        P(wplan), P(ccsr.row_ptr), P(ccsr.col), P(ccsr.ew), P(X), H, 0, n, H, P(Y), H,
                        st), "mignn_gcn_aggregate_win")),
            "ring": ("gcn_ring_kernel<%d, aggregate> (mignn_gcn_aggregate_ring)" % H,
                     lambda: _lib.check(L.mignn_gcn_aggregate_ring(
                         P(rplan), P(bcsr.row_ptr), P(bcsr.col), P(bcsr.ew), P(X), H, 0, n, H, P(Y), H,
                         st), "mignn_gcn_aggregate_ring")),
        }
        by = 4 * (2 * n * H + (n + 1) + nnz + n)
        out = {}
        for name, (kname, run) in runs.items():
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(k):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / k
            out[name] = {"kernel": kname, "bound": "hbm",
                         "achieved": round(by / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(by / (ms * 1e-3) / HBM_PEAK, 4),
                         "traffic": None, "avg_launch_ms": round(ms, 4), "launches": k,
                         "algorithmic_bytes_per_launch": by}
        first = min(out, key=lambda kk: out[kk]["avg_launch_ms"])
        best = dict(out[first])
        best.update({"H": H, "rows": n, "csr_entries": nnz,
                     "others": {kk: v for kk, v in out.items() if kk != first}})
        res[f"H{H}"] = best
        del X, Y
    del ccsr, bcsr
    return res


GCN_KERNEL_NAMES = {"pc": "gcn_f16x3_kernel<%d> (mignn_gcn_layer_f16x3)",
                    "ring": "gcn_ring_kernel<%d> (mignn_gcn_layer_ring)",
                    "win": "gcn_win_kernel<%d> / gcn_win64_kernel at H = 64 (mignn_gcn_layer_win)"}


def gcn_roofline(launches, H, deg_plus_self, precision, traffic, route="pc"):
    """Roofline of the fused GCN layer kernel from its timed launches."""
    if not launches:
        return None
    tot_ms = sum(e0.elapsed_time(e1) for e0, e1, _ in launches)
    n_rows = sum(n for _, _, n in launches)
    tot_bytes = layer_bytes(n_rows, n_rows * deg_plus_self, H, gcn=True)
    tot_flops = layer_flops("GCN", n_rows, n_rows * deg_plus_self, H)
    t_s = tot_ms / 1e3
    gbs = tot_bytes / t_s
    t_hbm = tot_bytes / HBM_PEAK
    if precision == "f16x3":
        # 3 fp16 MFMA products per fp32 product on the transform; the
        # gather-aggregate FMAs on the fp32 VALU
        t_comp = (3 * 2 * n_rows * H * H / F16_MFMA_PEAK
                  + 2 * n_rows * deg_plus_self * H / F32_MFMA_PEAK)
        kname = GCN_KERNEL_NAMES[route] % H
        comp_peak, comp_note = F16_MFMA_PEAK, "f16 MFMA x3 (split fp32) + f32 VALU aggregate"
    else:
        t_comp = tot_flops / F32_MFMA_PEAK
        kname = "fused_tile_kernel<%d, %d, 0, true> (mignn_gcn_layer)" % (H, H)
        comp_peak, comp_note = F32_MFMA_PEAK, "f32 MFMA"
    bound_hbm = t_hbm >= t_comp
    t_bound = max(t_hbm, t_comp)
    nl = len(launches)
    return {
        "kernel": kname,
        "bound": "hbm" if bound_hbm else "mfma",
        "achieved": round((gbs / 1e9) if bound_hbm else (tot_flops / t_s / 1e12), 3),
        "peak": round((HBM_PEAK / 1e9) if bound_hbm else (comp_peak / 1e12), 1),
        "unit": "GB/s" if bound_hbm else "TFLOP/s",
        "frac": round(t_bound / t_s, 4),
        "traffic": traffic,
        "avg_launch_ms": round(tot_ms / nl, 4),
        "launches": nl,
        "algorithmic_bytes_per_launch": int(tot_bytes / nl),
        "algorithmic_flops_per_launch": int(tot_flops / nl),
        "hbm_side": {"achieved_GBps": round(gbs / 1e9, 1), "peak_GBps": HBM_PEAK / 1e9,
                     "frac": round(gbs / HBM_PEAK, 4), "t_min_ms": round(1e3 * t_hbm / nl, 4)},
        "compute_side": {"model": comp_note, "t_min_ms": round(1e3 * t_comp / nl, 4),
                         "frac": round(t_comp / t_s, 4)},
    }


LEGS = {
    # name: (layer_type, hidden, layers, grid, shuffle, graph setup inside the step)
    "gcn_h64": ("GCN", 64, 4, (250, 200, 200), None, True),
    "shuffled": ("GCN", 128, 4, (250, 200, 200), 0, True),
    "gat": ("GAT", 128, 4, (100, 100, 100), None, False),
    "transformer": ("Transformer", 256, 6, (250, 200, 200), None, False),
    "gin": ("GIN", 256, 8, (500, 400, 63), None, False),
}
LEG_CONFIG = {"gcn_h64": "SURVEY 8d H=64 HBM-target layer", "shuffled": "configs[1] model, shuffled order",
              "gat": "configs[2]", "transformer": "configs[3]",
              "gin": "configs[4] model, one GPU's shard of the 100M mesh"}
# bounded CPU samples of each leg's model (a few seconds of oracle work each,
# timed on a smaller mesh than the leg's: the CPU rate is not size-independent
# -- the headline's 10M-node CPU forward runs at ~0.7x its 1M-node rate -- so
# each leg's cpu_baseline names its sample size)
LEG_CPU_SAMPLE = {"gcn_h64": (100, 100, 100), "shuffled": (80, 80, 80), "gat": (60, 60, 60),
                  "transformer": (40, 40, 32), "gin": (50, 50, 40)}


def cpu_thread_sweep(dev):
    """The torch-CPU thread count used for every CPU baseline: the fastest of
    a sweep up to this process's CPU affinity (torch's CPU kernels ran 3.6x
    slower on all 256 hardware threads of the 2-socket host than on 32)."""
    from oracle import flowgnn_oracle as orc
    from mignn import FlowGNN
    from mignn.synthetic import grid_graph, seeded_state_dict
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    avail = max(1, avail or 1)
    cfg = dict(hidden_dim=128, num_layers=4, layer_type="GCN")
    sd = seeded_state_dict(FlowGNN(input_dim=3, output_dim=7, **cfg).state_dict(), seed=0)
    xs, eis = (t.cpu() for t in grid_graph(40, 40, 40, device=dev))
    sweep = {}
    for nt in sorted({c for c in (8, 16, 32, 64, 128, avail) if c <= avail}):
        torch.set_num_threads(nt)
        orc.flowgnn_forward(sd, cfg, xs, eis, None, dtype=torch.float32)
        t0 = time.perf_counter()
        orc.flowgnn_forward(sd, cfg, xs, eis, None, dtype=torch.float32)
        sweep[nt] = round(time.perf_counter() - t0, 4)
    threads = min(sweep, key=sweep.get)
    return {"threads": threads, "cpus_available": avail, "os_cpu_count": os.cpu_count(),
            "sweep_s_40x40x40": sweep}


def cpu_time_model(sd, cfg, x, ei, cpu_threads, reps=1):
    """Median seconds of the torch-CPU oracle forward (fp32) on (x, ei)."""
    from oracle import flowgnn_oracle as orc
    torch.set_num_threads(cpu_threads["threads"])
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float32)
        times.append(time.perf_counter() - t0)
    return statistics.median(times)


def eval_leg(name, dev, precision, steps, warmup, cpu_threads=None):
    """One other-config forward (see the docstring): ms per forward, edges/s,
    per-layer roofline."""
    from mignn import FlowGNN
    from mignn.synthetic import grid_graph, seeded_state_dict
    lt, H, L, dims, shuffle, setup_in_step = LEGS[name]
    cfg = dict(hidden_dim=H, num_layers=L, layer_type=lt)
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    model.precision = precision
    x, ei = grid_graph(*dims, device=dev, permute_seed=shuffle)
    N, E = x.shape[0], ei.shape[1]
    rec = [None]
    launches = []
    restore = time_layers(model, rec)
    model._csr.capacity = 0 if setup_in_step else 4
    with torch.no_grad():
        for _ in range(warmup):
            model(x, ei)
        torch.cuda.synchronize()
        rec[0] = launches
        t0 = time.perf_counter()
        for _ in range(steps):
            model(x, ei)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rec[0] = None
    restore()
    e_rows = E + N if lt in ("GCN", "GAT") else E
    out = {"config": LEG_CONFIG[name],
           "workload": f"{lt.lower()}_L{L}_H{H}_periodic_hex_{dims[0]}x{dims[1]}x{dims[2]}"
                       + ("_shuffled" if shuffle is not None else ""),
           "nodes": N, "edges": E, "graph_setup_in_step": setup_in_step,
           "ms_per_forward": round(1e3 * el / steps, 3), "edges_per_s": L * E * steps / el}
    if lt == "GCN" and H in (64, 128):
        out["roofline"] = gcn_roofline(launches, H, e_rows / N, precision, None,
                                       model._gcn_kernel(H))
    else:
        tot_ms = sum(e0.elapsed_time(e1) for e0, e1, _ in launches)
        n_rows = sum(n for _, _, n in launches)
        fl = layer_flops(lt, n_rows, n_rows * e_rows / N, H)
        by = layer_bytes(n_rows, n_rows * e_rows / N, H, gcn=lt == "GCN")
        t_s = tot_ms / 1e3
        g = gemm_flops(lt, n_rows, H)
        if precision == "f16x3":
            # the FlowGNN.precision "f16x3" GEMMs (every K or N > 128 transform:
            # all of H = 256, GAT's head-mean GEMM): 3 f16 MFMAs per fp32
            # product; the aggregation on the f32 VALU
            t_comp = 3 * g / F16_MFMA_PEAK + (fl - g) / F32_MFMA_PEAK
            arith = ("split-fp16 GEMMs (3 f16 MFMA per fp32 product, 2.5 PF) + f32 VALU "
                     "aggregation (157 TF)")
        else:
            t_comp = fl / F32_MFMA_PEAK
            arith = "exact fp32 (f32 MFMA GEMMs, f32 VALU aggregation)"
        t_hbm = by / HBM_PEAK
        nl = len(launches)
        mfma = t_comp >= t_hbm
        out["roofline"] = {
            "unit_of_timing": "one layer (all its launches: aggregation + MFMA GEMMs), HIP events",
            "bound": "mfma" if mfma else "hbm",
            "achieved": round(fl / t_s / 1e12, 3) if mfma else round(by / t_s / 1e9, 1),
            # effective compute peak of this layer's flop mix (fp32-equivalent
            # flops / t_comp) or HBM peak
            "peak": round(fl / t_comp / 1e12, 1) if mfma else HBM_PEAK / 1e9,
            "unit": "TFLOP/s" if mfma else "GB/s",
            "frac": round(max(t_comp, t_hbm) / t_s, 4),
            "avg_layer_ms": round(tot_ms / nl, 3), "layers_timed": nl,
            "t_min_ms": {"compute": round(1e3 * t_comp / nl, 3), "hbm": round(1e3 * t_hbm / nl, 3)},
            "executed_flops_per_layer": int(fl / nl),
            "gemm_flops_per_layer": int(g / nl),
            "reference_formulation_flops_per_layer": int(
                (26 * N * H * H + 16 * E * H) if lt == "Transformer" else fl / nl),
            "algorithmic_bytes_per_layer": int(by / nl),
            "arithmetic": arith,
        }
    del model, x, ei
    torch.cuda.empty_cache()
    if cpu_threads is not None:
        cdims = LEG_CPU_SAMPLE[name]
        xc, eic = (t.cpu() for t in grid_graph(*cdims, device=dev, permute_seed=shuffle))
        tc = cpu_time_model(sd, cfg, xc, eic, cpu_threads)
        out["cpu_baseline"] = {
            "value": L * eic.shape[1] / tc, "unit": "edges/s", "cores": cpu_threads["threads"],
            "kind": "port", "s_per_forward": round(tc, 3),
            "sample": f"{lt} L{L} H{H} forward on the {cdims[0]}x{cdims[1]}x{cdims[2]} periodic "
                      f"mesh ({xc.shape[0]} nodes, {eic.shape[1]} edges"
                      + (", shuffled" if shuffle is not None else "") + "), torch-CPU oracle "
                      "fp32, one timed run on this bounded sample (not the leg's full size)",
            "gpu_over_cpu": round(out["edges_per_s"] / (L * eic.shape[1] / tc), 1)}
    return out


def config4_leg(dev, args, world, rank):
    """BASELINE configs[4] at the bench's N: GIN L8 H256 on the 500 x 400 x
    (63 N) periodic mesh (100.8M nodes at N = 8), k-slab node ranges, one
    FlowGNNShard per rank (mignn.dist: layer 0 composed with input_proj from
    the exchanged ghost coordinates, an RCCL halo of one 200k-node plane per
    side for each later layer, interior rows overlapping it).  The same code
    runs at N = 1 (one shard, no ghosts), so the N = 1, 2, 4, 8 lines are one
    curve.  The partition and rank-local CSR are built once, outside the
    timed loop (steady state on a fixed mesh, as the other legs);
    edges/s = L * E_total * K / t, t = max over ranks."""
    from mignn import FlowGNN
    from mignn.dist import (DistExchange, DistRequests, FlowGNNShard, LocalExchange, RangeLayout,
                            build_local_layouts, sharded_forward)
    from mignn.gnn_model import locality_order
    from mignn.synthetic import grid_graph, seeded_state_dict
    nx, ny, nz = 500, 400, 63
    L, H = 8, 256
    cfg = dict(hidden_dim=H, num_layers=L, layer_type="GIN")
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    model.load_state_dict(seeded_state_dict(model.state_dict(), seed=0))
    model = model.to(dev).eval()
    model.precision = args.precision
    x, ei = grid_graph(nx, ny, nz * world, device=dev, z_begin=rank * nz, z_count=nz)
    n_loc, e_loc = x.shape[0], ei.shape[1]
    bounds = [r * n_loc for r in range(world + 1)]
    order = (lambda p, e: locality_order(p, e)[0]) if model._use_reorder(x) else None
    t_setup = time.perf_counter()
    if world == 1:
        (lay,) = build_local_layouts([ei], bounds, pos=[x], order_fn=order)
        exch = LocalExchange()
    else:
        lay = RangeLayout(ei, bounds, rank, DistRequests(), pos=x, order_fn=order)
        exch = DistExchange()
    sh = FlowGNNShard(model, lay, x)
    sh.setup(exch, [sh])
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup
    del ei
    steps = max(1, min(args.steps, 3))
    with torch.no_grad():
        for _ in range(1 if args.warmup > 0 else 0):
            sharded_forward([sh], exch, [x])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            sharded_forward([sh], exch, [x])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    from mignn import _lib
    dev_err = _lib.device_errors(clear=True)
    if world > 1:
        t = torch.tensor([el, float(dev_err)], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, dev_err = t[0].item(), int(t[1].item())
    if dev_err:
        raise SystemExit(f"bench: device error word 0x{dev_err:x} after the config4 timed loop")
    out = {"config": "configs[4]: GIN L8 H256, 100.8M nodes at N = 8 (12.6M per GPU)",
           "workload": f"gin_L{L}_H{H}_periodic_hex_{nx}x{ny}x{nz}_per_gpu",
           "n_gpus": world, "nodes": n_loc * world, "edges": e_loc * world,
           "parallelism": "single shard" if world == 1 else f"node_range{world}+rccl_halo",
           "ghost_rows_per_gpu": lay.n_ghost, "interior_rows_per_gpu": lay.n_int,
           "layer0": model._layer0_kind() or "input_proj + layer 0",
           "graph_setup_in_step": False, "setup_s_rank0": round(t_setup, 2),
           "steps": steps, "ms_per_forward": round(1e3 * el / steps, 3),
           "edges_per_s": L * e_loc * world * steps / el, "scaling": "weak"}
    del sh, lay, x, model
    torch.cuda.empty_cache()
    return out


def bfs_leg(dev, cpu_threads=None):
    """configs[1]: 4-layer GCN H=128 on the reference-built BFS mesh vs the
    committed reference-CPU output."""
    import numpy as np
    from mignn import FlowGNN

    g = np.load(os.path.join(HERE, "tests", "golden", "bfs_graphs.npz"))
    m = np.load(os.path.join(HERE, "tests", "golden", "models.npz"))
    from mignn.synthetic import seeded_state_dict_from_layout
    name = "c2_gcn_h128_l4"
    cfg = json.loads(str(m[f"{name}/cfg"]))
    sd = seeded_state_dict_from_layout(str(m[f"{name}/sd_layout"]), int(m[f"{name}/seed"]),
                                       str(m[f"{name}/sd_sha256"]))
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
    # field space: the reference's float64 denormalisation (inference.py:76-85
    # -> FieldNormalizer.inverse_transform, normalization.py:111-133) of both
    # outputs, with the scalers FieldNormalizer.fit produced on the case
    # (tests/golden/normalizer.json); ours through the engine's device path
    import numpy as np
    from mignn.normalization import FieldNormalizer
    with open(os.path.join(HERE, "tests", "golden", "normalizer.json")) as fh:
        js = json.load(fh)
    norm = FieldNormalizer()
    norm.scalers = {k: {"mean": np.asarray(v["mean"], dtype=np.float64) if v["per_component"]
                        else np.float64(v["mean"]),
                        "std": np.asarray(v["std"], dtype=np.float64) if v["per_component"]
                        else np.float64(v["std"]),
                        "per_component": v["per_component"]} for k, v in js.items()}
    ours = {k: v.cpu().numpy() for k, v in norm.inverse_transform(model.predict_fields(y)).items()}
    refs = {}
    for k, v in model.predict_fields(y32).items():          # numpy float64, as the reference
        sc = js[k]
        refs[k] = v.numpy() * np.asarray(sc["std"], dtype=np.float64) + np.asarray(sc["mean"], dtype=np.float64)
    fields = {}
    for k in refs:
        d = np.abs(np.asarray(ours[k], dtype=np.float64) - refs[k])
        fields[k] = {"mae": float(d.mean()), "max_abs": float(d.max()),
                     "field_std": float(np.std(refs[k])),
                     "max_abs_over_field_std": float(d.max() / max(np.std(refs[k]), 1e-300))}
    cpu = None
    if cpu_threads is not None:
        # the reference's own inference size (inference.py:73): the whole mesh
        tc = cpu_time_model(sd, cfg, x.cpu(), ei.cpu(), cpu_threads, reps=3)
        cpu = {"value": cfg["num_layers"] * ei.shape[1] / tc, "unit": "edges/s",
               "cores": cpu_threads["threads"], "kind": "port", "s_per_forward": round(tc, 4),
               "sample": "the whole train-path BFS mesh, torch-CPU oracle fp32, median of 3"}
    return {"config": "configs[1]: GCN L4 H128, train-path BFS mesh",
            "cpu_baseline": cpu,
            "nodes": int(x.shape[0]), "edges": int(ei.shape[1]),
            "ms_per_forward": round(t * 1e3, 4),
            "edges_per_s": cfg["num_layers"] * ei.shape[1] / t,
            "max_abs_err_vs_ref_cpu": err.max().item(), "mae_vs_ref_cpu": err.mean().item(),
            "denormalized_fields_vs_ref_cpu": fields}


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


def cpu_leg(model, sd, cfg, args, dev, cpu_threads):
    """The CPU oracle on the headline workload itself (args.grid, one timed
    forward: ~80 s on 32 host threads at 10M nodes) and, beside it, on a
    1M-node sample (median of 2 after a warm-up, with the accuracy of both
    fp32 paths against fp64 there)."""
    from oracle import flowgnn_oracle as orc
    from mignn.synthetic import grid_graph

    threads = cpu_threads["threads"]
    avail = cpu_threads["cpus_available"]
    sweep = cpu_threads["sweep_s_40x40x40"]
    torch.set_num_threads(threads)
    full = None
    if not args.cpu_sample_only:
        nx, ny, nz = (int(v) for v in args.grid.split(","))
        xf, eif = (t.cpu() for t in grid_graph(nx, ny, nz, device=dev))
        progress(f"cpu baseline: the headline forward on {xf.shape[0]} nodes (one timed run)")
        t0 = time.perf_counter()
        with torch.no_grad():
            orc.flowgnn_forward(sd, cfg, xf, eif, None, dtype=torch.float32)
        tf = time.perf_counter() - t0
        full = {"value": cfg["num_layers"] * eif.shape[1] / tf, "s_per_forward": round(tf, 3),
                "nodes": int(xf.shape[0]), "edges": int(eif.shape[1])}
        del xf, eif
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
    # accuracy on the same 1M-node sample: both fp32 paths against the fp64
    # oracle (the GPU-vs-fp32-CPU difference alone mixes both rounding errors)
    y64 = orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float64)
    acc = {"gpu_vs_fp64_max_abs_err": (yg.double() - y64).abs().max().item(),
           "cpu_fp32_vs_fp64_max_abs_err": (y.double() - y64).abs().max().item(),
           "gpu_vs_cpu_fp32_max_abs_err": (yg - y).abs().max().item(),
           "output_max_abs": y64.abs().max().item()}
    cpu_model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    sample_1m = {"value": cfg["num_layers"] * ei.shape[1] / t, "s_per_forward": round(t, 3),
                 "sample": f"{cx}x{cy}x{cz} periodic mesh ({x.shape[0]} nodes, {ei.shape[1]} "
                           f"edges), median of 2 after 1 warm-up",
                 "accuracy": acc}
    wl = (f"{cfg['layer_type']} L{cfg['num_layers']} H{cfg['hidden_dim']} forward, torch-CPU oracle "
          f"fp32 (the reference forward's op pattern), {threads} threads")
    if full is not None:
        value, s_fwd = full["value"], full["s_per_forward"]
        sample = (f"{wl}, on the headline mesh itself ({args.grid.replace(',', 'x')}: "
                  f"{full['nodes']} nodes, {full['edges']} edges), one timed forward in this run "
                  f"(after the thread sweep's warm-up)")
    else:
        value, s_fwd = sample_1m["value"], sample_1m["s_per_forward"]
        sample = f"{wl}, on the {cx}x{cy}x{cz} sample only (--cpu-sample-only)"
    return {"value": value, "unit": "edges/s", "cores": threads,
            "os_cpu_count": os.cpu_count(), "cpus_available": avail,
            "thread_sweep_s_40x40x40": sweep,
            "kind": "port", "sample": sample, "s_per_forward": s_fwd, "cpu_model": cpu_model,
            "sample_1M": sample_1m, "accuracy_1M": acc,
            "full_size": cpu_full_record()}


def cpu_full_record():
    """The same oracle timed at the configurations' own sizes (10M headline,
    >= 0.5M for the legs; scripts/cpu_full.py, a separate run on a GPU box's
    host, committed under profiles/): too long for the default bench run."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_cpu_full.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as fh:
            rec = json.load(fh)
    except (OSError, ValueError):
        return None
    return {"file": os.path.relpath(files[-1], HERE),
            "runs": {k: {"workload": v["workload"], "edges_per_s": v["edges_per_s"],
                         "median_s": v["median_s"], "timed_runs": v["timed_runs"],
                         "cores": v["cores"]} for k, v in rec.get("runs", {}).items()}}


if __name__ == "__main__":
    main()
