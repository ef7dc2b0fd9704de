"""Hot-kernel timing (round 4): the tile-plan GCN layer (mignn_gcn_layer_planned),
its aggregate alone (mignn_gcn_aggregate_planned) and the plan build against
the producer / consumer kernel (mignn_gcn_layer_f16x3) on the bench mesh
(250x200x200 periodic hex, 10M nodes, locality order), HIP events on the
launch stream, interleaved rounds, median.  Env: TB_H (comma list, 128,64),
TB_GRID, TB_REPS.  Prints one JSON object."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
nx, ny, nz = (int(v) for v in os.environ.get("TB_GRID", "250,200,200").split(","))
pos, ei = grid_graph(nx, ny, nz, device=dev)
n = pos.shape[0]
perm, inv = locality_order(pos, ei)
csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
del ei
nnz = int(csr.row_ptr[-1].item())
L = _lib.diag_lib()
P = _lib.ptr
st = _lib.stream()
reps = int(os.environ.get("TB_REPS", "7"))
res = {"grid": [nx, ny, nz], "n": n, "nnz": nnz, "by_h": {}}


def timed(cases):
    times = {k: [] for k in cases}
    for rnd in range(reps + 1):
        for k, f in cases.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            e1.synchronize()
            if rnd > 0:
                times[k].append(e0.elapsed_time(e1) / 3)
    return {k: round(statistics.median(v), 4) for k, v in times.items()}


for H in [int(v) for v in os.environ.get("TB_H", "128,64").split(",")]:
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, H, device=dev, generator=g)
    W = torch.randn(H, H, device=dev, generator=g) * 0.05
    b = torch.randn(H, device=dev, generator=g) * 0.05
    sc = torch.rand(H, device=dev, generator=g) + 0.5
    sh = torch.randn(H, device=dev, generator=g) * 0.1
    nb = L.mignn_gcn_plan_bytes(0, n)
    plan = torch.empty(nb, dtype=torch.uint8, device=dev)
    Y = torch.empty_like(X)
    Y0 = torch.empty_like(X)

    def mk_plan():
        _lib.check(L.mignn_gcn_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), 0, n, H, P(plan), nb, st),
                   "plan")

    def planned():
        _lib.check(L.mignn_gcn_layer_planned(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                             0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H, st),
                   "planned")

    def agg():
        _lib.check(L.mignn_gcn_aggregate_planned(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew),
                                                 P(X), H, 0, n, H, P(Y), H, st), "agg")

    def pc():
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                           P(W), P(b), P(sc), P(sh), 15, P(Y0), H, st), "pc")

    nbr = L.mignn_gcn_ring_plan_bytes(0, n, H)
    rplan = torch.empty(nbr, dtype=torch.uint8, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    Yr = torch.empty_like(X)

    def mk_rplan(st_=None):
        _lib.check(L.mignn_gcn_ring_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), 0, n, H, P(rplan),
                                         nbr, st_, st), "rplan")

    def ring():
        _lib.check(L.mignn_gcn_layer_ring(P(rplan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                          0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yr), H, st),
                   "ring")

    mk_rplan(P(stats))
    ring()
    torch.cuda.synchronize()
    res.setdefault("ring_plan_stats", {})[H] = stats.tolist()
    Ya = torch.empty_like(X)

    def ring_agg():
        _lib.check(L.mignn_gcn_aggregate_ring(P(rplan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X),
                                              H, 0, n, H, P(Ya), H, st), "ring_agg")

    cases = {"plan": mk_plan, "planned": planned, "aggregate": agg, "pc_f16x3": pc,
             "ring_plan": mk_rplan, "ring": ring, "ring_aggregate": ring_agg}
    for m in [int(v) for v in os.environ.get("TB_RING_MODES", "").split(",") if v]:
        def fr(m=m):
            _lib.check(L.mignn_diag_ring(m, P(rplan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                         0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y0), H, st), "dring")
        cases[f"ring_mode{m}"] = fr
    if H == 128:
        for m in [int(v) for v in os.environ.get("TB_MODES", "").split(",") if v]:
            for a in (0, 1):
                if a == 0 and m & 8:
                    continue

                def f(m=m, a=a):
                    _lib.check(L.mignn_diag_gcn_tile(m, a, P(plan), P(csr.row_ptr), P(csr.col),
                                                     P(csr.ew), P(X), H, 0, n, H, P(W), P(b), P(sc),
                                                     P(sh), 15, P(Y0), H, st), "diag")
                cases[f"{'agg' if a else 'layer'}_mode{m}"] = f
    mk_plan()
    planned()
    pc()
    torch.cuda.synchronize()
    # variants that keep the arithmetic (mode 16: direct-store epilogue) must
    # write the product ring kernel's bits
    for m in [int(v) for v in os.environ.get("TB_RING_MODES", "").split(",") if v]:
        if m & 15 == 0 and not m & 32:
            ring()
            cases[f"ring_mode{m}"]()
            torch.cuda.synchronize()
            res.setdefault("ring_mode_bitwise_equal", {})[f"{H}_{m}"] = bool(torch.equal(Y0, Yr))
    pc()
    torch.cuda.synchronize()
    diff = (Y - Y0).abs().max().item()
    agg()
    ring_agg()
    torch.cuda.synchronize()
    res.setdefault("ring_aggregate_vs_planned_max_diff", {})[H] = (Ya - Y).abs().max().item()
    planned()
    torch.cuda.synchronize()
    res.setdefault("ring_vs_pc_max_diff", {})[H] = (Yr - Y0).abs().max().item()
    same = (Y == Y0).all(1).float().mean().item()
    ms = timed(cases)
    by = 4 * (2 * n * H + (n + 1) + nnz + n)     # algorithmic bytes of the layer
    by_agg = 4 * (2 * n * H + (n + 1) + nnz + n)
    res["by_h"][H] = {"ms": ms, "max_diff_vs_pc": diff, "bitwise_equal_rows_vs_pc": same,
                      "frac_of_8TBps": {k: round((by_agg if "aggregate" in k else by) / (v * 1e-3) / 8e12, 4)
                                        for k, v in ms.items() if "plan" not in k}}
    print(json.dumps({H: res["by_h"][H]}), file=sys.stderr, flush=True)
    del X, Y, Y0, plan
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
