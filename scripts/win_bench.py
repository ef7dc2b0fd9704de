"""Hot-kernel timing (round 5): the window GCN layer (mignn_gcn_layer_win, the
column order) against the producer / consumer kernel (mignn_gcn_layer_f16x3)
and the ring kernel (mignn_gcn_layer_ring), both in the block order, on the
bench mesh (250x200x200 periodic hex, 10M nodes); the aggregate alone of the
window and ring kernels; the window plan build; window ablations
(mignn_diag_win modes: 1 ext rows from the zero row, 2 own rows from it, 3 both, 4 no MFMAs, 33
aggregate with ext from the zero row).  HIP events on the launch stream,
interleaved rounds, median.  Env: WB_H (comma list, 128,64), WB_GRID,
WB_REPS, WB_MODES (comma list of diag modes), WB_OLD (0: skip pc / ring),
WB_LIBS (name=path,...: variant builds timed beside the product).
Prints one JSON object."""
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
nx, ny, nz = (int(v) for v in os.environ.get("WB_GRID", "250,200,200").split(","))
pos, ei = grid_graph(nx, ny, nz, device=dev)
n = pos.shape[0]
old = os.environ.get("WB_OLD", "1") != "0"
perm_c, inv_c, info = locality_order(pos, ei, cols=True)
csr_c = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv_c)
csr_b = None
if old:
    _, inv_b = locality_order(pos, ei)
    csr_b = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv_b)
pos_c = pos[perm_c].contiguous()          # coordinates in the column order (layer-0 codes)
del ei, pos
nnz = int(csr_c.row_ptr[-1].item())
# the product entry points from the product library (the diag build carries
# bounds checks and trace branches: slower); the ablation modes from the
# diag library
LP = _lib.lib()
L = _lib.diag_lib()
P = _lib.ptr
# WB_LIBS: comma list of variant builds of libmignn.so (name=path); each
# gets its own "win@name" timing at every H
VARIANTS = {}
for item in [v for v in os.environ.get("WB_LIBS", "").split(",") if v]:
    name, path = item.split("=")
    VARIANTS[name] = _lib._load(path, _lib.SIGNATURES)
st = _lib.stream()
reps = int(os.environ.get("WB_REPS", "7"))
res = {"grid": [nx, ny, nz], "n": n, "nnz": nnz, "order_info": info.tolist(), "by_h": {}}


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


for H in [int(v) for v in os.environ.get("WB_H", "128,64").split(",")]:
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, H, device=dev, generator=g)
    W = torch.randn(H, H, device=dev, generator=g) * 0.05
    b = torch.randn(H, device=dev, generator=g) * 0.05
    sc = torch.rand(H, device=dev, generator=g) + 0.5
    sh = torch.randn(H, device=dev, generator=g) * 0.1
    nbw = LP.mignn_gcn_win_plan_bytes(0, n, H)
    wplan = torch.empty(nbw, dtype=torch.uint8, device=dev)
    wstats = torch.zeros(4, dtype=torch.int64, device=dev)
    Yw, Ywa, Yd = torch.empty_like(X), torch.empty_like(X), torch.empty_like(X)

    def mk_wplan(s_=None):
        _lib.check(LP.mignn_gcn_win_plan(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), 0, n, H, P(info),
                                        P(wplan), nbw, s_, st), "wplan")

    def win():
        _lib.check(LP.mignn_gcn_layer_win(P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X),
                                         H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yw), H, st), "win")

    def win_agg():
        _lib.check(LP.mignn_gcn_aggregate_win(P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew),
                                             P(X), H, 0, n, H, P(Ywa), H, st), "win_agg")

    mk_wplan(P(wstats))
    torch.cuda.synchronize()
    hdr = wplan[:64].cpu()
    res.setdefault("win_plan_stats", {})[H] = wstats.tolist()
    res.setdefault("win_header", {})[H] = hdr[:32].view(torch.int32).tolist() + hdr[32:64].view(torch.int64).tolist()
    cases = {"win_plan": mk_wplan, "win": win, "win_aggregate": win_agg}
    codes = xcoef = None
    if H == 128:
        # the codes form (layer 1 from layer 0's row codes: the headline's layer 1)
        codes = torch.zeros((n, 8), dtype=torch.float32, device=dev)
        xcoef = (torch.randn(H, 8, device=dev, generator=g) * 0.5).contiguous()
        _lib.check(LP.mignn_gcn_layer0_codes(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(pos_c), 3, 3,
                                             0, n, P(codes), 8, st), "codes")
        Ywc = torch.empty_like(X)

        def win_codes(VL=LP, pl=wplan, Yo=Ywc):
            # layers 0 + 1 as the model runs them: the codes written just
            # before the codes form reads them (MALL-resident, as in the
            # forward -- codes left in HBM by other kernels time differently)
            _lib.check(VL.mignn_gcn_layer0_codes(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(pos_c),
                                                 3, 3, 0, n, P(codes), 8, st), "codes")
            _lib.check(VL.mignn_gcn_layer_win_codes(P(pl), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew),
                                                    P(codes), 8, 0, n, H, P(xcoef), P(W), P(b), P(sc),
                                                    P(sh), 15, P(Yo), H, st), "win_codes")
        cases["win_layers01_codes"] = win_codes
    vout, vchecks = {}, {}
    for vname, VL in VARIANTS.items():
        # each variant builds its own plan (plan formats may differ)
        vnb = VL.mignn_gcn_win_plan_bytes(0, n, H)
        vplan = torch.empty(vnb, dtype=torch.uint8, device=dev)
        vst = torch.zeros(4, dtype=torch.int64, device=dev)
        _lib.check(VL.mignn_gcn_win_plan(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), 0, n, H, P(info),
                                         P(vplan), vnb, P(vst), st), "vplan")
        torch.cuda.synchronize()
        res.setdefault("variant_plan", {}).setdefault(H, {})[vname] = {"bytes": vnb, "stats": vst.tolist()}
        Yv, Yva = torch.empty_like(X), torch.empty_like(X)
        Yvc = torch.empty_like(X) if codes is not None else None
        vout[vname] = (Yv, Yva, Yvc)

        def fv(VL=VL, vplan=vplan, Yv=Yw):
            # (timed into the product's output buffer: same pages for every variant)
            _lib.check(VL.mignn_gcn_layer_win(P(vplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X),
                                              H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yv), H, st), "wv")
        def vcheck(VL=VL, vplan=vplan, Yv=Yv, Yva=Yva, Yvc=Yvc):
            _lib.check(VL.mignn_gcn_layer_win(P(vplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X),
                                              H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yv), H, st), "wv")
            _lib.check(VL.mignn_gcn_aggregate_win(P(vplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew),
                                                  P(X), H, 0, n, H, P(Yva), H, st), "wva")
            if Yvc is not None:
                win_codes(VL, vplan, Yvc)
        vchecks[vname] = vcheck

        def fva(VL=VL, vplan=vplan):
            _lib.check(VL.mignn_gcn_aggregate_win(P(vplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew),
                                                  P(X), H, 0, n, H, P(Ywa), H, st), "wva")
        cases[f"win@{vname}"] = fv
        cases[f"win_aggregate@{vname}"] = fva
        if codes is not None:
            cases[f"win_layers01_codes@{vname}"] = (lambda VL=VL, vplan=vplan: win_codes(VL, vplan, Ywc))
    for m in [int(v) for v in os.environ.get("WB_MODES", "").split(",") if v]:
        def fw(m=m):
            _lib.check(L.mignn_diag_win(m, P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X),
                                        H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yd), H, st), "dwin")
        cases[f"win_mode{m}"] = fw
    if old:
        Y0, Yr, Yra = torch.empty_like(X), torch.empty_like(X), torch.empty_like(X)
        nbr = L.mignn_gcn_ring_plan_bytes(0, n, H)
        rplan = torch.empty(nbr, dtype=torch.uint8, device=dev)

        def pc():
            _lib.check(L.mignn_gcn_layer_f16x3(P(csr_b.row_ptr), P(csr_b.col), P(csr_b.ew), P(X), H, 0, n,
                                               H, P(W), P(b), P(sc), P(sh), 15, P(Y0), H, st), "pc")

        def ring():
            _lib.check(L.mignn_gcn_layer_ring(P(rplan), P(csr_b.row_ptr), P(csr_b.col), P(csr_b.ew), P(X),
                                              H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Yr), H, st),
                       "ring")

        def ring_agg():
            _lib.check(L.mignn_gcn_aggregate_ring(P(rplan), P(csr_b.row_ptr), P(csr_b.col), P(csr_b.ew),
                                                  P(X), H, 0, n, H, P(Yra), H, st), "ring_agg")
        _lib.check(L.mignn_gcn_ring_plan(P(csr_b.row_ptr), P(csr_b.col), P(csr_b.ew), 0, n, H, P(rplan),
                                         nbr, None, st), "rplan")
        cases.update({"pc_f16x3": pc, "ring": ring, "ring_aggregate": ring_agg})
    # correctness on the bench mesh: the window layer vs the same layer on
    # the block-order CSR by the pc kernel (rows matched through the orders)
    win()
    win_agg()
    if codes is not None:
        win_codes()
    torch.cuda.synchronize()
    out = {"win_deterministic": None}
    Yw2 = Yw.clone()
    win()
    torch.cuda.synchronize()
    out["win_deterministic"] = bool(torch.equal(Yw, Yw2))
    del Yw2
    for vname in vout:
        vchecks[vname]()
        torch.cuda.synchronize()
        Yv, Yva, Yvc = vout[vname]
        out[f"win_vs_{vname}_max_diff"] = (Yw - Yv).abs().max().item()
        out[f"win_vs_{vname}_bitwise"] = bool(torch.equal(Yw, Yv))
        out[f"agg_vs_{vname}_bitwise"] = bool(torch.equal(Ywa, Yva))
        if Yvc is not None:
            out[f"codes_vs_{vname}_bitwise"] = bool(torch.equal(Ywc, Yvc))
    if old:
        pc()
        torch.cuda.synchronize()
        # internal row of node v: inv_c[v] (column order), inv_b[v] (block order);
        # X is indexed by internal rows of each order, so compare on a common X:
        # rerun pc on the column-order CSR (the kernel is order-agnostic)
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X), H, 0, n,
                                           H, P(W), P(b), P(sc), P(sh), 15, P(Y0), H, st), "pc_c")
        torch.cuda.synchronize()
        out["win_vs_pc_max_diff"] = (Yw - Y0).abs().max().item()
        out["pc_out_absmax"] = Y0.abs().max().item()
        pc()
        torch.cuda.synchronize()
    ms = timed(cases)
    by = 4 * (2 * n * H + (n + 1) + nnz + n)     # algorithmic bytes of the layer
    out.update({"ms": ms, "frac_of_8TBps": {k: round(by / (v * 1e-3) / 8e12, 4)
                                             for k, v in ms.items() if "plan" not in k}})
    res["by_h"][H] = out
    print(json.dumps({H: out}), file=sys.stderr, flush=True)
    del X, Yw, Ywa, Yd, wplan
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
