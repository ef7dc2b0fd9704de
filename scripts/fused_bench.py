"""Fused H = 256 layer timing (round 3): mignn_gin_layer_fused (8- and 4-wave
blocks) vs the launches it replaces (sum aggregate + two split-fp16 GEMMs) on
configs[4]'s per-GPU shard mesh (500 x 400 x 63 periodic hex, 12.6M nodes,
locality order), HIP events, interleaved rounds; max |fused - unfused|.
Env: FB_GRID (500,400,63), FB_REPS (5), FB_MODE (gin | gcn), FB_LIBS
(name=path,...: variant builds of libmignn.so timed beside it, GIN: each
with its own nn.2 image from its own mignn_gin_fused_prep)."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, f16x3_image, gin_fused_image, linear_f16x3, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
mode = os.environ.get("FB_MODE", "gin")
H = 128 if mode == "gat" else 256
nx, ny, nz = (int(v) for v in os.environ.get("FB_GRID", "500,400,63").split(","))
pos, ei = grid_graph(nx, ny, nz, device=dev)
n = pos.shape[0]
perm, inv = locality_order(pos, ei)
csr = build_csr(ei, n, _lib.CSR_VERBATIM if mode == "gin" else _lib.CSR_ONE_SELF_LOOP, relabel=inv)
E_in = int(ei.shape[1])
del ei, pos
res_edges = E_in
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
W1 = torch.randn(H, H, device=dev, generator=g) / 16
W2 = torch.randn(H, H, device=dev, generator=g) / 16
b1 = torch.randn(H, device=dev, generator=g) * 0.05
b2 = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
if mode == "gat":
    WLOG = torch.randn(8, H, device=dev, generator=g) / H ** 0.5
    WCAT = torch.randn(H, 4 * H, device=dev, generator=g) / (2 * H) ** 0.5
    img1 = f16x3_image(WCAT)
    GSCR = torch.empty(max(_lib.diag_lib().mignn_gat_layer_scratch_bytes(n, n, H, 4), 1), dtype=torch.uint8,
                       device=dev)
else:
    img1, img2, img2s = f16x3_image(W1), gin_fused_image(W2), f16x3_image(W2)
L = _lib.diag_lib()
P = _lib.ptr
st = _lib.stream()


def gat(on, diag=0):
    def f(Y):
        _lib.check(L.mignn_diag_set_gat_fused(on), "gat_fused")
        _lib.check(L.mignn_diag_set_fused_flags(diag), "diag")
        _lib.check(L.mignn_gat_layer(P(csr.row_ptr), P(csr.col), P(X), H, n, 0, n, H, 4, 0.2,
                                     P(WLOG), None, 8, P(WCAT), P(img1), P(b1), P(sc), P(sh), 15,
                                     P(GSCR), GSCR.numel(), P(Y), H, st), "gat_layer")
    return f


def fused(diag=0):
    def f(Y):
        _lib.check(L.mignn_diag_set_fused_flags(diag), "diag")
        if mode == "gin":
            _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 0.0,
                                               P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), 15,
                                               P(Y), H, st), "gin_fused")
        else:
            _lib.check(L.mignn_gcn_layer_fused(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0,
                                               n, H, P(img1), P(b1), P(sc), P(sh), 15, P(Y), H,
                                               st), "gcn_fused")
    return f


AGG = torch.empty(n, H, device=dev)
H1 = torch.empty(n, H, device=dev)


def unfused(Y):
    if mode == "gin":
        _lib.check(L.mignn_sum_aggregate(P(csr.row_ptr), P(csr.col), P(X), H, 1.0, 0, n, H, P(AGG),
                                         H, st), "sum")
        linear_f16x3(AGG, img1, H, b1, relu=True, out=H1)
        linear_f16x3(H1, img2s, H, b2, relu=True, residual=X, scale=sc, shift=sh, out=Y)
    else:
        _lib.check(L.mignn_gcn_aggregate(P(csr.row_ptr), P(csr.col), P(csr.dinv), P(X), H, 0, n,
                                         H, P(AGG), H, st), "gcn_agg")
        linear_f16x3(AGG, img1, H, b1, relu=True, residual=X, scale=sc, shift=sh, out=Y)


cases = ({"unfused": gat(0), "fused": gat(1)} if mode == "gat" else
         {"unfused": unfused, "fused": fused()})
for item in [v for v in os.environ.get("FB_LIBS", "").split(",") if v and mode == "gin"]:
    vname, vpath = item.split("=")
    VL = _lib._load(vpath, _lib.SIGNATURES)
    vimg2 = torch.empty(VL.mignn_gin_fused_prep_bytes(H), dtype=torch.uint8, device=dev)
    _lib.check(VL.mignn_gin_fused_prep(P(W2), H, P(vimg2), vimg2.numel(), st), "vprep")

    def fv(Y, VL=VL, vimg2=vimg2):
        _lib.check(VL.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 0.0,
                                            P(img1), P(b1), P(vimg2), P(b2), P(sc), P(sh), 15,
                                            P(Y), H, st), "gin_fused_v")
    cases[f"fused@{vname}"] = fv
for dflag in [int(v) for v in os.environ.get("FB_ABLATE", "").split(",") if v]:
    cases[f"fused_ablate_{dflag}"] = gat(1, dflag) if mode == "gat" else fused(dflag)
outs = {k: torch.full_like(X, float("nan")) for k in cases}
for k, f in cases.items():
    f(outs[k])
torch.cuda.synchronize()
res = {"mode": mode, "grid": [nx, ny, nz], "n": n,
       "check": {k: {"max_vs_unfused": (outs[k] - outs["unfused"]).abs().max().item(),
                     "nan_rows": int(torch.isnan(outs[k]).any(1).sum().item())} for k in cases},
       "ref_max": outs["unfused"].abs().max().item()}
del outs
_lib.check(L.mignn_diag_set_fused_flags(0), "diag")
Y = torch.empty_like(X)
reps = int(os.environ.get("FB_REPS", "5"))
times = {k: [] for k in cases}
for rnd in range(reps + 1):
    for k, f in cases.items():
        f(Y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            f(Y)
        e1.record()
        e1.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1) / 3)
res["ms"] = {k: round(statistics.median(v), 4) for k, v in times.items()}
_lib.check(L.mignn_diag_set_fused_flags(0), "diag")
E = int(csr.row_ptr[-1].item())
by = 4 * (2 * n * H + (n + 1) + E)
fl = {"gin": 4, "gcn": 2, "gat": 8}[mode] * n * H * H * 3
res["frac_hbm"] = {k: round(by / (v * 1e-3) / 8e12, 4) for k, v in res["ms"].items()}
res["f16_tflops"] = {k: round(fl / (v * 1e-3) / 1e12, 1) for k, v in res["ms"].items()}
print(json.dumps(res), flush=True)
