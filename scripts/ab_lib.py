"""A/B of one fused layer entry between two builds of libmignn.so (the
current one and gnn-bfs-rans_amd/mignn/libmignn_prev.so, built from an earlier
tree), same inputs, interleaved rounds, HIP events, median.  Env: AB_MODE
(gin | gcn | gat), AB_GRID."""
import ctypes
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, f16x3_image, gin_fused_image, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
mode = os.environ.get("AB_MODE", "gin")
H = int(os.environ.get("AB_H", "128")) if mode in ("gat", "pc", "ring") else 256
nx, ny, nz = (int(v) for v in os.environ.get("AB_GRID", "500,400,63").split(","))
pos, ei = grid_graph(nx, ny, nz, device=dev)
n = pos.shape[0]
_, inv = locality_order(pos, ei)
csr = build_csr(ei, n, _lib.CSR_VERBATIM if mode == "gin" else _lib.CSR_ONE_SELF_LOOP, relabel=inv)
del ei, pos
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
W1 = torch.randn(H, H, device=dev, generator=g) / 16
W2 = torch.randn(H, H, device=dev, generator=g) / 16
b1 = torch.randn(H, device=dev, generator=g) * 0.05
b2 = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
img1, img2 = (f16x3_image(W1), gin_fused_image(W2)) if H == 256 else (None, None)
if mode == "gat":
    WLOG = torch.randn(8, H, device=dev, generator=g) / H ** 0.5
    WCAT = torch.randn(H, 4 * H, device=dev, generator=g) / (2 * H) ** 0.5
    imgc = f16x3_image(WCAT)
    GSCR = torch.empty(max(_lib.lib().mignn_gat_layer_scratch_bytes(n, n, H, 4), 1),
                       dtype=torch.uint8, device=dev)
# AB_LIBS (name=path,...): variant builds (scripts/build_variant.sh) timed
# beside the in-tree library; default: libmignn_prev.so
libs = {"cur": _lib.lib()}
for item in [v for v in os.environ.get("AB_LIBS", "").split(",") if v]:
    name, path = item.split("=")
    libs[name] = _lib._load(path, _lib.SIGNATURES)
if len(libs) == 1:
    libs["prev"] = _lib._load(os.path.join(HERE, "gnn-bfs-rans_amd", "mignn", "libmignn_prev.so"),
                              _lib.SIGNATURES)
P = _lib.ptr
st = _lib.stream()


def run(L, Y):
    if mode == "gin":
        _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 0.0,
                                           P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), 15,
                                           P(Y), H, st), "gin")
    elif mode == "gemm":
        _lib.check(L.mignn_linear_f16x3(P(X), H, n, H, None, 0, 0, P(GIMG), GN, P(GB), None, 0,
                                        None, None, 1, P(Y), GN, st), "gemm")
    elif mode == "tf":
        _lib.check(L.mignn_transformer_layer_fused(
            P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 4, 1.0 / H ** 0.5, P(TQIMG), P(TBQ),
            P(TFIMG), P(TBO), P(sc), P(sh), 15, P(TSCR), TSCR.numel(), P(Y), H, st), "tf")
    elif mode == "pc":
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                           P(W1), P(b1), P(sc), P(sh), 15, P(Y),
                                           H, st), "pc")
    elif mode == "ring":
        _lib.check(L.mignn_gcn_layer_ring(P(RPLAN), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                          0, n, H, P(W1), P(b1), P(sc), P(sh), 15, P(Y), H, st),
                   "ring")
    elif mode == "gat":
        _lib.check(L.mignn_gat_layer(P(csr.row_ptr), P(csr.col), P(X), H, n, 0, n, H, 4, 0.2,
                                     P(WLOG), None, 8, P(WCAT), P(imgc), P(b1), P(sc), P(sh), 15,
                                     P(GSCR), GSCR.numel(), P(Y), H, st), "gat")
    else:
        _lib.check(L.mignn_gcn_layer_fused(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n,
                                           H, P(img1), P(b1), P(sc), P(sh), 15, P(Y), H, st), "gcn")


if mode == "ring":
    nbr = _lib.lib().mignn_gcn_ring_plan_bytes(0, n, H)
    RPLAN = torch.empty(nbr, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().mignn_gcn_ring_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), 0, n, H,
                                              P(RPLAN), nbr, None, st), "rplan")
if mode == "tf":
    TWQ = torch.randn(4 * H + 4, H, device=dev, generator=g) / 16
    TBQ = torch.randn(4 * H + 4, device=dev, generator=g) * 0.05
    TWO = torch.randn(H, 4 * H + 4 + H, device=dev, generator=g) / 32
    TBO = torch.randn(H, device=dev, generator=g) * 0.05
    TQIMG = f16x3_image(TWQ)
    Lc = _lib.lib()
    TFIMG = torch.empty(Lc.mignn_transformer_fused_prep_bytes(H, 4), dtype=torch.uint8, device=dev)
    _lib.check(Lc.mignn_transformer_fused_prep(P(TWO), H, 4, P(TFIMG), TFIMG.numel(), st), "prep")
    TSCR = torch.empty(Lc.mignn_transformer_layer_scratch_bytes(n, H, 4), dtype=torch.uint8,
                       device=dev)

if mode == "gemm":
    # TransformerConv's Q~K shape: [n, 256] x [256 -> 4 x 256] + bias
    GN = 4 * H
    GW = torch.randn(GN, H, device=dev, generator=g) / 16
    GB = torch.randn(GN, device=dev, generator=g) * 0.05
    GIMG = f16x3_image(GW)
    Ys = {k: torch.empty((n, GN), device=dev) for k in libs}
else:
    Ys = {k: torch.empty_like(X) for k in libs}
for k, L in libs.items():
    run(L, Ys[k])
torch.cuda.synchronize()
res = {"mode": mode, "n": n, "h": H,
       "max_diff": {k: (Ys["cur"] - v).abs().nan_to_num(0.0).max().item() for k, v in Ys.items()},
       "nan_rows": {k: int(torch.isnan(v).any(1).sum().item()) for k, v in Ys.items()},
       "bitwise_equal": {k: bool(torch.equal(Ys["cur"].view(torch.int32), v.view(torch.int32)))
                         for k, v in Ys.items()}}
times = {k: [] for k in libs}
for rnd in range(int(os.environ.get("AB_REPS", "5")) + 1):
    for k, L in libs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(L, Ys[k])
        e1.record()
        e1.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1) / 3)
res["ms"] = {k: round(statistics.median(v), 4) for k, v in times.items()}
print(json.dumps(res), flush=True)
