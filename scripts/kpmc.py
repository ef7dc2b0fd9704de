"""Short PMC target (round 4): the hot-kernel candidates on the bench mesh
(250x200x200, locality order, H = KP_H), each launched KP_REPS times, nothing
else -- run under `rocprofv3 --pmc ...` (scripts/gpu_kpmc.sh).  KP_KINDS:
pc, ring, win, winagg, wincodes (the codes form, MODE 64), windiag, gin, tf,
gat, head (the fused output head at H = KP_H, out 7)."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
H = int(os.environ.get("KP_H", "128"))
reps = int(os.environ.get("KP_REPS", "2"))
kinds = os.environ.get("KP_KINDS", "pc,ring,win,winagg").split(",")
pos, ei = grid_graph(250, 200, 200, device=dev)
n = pos.shape[0]
_, inv = locality_order(pos, ei)
csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
del ei
L = _lib.lib()
P = _lib.ptr
st = _lib.stream()
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
W = torch.randn(H, H, device=dev, generator=g) * 0.05
b = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
Y = torch.empty_like(X)
if "win" in kinds or "winagg" in kinds or "windiag" in kinds or "wincodes" in kinds:
    # the window kernel on the column-order CSR of the same mesh
    _pos, _ei = grid_graph(250, 200, 200, device=dev)
    _, inv_c, info_c = locality_order(_pos, _ei, cols=True)
    csr_c = build_csr(_ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv_c)
    del _pos, _ei
    nbw = L.mignn_gcn_win_plan_bytes(0, n, H)
    wplan = torch.empty(nbw, dtype=torch.uint8, device=dev)
    _lib.check(L.mignn_gcn_win_plan(P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), 0, n, H, P(info_c),
                                    P(wplan), nbw, None, st), "wp")
if "wincodes" in kinds:
    # the codes form of the window kernel (layer 1 from layer-0 row codes):
    # codes [n, 8] (last column 0) and an expansion table [H][8]
    CODES = torch.rand(n, 8, device=dev, generator=g)
    CODES[:, 7] = 0.0
    XCOEF = torch.randn(H, 8, device=dev, generator=g) * 0.5
if "ring" in kinds:
    nbr = L.mignn_gcn_ring_plan_bytes(0, n, H)
    rplan = torch.empty(nbr, dtype=torch.uint8, device=dev)
    _lib.check(L.mignn_gcn_ring_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), 0, n, H, P(rplan), nbr,
                                     None, st), "rp")
if "gin" in kinds or "tf" in kinds:
    # H = 256 fused layers (KP_H=256): GIN (verbatim CSR) and TransformerConv
    from mignn.gnn_model import f16x3_image, gin_fused_image  # noqa: E402
    W2 = torch.randn(H, H, device=dev, generator=g) * 0.05
    GI1, GI2 = f16x3_image(W), gin_fused_image(W2)
    TWQ = torch.randn(4 * H + 4, H, device=dev, generator=g) / 16
    TBQ = torch.randn(4 * H + 4, device=dev, generator=g) * 0.05
    TWO = torch.randn(H, 4 * H + 4 + H, device=dev, generator=g) / (5 * H) ** 0.5
    TQIMG = f16x3_image(TWQ)
    TFIMG = torch.empty(L.mignn_transformer_fused_prep_bytes(H, 4), dtype=torch.uint8, device=dev)
    if "tf" in kinds:
        _lib.check(L.mignn_transformer_fused_prep(P(TWO), H, 4, P(TFIMG), TFIMG.numel(), st), "prep")
        TSCR = torch.empty(L.mignn_transformer_layer_scratch_bytes(n, H, 4), dtype=torch.uint8,
                           device=dev)
if "gat" in kinds:
    # the fused GAT layer (4 heads, split-fp16 image of Wcat [H, 4H]) on the same mesh
    from mignn.gnn_model import f16x3_image  # noqa: E402
    WLOG = torch.randn(8, H, device=dev, generator=g) / H ** 0.5
    WCAT = torch.randn(H, 4 * H, device=dev, generator=g) / (2 * H) ** 0.5
    GIMG = f16x3_image(WCAT)
    GSCR = torch.empty(max(L.mignn_gat_layer_scratch_bytes(n, n, H, 4), 1), dtype=torch.uint8,
                       device=dev)
if "head" in kinds:
    HW = [torch.randn(H, H, device=dev, generator=g) * 0.08, torch.randn(H, H, device=dev, generator=g) * 0.08,
          torch.randn(H // 2, H, device=dev, generator=g) * 0.08, torch.randn(7, H // 2, device=dev, generator=g) * 0.1]
    HB = [torch.randn(w.shape[0], device=dev, generator=g) * 0.05 for w in HW]
    HIMG = torch.empty(L.mignn_mlp_head_prep_bytes(H), dtype=torch.uint8, device=dev)
    _lib.check(L.mignn_mlp_head_prep(P(HW[0]), P(HB[0]), P(HW[1]), P(HB[1]), P(HW[2]), P(HB[2]), P(HW[3]),
                                     P(HB[3]), H, 7, P(HIMG), HIMG.numel(), st), "head prep")
    XR = torch.relu(X)
    HOUT = torch.empty(n, 7, device=dev)
for _ in range(reps):
    if "head" in kinds:
        _lib.check(L.mignn_mlp_head(P(XR), H, n, H, P(HIMG), 7, P(HOUT), 7, None, st), "head")
    if "gin" in kinds:
        _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 0.0,
                                           P(GI1), P(b), P(GI2), P(b), P(sc), P(sh), 15, P(Y), H,
                                           st), "gin")
    if "tf" in kinds:
        _lib.check(L.mignn_transformer_layer_fused(
            P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, 4, 1.0 / H ** 0.5, P(TQIMG), P(TBQ),
            P(TFIMG), P(b), P(sc), P(sh), 15, P(TSCR), TSCR.numel(), P(Y), H, st), "tf")
    if "gat" in kinds:
        _lib.check(L.mignn_gat_layer(P(csr.row_ptr), P(csr.col), P(X), H, n, 0, n, H, 4, 0.2,
                                     P(WLOG), None, 8, P(WCAT), P(GIMG), P(b), P(sc), P(sh), 15,
                                     P(GSCR), GSCR.numel(), P(Y), H, st), "gat")
    if "pc" in kinds:
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                           P(W), P(b), P(sc), P(sh), 15, P(Y), H, st), "pc")
    if "win" in kinds:
        _lib.check(L.mignn_gcn_layer_win(P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X), H,
                                         0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H, st), "win")
    if "wincodes" in kinds:
        _lib.check(L.mignn_gcn_layer_win_codes(P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew),
                                               P(CODES), 8, 0, n, H, P(XCOEF), P(W), P(b), P(sc),
                                               P(sh), 15, P(Y), H, st), "wincodes")
    if "winagg" in kinds:
        _lib.check(L.mignn_gcn_aggregate_win(P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X),
                                             H, 0, n, H, P(Y), H, st), "winagg")
    if "ring" in kinds:
        _lib.check(L.mignn_gcn_layer_ring(P(rplan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                          0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H, st), "ring")
    if "windiag" in kinds:
        # the window kernel's ablations (diag build; kernel names carry the
        # mode): 1 ext rows from the zero row, 4 no MFMAs, 32 aggregate only,
        # 33 aggregate only + ext from the zero row -- the per-phase VALU split
        LD = _lib.diag_lib()
        for m in (1, 4, 32, 33):
            _lib.check(LD.mignn_diag_win(m, P(wplan), P(csr_c.row_ptr), P(csr_c.col), P(csr_c.ew), P(X), H,
                                         0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H, st), "windiag")
torch.cuda.synchronize()
print("ok")
