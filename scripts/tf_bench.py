"""Fused TransformerConv timing (round 3): mignn_transformer_layer_fused vs
mignn_transformer_layer (Q~K GEMM + softmax aggregation + output GEMM) on
configs[3]'s mesh (250 x 200 x 200 periodic hex, 10M nodes, locality order),
HIP events, interleaved rounds; also the Q~K GEMM alone (the part both share).
Env: TB_GRID (250,200,200), TB_REPS (3)."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, f16x3_image, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
H, HEADS = 256, 4
nx, ny, nz = (int(v) for v in os.environ.get("TB_GRID", "250,200,200").split(","))
pos, ei = grid_graph(nx, ny, nz, device=dev)
n = pos.shape[0]
perm, inv = locality_order(pos, ei)
csr = build_csr(ei, n, _lib.CSR_VERBATIM, relabel=inv)
del ei, pos
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
WQK = torch.randn(HEADS * H, H, device=dev, generator=g) / 16
BQK = torch.randn(HEADS * H, device=dev, generator=g) * 0.1
WOUT = torch.randn(H, HEADS * H + HEADS + H, device=dev, generator=g) / 36
BOUT = torch.randn(H, device=dev, generator=g) * 0.1
SC = torch.rand(H, device=dev, generator=g) + 0.5
SH = torch.randn(H, device=dev, generator=g) * 0.1
L = _lib.diag_lib()
P = _lib.ptr
st = _lib.stream()
IMG_Q, IMG_O = f16x3_image(WQK), f16x3_image(WOUT)
FIMG = torch.empty(L.mignn_transformer_fused_prep_bytes(H, HEADS), dtype=torch.uint8, device=dev)
_lib.check(L.mignn_transformer_fused_prep(P(WOUT), H, HEADS, P(FIMG), FIMG.numel(), st), "prep")
NB = L.mignn_transformer_layer_scratch_bytes(n, H, HEADS)
SCR = torch.empty(NB, dtype=torch.uint8, device=dev)


def fused(Y, diag=0):
    _lib.check(L.mignn_diag_set_fused_flags(diag), "diag")
    _lib.check(L.mignn_transformer_layer_fused(
        P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, HEADS, 1.0 / 16, P(IMG_Q), P(BQK), P(FIMG),
        P(BOUT), P(SC), P(SH), 15, P(SCR), NB, P(Y), H, st), "fused")


def launches(Y):
    _lib.check(L.mignn_transformer_layer(
        P(csr.row_ptr), P(csr.col), P(X), H, 0, n, H, HEADS, 1.0 / 16, P(WQK), P(IMG_Q), P(BQK),
        P(WOUT), P(IMG_O), P(BOUT), P(SC), P(SH), 15, P(SCR), NB, P(Y), H, st), "launches")


def qk_gemm(Y):
    _lib.check(L.mignn_linear_f16x3(P(X), H, n, H, None, 0, 0, P(IMG_Q), HEADS * H, P(BQK), None,
                                    0, None, None, 1, P(SCR), HEADS * H, st), "qk")


cases = {"fused": fused, "launches": launches, "qk_gemm": qk_gemm}
# ablations (wrong results; timing only): 4096 no pass 1, 256 no weighted sums, 512 no MFMA
for dflag in [int(v) for v in os.environ.get("TB_ABLATE", "").split(",") if v]:
    cases[f"fused_ablate_{dflag}"] = (lambda d: (lambda Y: fused(Y, d)))(dflag)

outs = {k: torch.full_like(X, float("nan")) for k in ("fused", "launches")}
for k in outs:
    cases[k](outs[k])
torch.cuda.synchronize()
ref = outs["launches"]
res = {"grid": [nx, ny, nz], "n": n, "entries": int(csr.row_ptr[-1].item()),
       "max_rel_fused_vs_launches": ((outs["fused"] - ref).abs().max() / ref.abs().max()).item(),
       "nan_rows": int(torch.isnan(outs["fused"]).any(1).sum().item())}
del outs
Y = torch.empty_like(X)
reps = int(os.environ.get("TB_REPS", "3"))
times = {k: [] for k in cases}
for rnd in range(reps + 1):
    for k, f in cases.items():
        f(Y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            f(Y)
        e1.record()
        e1.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1) / 2)
_lib.check(L.mignn_diag_set_fused_flags(0), "diag")
res["ms"] = {k: round(statistics.median(v), 3) for k, v in times.items()}
res["ms"]["fused_agg_transform"] = round(res["ms"]["fused"] - res["ms"]["qk_gemm"], 3)
print(json.dumps(res), flush=True)
