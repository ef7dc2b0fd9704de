"""Timeline of the window GCN kernel (mignn_diag_win_trace): median cycles per
phase over workgroups 0..7, steps 8..62, waves 0 and 4 (10M mesh, column
order).  Points (H = 128, round 6 pipelined step): 0 top, 1 after B0, 2 phase A
with tile s-2's MFMA groups, 3 epilogue + stores + seeds, 4 B1 + DMA issue,
5 phase B + split; aggregate mode (32): 0 top, 1 after B0, 2 phase A, 3
phase B, 4 after B2.  Env: WT_H (128), WT_MODE (diag mode, 0)."""
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
H = int(os.environ.get("WT_H", "128"))
mode = int(os.environ.get("WT_MODE", "0"))
pos, ei = grid_graph(250, 200, 200, device=dev)
n = pos.shape[0]
_, inv, info = locality_order(pos, ei, cols=True)
csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
del ei
L = _lib.diag_lib()
P = _lib.ptr
st = _lib.stream()
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
W = torch.randn(H, H, device=dev, generator=g) * 0.05
b = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
nb = L.mignn_gcn_win_plan_bytes(0, n, H)
plan = torch.empty(nb, dtype=torch.uint8, device=dev)
_lib.check(L.mignn_gcn_win_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), 0, n, H, P(info), P(plan), nb,
                                None, st), "plan")
Y = torch.empty_like(X)
tr = torch.zeros(8 * 64 * 2 * 16, dtype=torch.int64, device=dev)


def run():
    _lib.check(L.mignn_diag_win(mode, P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                P(W), P(b), P(sc), P(sh), 15, P(Y), H, st), "win")


for _ in range(5):
    run()
_lib.check(L.mignn_diag_win_trace(P(tr)), "trace")
run()
torch.cuda.synchronize()
_lib.check(L.mignn_diag_win_trace(None), "trace")
t = tr.view(8, 64, 2, 16).cpu()
res = {"H": H, "mode": mode}
if H == 64:
    pts = [0, 1, 2, 3, 6, 4, 5] if not mode & 32 else [0, 1, 2, 3, 6, 5]
else:
    # (round 6 pipelined step: 0 top, 1 after B0, 2 phase A with tile s-2's
    # MFMA groups, 3 epilogue + stores + seeds (before B1), 4 B1 + DMA issue,
    # 5 phase B + split (+ codes expansion))
    pts = [0, 1, 2, 3, 4, 5] if not mode & 32 else [0, 1, 2, 3, 4]
for wv in ((0,) if H == 64 else (0, 1)):
    d = {}
    for a, b_ in zip(pts, pts[1:] + [0]):
        vals = []
        for blk in range(8):
            for s in range(8, 62):
                t1 = t[blk, s + 1, wv, b_] if b_ == 0 else t[blk, s, wv, b_]
                vals.append(int(t1 - t[blk, s, wv, a]))
        d[f"{a}->{b_}"] = statistics.median(vals)
    step = [int(t[blk, s + 1, wv, 0] - t[blk, s, wv, 0]) for blk in range(8) for s in range(8, 62)]
    d["step"] = statistics.median(step)
    res[f"wave{4 * wv}"] = d
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    run()
e1.record()
e1.synchronize()
res["ms"] = e0.elapsed_time(e1) / 5
print(json.dumps(res))
