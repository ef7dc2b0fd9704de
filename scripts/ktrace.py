"""Per-step timeline of the fused tile kernel (MIGNN_DIAG_TRACE): s_memtime
stamps of one producer and one consumer wave in workgroups 0..7."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
nx, ny, nz = (int(v) for v in os.environ.get("KB_GRID", "250,200,200").split(","))
H = 128
x0, ei = grid_graph(nx, ny, nz, device=dev)
n = x0.shape[0]
csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
del ei
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
Y = torch.empty_like(X)
W = torch.randn(H, H, device=dev, generator=g) * 0.05
b = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
L = _lib.lib()
P = _lib.ptr
st = _lib.stream()
tr = torch.zeros(8 * 64 * 8, dtype=torch.int64, device=dev)
_lib.check(L.mignn_diag_set_trace(P(tr)), "trace")
for extra, name in ((0, "full"), (512, "no_mfma"), (256, "no_gather")):
    for _ in range(3):
        tr.zero_()
        _lib.check(L.mignn_diag_gcn_layer(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H, P(W),
                                     P(b), P(sc), P(sh), 15 | 2048 | extra, P(Y), H, st), "gcn")
        torch.cuda.synchronize()
    t = tr.view(8, 64, 8).cpu().double()
    s = slice(4, 60)
    step = (t[:, 5:61, 0] - t[:, 4:60, 0]).mean().item()
    prod = (t[:, s, 1] - t[:, s, 0]).mean().item()
    mfma = (t[:, s, 3] - t[:, s, 2]).mean().item()
    epi = (t[:, s, 4] - t[:, s, 3]).mean().item()
    cstart = (t[:, s, 2] - t[:, s, 0]).mean().item()
    print(f"{name:10s} step {step:8.0f}  producer gather {prod:8.0f}  consumer mfma {mfma:8.0f}"
          f"  epilogue {epi:8.0f}  (consumer start - producer start {cstart:6.0f})  [s_memtime ticks]")
_lib.check(L.mignn_diag_set_trace(None), "trace")
