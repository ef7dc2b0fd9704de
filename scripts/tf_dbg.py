"""Debug: fused TransformerConv layer vs the launch sequence at a size where
two blocks share a CU; prints the differing rows' statistics."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402

if os.environ.get("TD_LIB"):                       # an alternative build (experiments)
    _lib.LIB_PATH = os.environ["TD_LIB"]
from mignn.gnn_model import build_csr  # noqa: E402
import test_gpu_fused256 as T  # noqa: E402

DEV = "cuda"
H = 256
for n in [int(v) for v in os.environ.get("TD_N", "3000,200000").split(",")]:
    ei = T._graph(n, 31)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    g = torch.Generator(device=DEV).manual_seed(15)
    x = torch.randn(n, H, device=DEV, generator=g)
    wqk = torch.randn(4 * H, H, device=DEV, generator=g) / 16
    bqk = torch.randn(4 * H, device=DEV, generator=g) * 0.1
    wout = torch.randn(H, 4 * H + 4 + H, device=DEV, generator=g) / (4 * H + 4 + H) ** 0.5
    bout = torch.randn(H, device=DEV, generator=g) * 0.1
    sc = torch.rand(H, device=DEV, generator=g) + 0.5
    sh = torch.randn(H, device=DEV, generator=g) * 0.1
    outs = []
    for fused in (True, False):
        o = torch.full((n, H), float("nan"), device=DEV)
        T._tf_layer(fused, csr, x, 0, n, wqk, bqk, wout, bout, sc, sh, 15, o)
        outs.append(o)
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max(1).values
    bad = torch.nonzero(d > 1e-4).flatten()
    deg = (csr.row_ptr[1:n + 1] - csr.row_ptr[:n]).long()
    print(n, "bad rows", bad.numel(), "max diff", d.max().item(),
          "bad deg hist", torch.bincount(deg[bad], minlength=13)[:16].tolist() if bad.numel() else [],
          "all deg>8 rows", int((deg > 8).sum()),
          "bad mod64", torch.bincount(bad % 64, minlength=64).tolist() if bad.numel() else [], flush=True)
