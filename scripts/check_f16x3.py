"""Quick GPU check of mignn_gcn_layer_f16x3 against an fp64 torch evaluation of
the same layer on the same CSR (development aid; the parity tests proper are
in tests/test_gpu_parity.py)."""
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
L = _lib.lib()
P = _lib.ptr


def ref_layer(csr, X, W, b, sc, sh, rb, re):
    rp = csr.row_ptr.cpu().long()
    col = csr.col.cpu().long()
    ew = csr.ew.cpu().double()
    Xd = X.cpu().double()
    n = re - rb
    rows = torch.repeat_interleave(torch.arange(csr.num_nodes), rp[1:] - rp[:-1])
    nnz = int(rp[-1])
    agg = torch.zeros(csr.num_nodes, X.shape[1], dtype=torch.float64)
    agg.index_add_(0, rows, ew[:nnz, None] * Xd[col[:nnz]])
    y = Xd[:csr.num_nodes] + b.cpu().double() + agg @ W.cpu().double().t()
    y = y * sc.cpu().double() + sh.cpu().double()
    return y.clamp_min(0)[rb:re]


worst = 0.0
for (nx, ny, nz, perm, H, extra_hub) in [(20, 16, 12, None, 128, False), (20, 16, 12, 3, 128, False),
                                           (23, 7, 5, None, 64, False), (31, 9, 7, 1, 64, False),
                                           (40, 30, 20, None, 128, True), (13, 11, 3, None, 128, False)]:
    x0, ei = grid_graph(nx, ny, nz, device=dev, permute_seed=perm)
    n = x0.shape[0]
    if extra_hub:   # node 5 receives from 300 nodes (hub row: slow path)
        src = torch.arange(100, 400, device=dev)
        ei = torch.cat([ei, torch.stack([src, torch.full_like(src, 5)])], 1)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(n, H, device=dev, generator=g)
    W = torch.randn(H, H, device=dev, generator=g) * 0.05
    b = torch.randn(H, device=dev, generator=g) * 0.05
    sc = torch.rand(H, device=dev, generator=g) + 0.5
    sh = torch.randn(H, device=dev, generator=g) * 0.1
    for (rb, re) in [(0, n), (7, n - 3)]:
        Y = torch.full((n, H), float("nan"), device=dev)
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb, re,
                                           H, P(W), P(b), P(sc), P(sh), 15, P(Y), H,
                                           _lib.stream()), "gcn16")
        torch.cuda.synchronize()
        ref = ref_layer(csr, X, W, b, sc, sh, rb, re)
        got = Y[rb:re].cpu().double()
        err = (got - ref).abs().max().item()
        untouched = torch.isnan(Y[:rb]).all().item() and torch.isnan(Y[re:]).all().item()
        print(f"grid {nx}x{ny}x{nz} perm={perm} H={H} hub={extra_hub} rows [{rb},{re}): "
              f"max|err| = {err:.3e} (max|ref| {ref.abs().max().item():.2f}), outside untouched: {untouched}")
        worst = max(worst, err)
        assert untouched
print("WORST", worst)
assert worst < 1e-5
