"""Records-path debugging: layer-1 outputs of the records kernel vs the
materialised path, with W = 0 (own-row expansion only) and random W."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gnn-bfs-rans_amd"))
from mignn import _lib  # noqa: E402

if os.environ.get("GB_LIB"):
    _lib.LIB_PATH = os.environ["GB_LIB"]
from mignn import FlowGNN  # noqa: E402
from mignn.gnn_model import EPI_AFFINE, EPI_BIAS, EPI_RELU, EPI_RESIDUAL  # noqa: E402
from mignn.synthetic import grid_graph, seeded_state_dict  # noqa: E402

dev = "cuda"
H = int(os.environ.get("RD_H", "64"))
m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=H, num_layers=3, layer_type="GCN")
m.load_state_dict(seeded_state_dict(m.state_dict(), seed=3))
m = m.to(dev).eval()
g = [int(v) for v in os.environ.get("RD_GRID", "40,36,30").split(",")]
x, ei = grid_graph(*g, device=dev)
N = x.shape[0]
csr = m._csr.get(ei, N, _lib.CSR_ONE_SELF_LOOP, x)
L, P = _lib.lib(), _lib.ptr
x0 = torch.empty(N, H, device=dev)
m._gcn_layer0(x, csr, x0)
rec = m._gcn_layer0_records(x, csr)
coef8 = m._layer0_coef8()
layer = m.gnn_layers[1]
scale, shift = m._bn(1)
for wname, W in (("W=0", torch.zeros_like(layer.lin.weight)), ("W", layer.lin.weight.detach())):
    for nm, bias in (("bias", layer.bias.detach()),):
        epi = EPI_BIAS | EPI_RESIDUAL | EPI_AFFINE | EPI_RELU
        ya = torch.empty(N, H, device=dev)
        yb = torch.empty(N, H, device=dev)
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(x0), H, 0, N,
                                           H, P(W), P(bias), P(scale), P(shift), epi, P(ya), H,
                                           _lib.stream()), "a")
        _lib.check(L.mignn_gcn_layer_f16x3_rec(P(csr.row_ptr), P(csr.col), P(csr.ew), P(rec),
                                               P(coef8), 0, N, H, P(W), P(bias), P(scale),
                                               P(shift), epi, P(yb), H, _lib.stream()), "b")
        torch.cuda.synchronize()
        d = (ya - yb).abs()
        bad = (d > 0).any(1).nonzero().flatten()
        steps = torch.bincount((bad // 64) // 256, minlength=(N // 64) // 256 + 1).tolist()
        print(f"H{H} {wname}: max diff {d.max().item():.3e}, rows differing {bad.numel()} / {N}, "
              f"first {bad[:10].tolist()}, per step {steps}", flush=True)
        if bad.numel():
            r = int(bad[0])
            c = (d[r] > 0).nonzero().flatten()
            print("  row", r, "cols", c[:16].tolist(), "a", ya[r, c[:4]].tolist(), "b",
                  yb[r, c[:4]].tolist(), "local row in tile", r % 64, flush=True)

# determinism: each path 3 times
for nm, fn in (("materialised", lambda o: L.mignn_gcn_layer_f16x3(
        P(csr.row_ptr), P(csr.col), P(csr.ew), P(x0), H, 0, N, H, P(layer.lin.weight),
        P(layer.bias), P(scale), P(shift), 15, P(o), H, _lib.stream())),
               ("records", lambda o: L.mignn_gcn_layer_f16x3_rec(
        P(csr.row_ptr), P(csr.col), P(csr.ew), P(rec), P(coef8), 0, N, H, P(layer.lin.weight),
        P(layer.bias), P(scale), P(shift), 15, P(o), H, _lib.stream()))):
    outs = []
    for _ in range(3):
        o = torch.full((N, H), float("nan"), device=dev)
        fn(o)
        torch.cuda.synchronize()
        outs.append(o)
    print(nm, "run-to-run rows differing:",
          [int((outs[0] != outs[k]).any(1).sum()) for k in (1, 2)],
          "nan rows", int(torch.isnan(outs[0]).any(1).sum()), flush=True)
