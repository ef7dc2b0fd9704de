"""Why does the GCN layer take longer inside the bench forward than in
kbench?  Times mignn_gcn_layer_f16x3 on (a) random X, (b) the model's own
activations, (c) the bench model's weights, on the bench graph."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import FlowGNN, _lib  # noqa: E402
from mignn.synthetic import grid_graph, seeded_state_dict  # noqa: E402

dev = torch.device("cuda", 0)
H = 128
model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, hidden_dim=H, num_layers=4,
                layer_type="GCN")
model.load_state_dict(seeded_state_dict(model.state_dict(), seed=0))
model = model.to(dev).eval()
x, ei = grid_graph(250, 200, 200, device=dev)
n = x.shape[0]
with torch.no_grad():
    model(x, ei)
csr = model._csr.get(ei, n, _lib.CSR_ONE_SELF_LOOP)
act = torch.empty(n, H, device=dev)
model._input_proj(x, act)
L, P, st = _lib.lib(), _lib.ptr, _lib.stream()
g = torch.Generator(device=dev).manual_seed(0)
Xr = torch.randn(n, H, device=dev, generator=g)
Wr = torch.randn(H, H, device=dev, generator=g) * 0.05
br = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
layer = model.gnn_layers[0]
scale, shift = model._bn(0)
Y = torch.empty_like(Xr)


def run(X, W, b, s, t):
    _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                       P(W), P(b), P(s), P(t), 15, P(Y), H, st), "gcn16")


cases = {"random_all": (Xr, Wr, br, sc, sh),
         "model_act_random_w": (act, Wr, br, sc, sh),
         "random_x_model_w": (Xr, layer.lin.weight, layer.bias, scale, shift),
         "model_all": (act, layer.lin.weight, layer.bias, scale, shift)}
res = {}
for rnd in range(4):
    for k, a in cases.items():
        run(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(*a)
        e1.record()
        e1.synchronize()
        if rnd:
            res.setdefault(k, []).append(round(e0.elapsed_time(e1) / 3, 3))
res["act_zero_frac"] = (act == 0).float().mean().item()
res["act_absmax"] = act.abs().max().item()
res["csr_nnz"] = int(csr.row_ptr[-1].item())
res["w_absmax"] = layer.lin.weight.abs().max().item()
print(json.dumps(res))
