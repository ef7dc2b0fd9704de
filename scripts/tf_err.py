"""configs[3] accuracy by fused part (round 3 diagnosis): the test_gpu_large
config3 check (48 sampled rows vs the fp64 oracle on their receptive field)
with MIGNN_FUSED256 = 1 / layer / head / 0."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "tests"))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from helpers import khop_subgraph  # noqa: E402
from mignn import FlowGNN  # noqa: E402
from mignn.synthetic import grid_graph, seeded_state_dict  # noqa: E402
from oracle import flowgnn_oracle as orc  # noqa: E402

dev = "cuda"
cfg = dict(hidden_dim=256, num_layers=6, layer_type="Transformer")
m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
sd = seeded_state_dict(m.state_dict(), seed=0)
m.load_state_dict(sd)
m = m.to(dev).eval()
dims = tuple(int(v) for v in os.environ.get("TE_GRID", "250,200,200").split(","))
x, ei = grid_graph(*dims, device=dev)
n = x.shape[0]
g = torch.Generator().manual_seed(1234)
seeds = torch.randperm(n, generator=g)[:48].to(dev)
ys = {}
with torch.no_grad():
    for mode in ("1", "layer", "head", "0"):
        m.fused256 = mode
        ys[mode] = m(x, ei)[seeds].cpu().double()
nodes, sub = khop_subgraph(ei, n, seeds, 6)
xs, subc = x[nodes].cpu(), sub.cpu()
r64 = orc.flowgnn_forward(sd, cfg, xs, subc, None, dtype=torch.float64)[:48]
r32 = orc.flowgnn_forward(sd, cfg, xs, subc, None, dtype=torch.float32)[:48]
print({"fp32_oracle": (r32.double() - r64).abs().max().item(), "ymax": r64.abs().max().item(),
       **{f"fused_{k}": (v - r64).abs().max().item() for k, v in ys.items()}}, flush=True)
