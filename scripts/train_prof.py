"""One layer type's train step (bench.py train_leg's step: forward with
batch-stat BN + dropout, WeightedMSELoss, backward, clip, Adam) run TP_STEPS
times on the TP_GRID periodic mesh -- for `rocprofv3 --kernel-trace --stats`
of the training kernels.  TP_TYPE: GCN / GIN / GAT / Transformer."""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import FlowGNN  # noqa: E402
from mignn.normalization import WeightedMSELoss  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
lt = os.environ.get("TP_TYPE", "GAT")
nx, ny, nz = (int(v) for v in os.environ.get("TP_GRID", "100,100,100").split(","))
x, ei = grid_graph(nx, ny, nz, device=dev)
n, e = x.shape[0], ei.shape[1]
target = torch.randn((n, 7), generator=torch.Generator().manual_seed(11)).to(dev)
weights = {"U": 1.0, "p": 3.0, "k": 0.5, "epsilon": 0.5, "nut": 0.5}
torch.manual_seed(0)
model = FlowGNN(input_dim=3, hidden_dim=128, output_dim=7, num_layers=4, layer_type=lt, dropout=0.1).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
crit = WeightedMSELoss(field_weights=weights, use_fieldwise=True, pressure_ref_weight=0.1)
ea = None if lt == "Transformer" else torch.zeros((e, 4), device=dev)
for i in range(int(os.environ.get("TP_STEPS", "4"))):
    t0 = time.time()
    opt.zero_grad()
    loss = crit(model(x, ei, ea), target, pressure_ref_weight=0.1)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    opt.step()
    torch.cuda.synchronize()
    print(lt, i, round((time.time() - t0) * 1e3, 2), "ms", float(loss), flush=True)
