"""The sharded (N > 1) route's cost per rank, measured in one process on
one GPU: the bench's weak-scaling mesh for P ranks (250 x 200 x (200 P),
k-slab ranges), all P shards driven by sharded_forward over LocalExchange
(device copies for the halo), so no two processes time-slice the GPU.
Times per step: the partition layout (RangeLayout, every rank), the shard
setup (rank-local CSR, ghost degrees, gcn_norm weights, ghost coordinates)
and the forward; per rank = total / P.  SB_P (2), SB_REPS (5), SB_ORDER
(cols: the column order, window kernel, the bench's N > 1 route; blocks).  Prints one
JSON object."""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import FlowGNN  # noqa: E402
from mignn.dist import FlowGNNShard, LocalExchange, build_local_layouts, sharded_forward  # noqa: E402
from mignn.gnn_model import locality_order  # noqa: E402
from mignn.synthetic import grid_graph, seeded_state_dict  # noqa: E402

dev = torch.device("cuda", 0)
P = int(os.environ.get("SB_P", "2"))
reps = int(os.environ.get("SB_REPS", "5"))
nx, ny, nz = 250, 200, 200
m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=128, num_layers=4, layer_type="GCN", dropout=0.0)
m.load_state_dict(seeded_state_dict(m.state_dict(), seed=1))
m = m.to(dev).eval()
xs, eis = [], []
for r in range(P):
    x, ei = grid_graph(nx, ny, nz * P, device=dev, z_begin=r * nz, z_count=nz)
    xs.append(x)
    eis.append(ei)
n = xs[0].shape[0]
bounds = [r * n for r in range(P + 1)]
if os.environ.get("SB_ORDER", "cols") == "cols":   # the window kernel's order (bench N > 1)
    order = lambda p, e: (lambda r: (r[0], r[2]))(locality_order(p, e, cols=True))  # noqa: E731
else:
    order = lambda p, e: locality_order(p, e)[0]  # noqa: E731
exch = LocalExchange()


def timed(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = f()
    torch.cuda.synchronize()
    return out, 1e3 * (time.perf_counter() - t0)


res = {"P": P, "rows_per_rank": n, "ms": {"layout": [], "setup": [], "forward": []}}
with torch.no_grad():
    for it in range(reps + 1):
        lays, t_lay = timed(lambda: build_local_layouts(eis, bounds, xs, order))
        shards = [FlowGNNShard(m, lay, x) for lay, x in zip(lays, xs)]

        def setup():
            shards[0].setup(exch, shards)
        _, t_set = timed(setup)
        _, t_fwd = timed(lambda: sharded_forward(shards, exch, xs))
        if it > 0:
            res["ms"]["layout"].append(t_lay)
            res["ms"]["setup"].append(t_set)
            res["ms"]["forward"].append(t_fwd)
        print(f"rep {it}: layout {t_lay:.2f} setup {t_set:.2f} forward {t_fwd:.2f} ms",
              file=sys.stderr, flush=True)
        del shards, lays
med = {k: round(statistics.median(v), 3) for k, v in res["ms"].items()}
res["median_ms"] = med
res["per_rank_ms"] = {k: round(v / P, 3) for k, v in med.items()}
res["gcn_route"] = m._gcn_kernel(128)
print(json.dumps(res), flush=True)
