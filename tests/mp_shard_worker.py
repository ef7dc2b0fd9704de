"""One rank of the multi-process shard-route check (tests/test_gpu_dist_mp.py).

The route behind bench.py's N > 1 number, end to end in separate processes:
k-slab node ranges of a periodic hex mesh, RangeLayout over DistRequests,
FlowGNNShard on the rank-local CSR in the column order (the window GCN
kernel, layer 1 expanded from layer 0's 32-B row codes, whose ghost codes
travel in layer 1's halo), sharded_forward over DistExchange.  Every rank
runs on cuda:0 of a one-GPU box under gloo (DistExchange stages the halo
through host memory there; under nccl the same object hands device tensors
to RCCL).  Each rank also runs the unsharded FlowGNN forward on the whole
mesh and compares its own rows.  Rank 0 prints one JSON line.

Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (set by the test),
MP_GRID "nx,ny,nz_per_rank", MP_H (hidden), MP_LAYERS, MP_TYPE.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "gnn-bfs-rans_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    nx, ny, nz = (int(v) for v in os.environ.get("MP_GRID", "48,40,12").split(","))
    H = int(os.environ.get("MP_H", "128"))
    L = int(os.environ.get("MP_LAYERS", "4"))
    lt = os.environ.get("MP_TYPE", "GCN")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")

    from mignn import FlowGNN, _lib
    from mignn.dist import DistExchange, DistRequests, FlowGNNShard, RangeLayout, sharded_forward
    from mignn.gnn_model import locality_order
    from mignn.synthetic import grid_graph, seeded_state_dict

    cfg = dict(hidden_dim=H, num_layers=L, layer_type=lt)
    model = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    model.load_state_dict(seeded_state_dict(model.state_dict(), seed=11))
    model = model.to(dev).eval()
    model.reorder = "1"          # the locality order at this small size too (bench: >= 2^20 rows)

    # this rank's slab, global ids (bench.py's N > 1 workload, smaller)
    x, ei = grid_graph(nx, ny, nz * world, device=dev, z_begin=rank * nz, z_count=nz)
    n_local = x.shape[0]
    bounds = [r * n_local for r in range(world + 1)]
    assert model._column_order()
    order = lambda p, e: (lambda r: (r[0], r[2]))(locality_order(p, e, cols=True))  # noqa: E731
    exch = DistExchange()
    lay = RangeLayout(ei, bounds, rank, DistRequests(), pos=x, order_fn=order)
    sh = FlowGNNShard(model, lay, x)
    sh.setup(exch, [sh])
    route = {"window": model._gcn_kernel(H, sh.csr) == "win",
             "codes": bool(model._use_gcn_codes(sh.csr))}
    with torch.no_grad():
        y_sh = sharded_forward([sh], exch, [x])[0]
        y_sh2 = sharded_forward([sh], exch, [x])[0]
    torch.cuda.synchronize()
    # the unsharded forward on the whole mesh (same GPU), this rank's rows
    xa, eia = grid_graph(nx, ny, nz * world, device=dev)
    with torch.no_grad():
        y_all = model(xa, eia)
    torch.cuda.synchronize()
    mine = y_all[bounds[rank]:bounds[rank + 1]]
    scale = max(1.0, y_all.abs().max().item())
    err = (y_sh - mine).abs().max().item()
    dev_err = _lib.device_errors(clear=True)
    stats = torch.tensor([err, scale, float(dev_err), float(not torch.equal(y_sh, y_sh2)),
                          float(lay.n_ghost), float(lay.n_int)], dtype=torch.float64)
    allst = [torch.zeros_like(stats) for _ in range(world)]
    dist.all_gather(allst, stats)
    if rank == 0:
        print(json.dumps({
            "world": world, "grid": [nx, ny, nz * world], "layer_type": lt, "hidden": H, "layers": L,
            "route": route,
            "max_err": [s[0].item() for s in allst], "scale": [s[1].item() for s in allst],
            "device_errors": [int(s[2].item()) for s in allst],
            "nondeterministic": [bool(s[3].item()) for s in allst],
            "n_ghost": [int(s[4].item()) for s in allst], "n_interior": [int(s[5].item()) for s in allst],
        }), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
