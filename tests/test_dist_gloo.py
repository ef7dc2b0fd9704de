"""Multi-rank path on the CPU: world_size-2 (and 3) `gloo` runs of the
k-slab partition + halo exchange (mignn/dist.py) -- the same driver the GPU
bench uses over RCCL -- with a CPU executor built from the oracle's
arithmetic.  Every rank's rows must match the single-process oracle forward of
the whole periodic mesh."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import grid_graph_np
from mignn.dist import LayerExecutor, SlabPartition, halo_exchange, sharded_forward
from mignn.gnn_model import FlowGNN
from mignn.synthetic import seeded_state_dict
from oracle import flowgnn_oracle as orc

NX, NY, NZL = 5, 4, 3        # per-rank slab: 5 x 4 x 3 = 60 nodes


class OracleExecutor(LayerExecutor):
    """CPU stand-in for FlowGNNExecutor (test infrastructure)."""

    def __init__(self, sd, cfg, part, ei_local, group=None):
        self.sd = {k: v.double() for k, v in sd.items()}
        self.cfg = cfg
        self.part = part
        self.num_layers = cfg["num_layers"]
        self.hidden_dim = cfg["hidden_dim"]
        self.overlap_ok = True
        src, dst = ei_local
        if cfg["layer_type"] == "GCN":
            keep = src != dst
            src, dst = src[keep], dst[keep]
            loops = torch.arange(part.n_own)
            src, dst = torch.cat([src, loops]), torch.cat([dst, loops])
            deg = torch.zeros(part.n_total, dtype=torch.float64).index_add_(
                0, dst, torch.ones(dst.shape[0], dtype=torch.float64))
            dinv = torch.where(deg > 0, deg.pow(-0.5), torch.zeros_like(deg)).view(-1, 1)
            for w in halo_exchange(dinv, part, group):     # ghost degrees from their owners
                w.wait()
            self.w = dinv[src, 0] * dinv[dst, 0]
        else:
            self.w = torch.ones(src.shape[0], dtype=torch.float64)
        self.src, self.dst = src, dst

    def input_proj(self, x_own, out):
        out.copy_(x_own.double() @ self.sd["input_proj.weight"].T + self.sd["input_proj.bias"])

    def layer(self, i, x, out, rb, re):
        sel = (self.dst >= rb) & (self.dst < re)
        s, d, w = self.src[sel], self.dst[sel], self.w[sel]
        agg = torch.zeros(re - rb, x.shape[1], dtype=x.dtype).index_add_(
            0, d - rb, x[s] * w.view(-1, 1))
        p = f"gnn_layers.{i}."
        if self.cfg["layer_type"] == "GCN":
            xn = agg @ self.sd[p + "lin.weight"].T + self.sd[p + "bias"]
        else:
            z = agg + (1 + float(self.sd[p + "eps"])) * x[rb:re]
            xn = torch.relu(z @ self.sd[p + "nn.0.weight"].T + self.sd[p + "nn.0.bias"])
            xn = xn @ self.sd[p + "nn.2.weight"].T + self.sd[p + "nn.2.bias"]
        b = f"batch_norms.{i}.module."
        y = orc.batch_norm_eval(x[rb:re] + xn, self.sd[b + "weight"], self.sd[b + "bias"],
                                self.sd[b + "running_mean"], self.sd[b + "running_var"])
        out[rb:re] = torch.relu(y)

    def output(self, x_own):
        sd = self.sd
        h = torch.relu(x_own @ sd["output_proj.0.weight"].T + sd["output_proj.0.bias"])
        h = torch.relu(h @ sd["output_proj.3.weight"].T + sd["output_proj.3.bias"])
        h = torch.relu(h @ sd["output_proj.6.weight"].T + sd["output_proj.6.bias"])
        return h @ sd["output_proj.8.weight"].T + sd["output_proj.8.bias"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, layer_type, outdir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.set_num_threads(1)
    cfg = dict(hidden_dim=16, num_layers=3, layer_type=layer_type)
    m = FlowGNN(input_dim=3, output_dim=7, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=5)
    part = SlabPartition(NX, NY, NZL, rank, world)
    x, ei = grid_graph_np(NX, NY, NZL * world, z_begin=rank * NZL, z_count=NZL)
    ei_local = part.localize(torch.from_numpy(ei))
    ex = OracleExecutor(sd, cfg, part, ei_local)
    y = sharded_forward(ex, part, torch.from_numpy(x).double())
    torch.save(y, os.path.join(outdir, f"y{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("layer_type", ["GCN", "GIN"])
def test_sharded_forward_matches_single_process(world, layer_type):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), layer_type, d), nprocs=world, join=True)
        ys = [torch.load(os.path.join(d, f"y{r}.pt"), weights_only=True) for r in range(world)]
    cfg = dict(hidden_dim=16, num_layers=3, layer_type=layer_type)
    m = FlowGNN(input_dim=3, output_dim=7, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=5)
    x, ei = grid_graph_np(NX, NY, NZL * world)
    ref = orc.flowgnn_forward(sd, cfg, torch.from_numpy(x), torch.from_numpy(ei), None,
                              dtype=torch.float64)
    got = torch.cat(ys, 0)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() < 1e-12


def test_partition_geometry():
    p = SlabPartition(5, 4, 3, rank=1, world=3)
    assert (p.plane, p.n_own, p.n_total) == (20, 60, 100)
    assert (p.lower_peer, p.upper_peer, p.z_begin) == (0, 2, 3)
    assert p.interior() == (20, 40) and p.boundary() == [(0, 20), (40, 60)]
    x, ei = grid_graph_np(5, 4, 9, z_begin=3, z_count=3)
    loc = p.localize(torch.from_numpy(ei))
    assert int(loc.min()) >= 0 and int(loc.max()) < p.n_total
    # own rows stay in order; the k-1 / k+1 planes map onto the two ghost planes
    assert torch.equal(loc[1], torch.from_numpy(ei[1]) - 60)
    with pytest.raises(ValueError):
        p.localize(torch.tensor([[0], [60]]))          # plane 0 is not a neighbour of rank 1
