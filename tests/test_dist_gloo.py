"""Multi-rank path on the CPU: world_size 2 and 3 `gloo` runs of the
contiguous node-range partition + halo exchange (mignn/dist.py) -- the same
driver the GPU bench uses over RCCL -- with a CPU shard built from the
oracle's arithmetic (float64).  Every rank's rows must match the
single-process oracle forward of the whole graph, for all four layer types,
on the periodic mesh in natural order (k-slabs) and in a shuffled order
(arbitrary halo lists)."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import grid_graph_np
from mignn.dist import (DistExchange, DistRequests, RangeLayout, Shard, build_local_layouts,
                        exchange_static, range_bounds, sharded_forward)
from mignn.gnn_model import FlowGNN
from mignn.synthetic import seeded_state_dict
from oracle import flowgnn_oracle as orc

NX, NY, NZ = 5, 4, 9          # 180 nodes


class OracleShard(Shard):
    """CPU stand-in for FlowGNNShard (test infrastructure): layer rows
    [rb, re) of the local order from the rank-local edge list, float64."""

    def __init__(self, sd, cfg, layout):
        self.sd = {k: v.double() for k, v in sd.items()}
        self.cfg, self.layout = cfg, layout
        self.num_layers, self.hidden_dim = cfg["num_layers"], cfg["hidden_dim"]
        src, dst = layout.edge_index
        if cfg["layer_type"] in ("GCN", "GAT"):       # one self-loop per node (PyG)
            keep = src != dst
            loops = torch.arange(layout.n_own)
            src, dst = torch.cat([src[keep], loops]), torch.cat([dst[keep], loops])
        self.src, self.dst = src, dst

    def setup(self, exchange):
        if self.cfg["layer_type"] == "GCN":
            lay = self.layout
            deg = torch.zeros(lay.n_total, dtype=torch.float64).index_add_(
                0, self.dst, torch.ones(self.dst.shape[0], dtype=torch.float64))
            dinv = torch.where(deg > 0, deg.pow(-0.5), torch.zeros_like(deg)).view(-1, 1)
            exchange_static([self], exchange, [dinv])       # ghost degrees from their owners
            self.w = dinv[self.src, 0] * dinv[self.dst, 0]

    def first_layer(self, x_own, buf):
        lay = self.layout
        buf[:lay.n_own] = (x_own.double()[lay.perm] @ self.sd["input_proj.weight"].T
                           + self.sd["input_proj.bias"])
        return 0

    def layer(self, i, x, out, rb, re):
        if re <= rb:
            return
        sel = (self.dst >= rb) & (self.dst < re)
        s, d = self.src[sel], self.dst[sel] - rb
        n = re - rb
        p = f"gnn_layers.{i}."
        sd, lt = self.sd, self.cfg["layer_type"]
        if lt == "GCN":
            h = x @ sd[p + "lin.weight"].T
            xn = torch.zeros(n, h.shape[1], dtype=x.dtype).index_add_(
                0, d, h[s] * self.w[sel].view(-1, 1)) + sd[p + "bias"]
        elif lt == "GIN":
            agg = torch.zeros(n, x.shape[1], dtype=x.dtype).index_add_(0, d, x[s])
            z = agg + (1 + float(sd[p + "eps"])) * x[rb:re]
            xn = torch.relu(z @ sd[p + "nn.0.weight"].T + sd[p + "nn.0.bias"])
            xn = xn @ sd[p + "nn.2.weight"].T + sd[p + "nn.2.bias"]
        elif lt == "GAT":
            W = sd[orc.gat_weight(sd, p)]
            C = W.shape[0] // 4
            h = (x @ W.T).view(-1, 4, C)
            a_s = (h * sd[p + "att_src"]).sum(-1)
            a_d = (h * sd[p + "att_dst"]).sum(-1)
            e = torch.nn.functional.leaky_relu(a_s[s] + a_d[d + rb], 0.2)
            alpha = orc.segment_softmax(e, d, n)
            xn = torch.zeros(n, 4, C, dtype=x.dtype).index_add_(
                0, d, h[s] * alpha.unsqueeze(-1)).mean(1) + sd[p + "bias"]
        else:
            C = sd[p + "lin_query.weight"].shape[0] // 4
            q = (x @ sd[p + "lin_query.weight"].T + sd[p + "lin_query.bias"]).view(-1, 4, C)
            k = (x @ sd[p + "lin_key.weight"].T + sd[p + "lin_key.bias"]).view(-1, 4, C)
            v = (x @ sd[p + "lin_value.weight"].T + sd[p + "lin_value.bias"]).view(-1, 4, C)
            alpha = orc.segment_softmax((q[d + rb] * k[s]).sum(-1) / C ** 0.5, d, n)
            xn = torch.zeros(n, 4, C, dtype=x.dtype).index_add_(
                0, d, v[s] * alpha.unsqueeze(-1)).mean(1)
            xn = xn + x[rb:re] @ sd[p + "lin_skip.weight"].T + sd[p + "lin_skip.bias"]
        b = f"batch_norms.{i}.module."
        y = orc.batch_norm_eval(x[rb:re] + xn, sd[b + "weight"], sd[b + "bias"],
                                sd[b + "running_mean"], sd[b + "running_var"])
        out[rb:re] = torch.relu(y)

    def output(self, x_own):
        sd = self.sd
        h = torch.relu(x_own @ sd["output_proj.0.weight"].T + sd["output_proj.0.bias"])
        h = torch.relu(h @ sd["output_proj.3.weight"].T + sd["output_proj.3.bias"])
        h = torch.relu(h @ sd["output_proj.6.weight"].T + sd["output_proj.6.bias"])
        y = h @ sd["output_proj.8.weight"].T + sd["output_proj.8.bias"]
        return y[self.layout.inv]                       # local order -> owned (global) order


class ChainedGatShard(OracleShard):
    """OracleShard for GAT whose layers take their attention logits from a
    [n_total, 8] tensor: layer i's owned rows' logits are formed from the
    previous layer's output rows (layer 0's from input_proj), and the ghost
    rows' logits arrive by the second halo exchange (halo_extra, tag
    TAG_EXTRA) -- FlowGNNShard's sharded GAT route, in float64."""

    def _logits(self, i, rows):
        p = f"gnn_layers.{i}."
        W = self.sd[orc.gat_weight(self.sd, p)]
        C = W.shape[0] // 4
        h = (rows @ W.T).view(-1, 4, C)
        return torch.cat([(h * self.sd[p + "att_src"]).sum(-1), (h * self.sd[p + "att_dst"]).sum(-1)], 1)

    def first_layer(self, x_own, buf):
        r = super().first_layer(x_own, buf)
        n = self.layout.n_own
        self.lg = torch.full((self.layout.n_total, 8), float("nan"), dtype=torch.float64)
        self.lg[:n] = self._logits(0, buf[:n])
        self.lg_next = torch.full_like(self.lg, float("nan"))
        return r

    def halo_extra(self, i):
        return self.lg

    def layer(self, i, x, out, rb, re):
        if re <= rb:
            return
        sel = (self.dst >= rb) & (self.dst < re)
        s, d = self.src[sel], self.dst[sel] - rb
        n = re - rb
        p = f"gnn_layers.{i}."
        sd = self.sd
        W = sd[orc.gat_weight(sd, p)]
        C = W.shape[0] // 4
        h = (x @ W.T).view(-1, 4, C)
        assert not torch.isnan(self.lg[s]).any()           # ghost logits landed
        e = torch.nn.functional.leaky_relu(self.lg[s, :4] + self.lg[d + rb, 4:], 0.2)
        alpha = orc.segment_softmax(e, d, n)
        xn = torch.zeros(n, 4, C, dtype=x.dtype).index_add_(
            0, d, h[s] * alpha.unsqueeze(-1)).mean(1) + sd[p + "bias"]
        b = f"batch_norms.{i}.module."
        y = orc.batch_norm_eval(x[rb:re] + xn, sd[b + "weight"], sd[b + "bias"],
                                sd[b + "running_mean"], sd[b + "running_var"])
        out[rb:re] = torch.relu(y)
        if i + 1 < self.num_layers:
            self.lg_next[rb:re] = self._logits(i + 1, out[rb:re])

    def end_layer(self, i):
        self.lg, self.lg_next = self.lg_next, self.lg
        self.lg_next.fill_(float("nan"))


def _graph(shuffle):
    x, ei = grid_graph_np(NX, NY, NZ)
    x, ei = torch.from_numpy(x), torch.from_numpy(ei)
    if shuffle:
        g = torch.Generator().manual_seed(3)
        perm = torch.randperm(x.shape[0], generator=g)        # old id -> new id
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(x.shape[0])
        x, ei = x[inv], perm[ei]
    return x, ei


def _cfg(lt):
    cfg = dict(hidden_dim=16, num_layers=3, layer_type=lt)
    sd = seeded_state_dict(FlowGNN(input_dim=3, output_dim=7, **cfg).state_dict(), seed=5)
    return cfg, sd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, layer_type, shuffle, outdir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.set_num_threads(1)
    chained = layer_type == "GAT_chained"
    cfg, sd = _cfg("GAT" if chained else layer_type)
    x, ei = _graph(shuffle)
    b = range_bounds(x.shape[0], world)
    mine = ei[:, (ei[1] >= b[rank]) & (ei[1] < b[rank + 1])]       # my in-edges, global ids
    lay = RangeLayout(mine, b, rank, DistRequests())
    sh = (ChainedGatShard if chained else OracleShard)(sd, cfg, lay)
    ex = DistExchange()
    sh.setup(ex)
    (y,) = sharded_forward([sh], ex, [x[b[rank]:b[rank + 1]].double()])
    torch.save(y, os.path.join(outdir, f"y{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("shuffle", [False, True])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("layer_type", ["GCN", "GIN", "GAT", "Transformer", "GAT_chained"])
def test_sharded_forward_matches_single_process(world, layer_type, shuffle):
    """GAT_chained: the sharded GAT route's second exchange (ghost logits,
    tag TAG_EXTRA) posted beside the feature halo at every layer."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), layer_type, shuffle, d), nprocs=world,
                 join=True)
        ys = [torch.load(os.path.join(d, f"y{r}.pt"), weights_only=True) for r in range(world)]
    cfg, sd = _cfg("GAT" if layer_type == "GAT_chained" else layer_type)
    x, ei = _graph(shuffle)
    ref = orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float64)
    got = torch.cat(ys, 0)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() < 1e-12


def test_layout_natural_order_is_kslabs():
    """Natural order: rank 1 of 3 owns k-planes 3..5; its ghosts are exactly the
    two neighbour planes (periodic), interior rows = planes 4, boundary = 3, 5."""
    x, ei = _graph(False)
    b = range_bounds(x.shape[0], 3)
    edges = [ei[:, (ei[1] >= b[r]) & (ei[1] < b[r + 1])] for r in range(3)]
    lays = build_local_layouts(edges, b)
    lay = lays[1]
    plane = NX * NY
    assert (lay.n_own, lay.n_ghost, lay.n_int) == (3 * plane, 2 * plane, plane)
    assert torch.equal(lay.ghost_gid, torch.cat([torch.arange(2 * plane, 3 * plane),
                                                 torch.arange(6 * plane, 7 * plane)]))
    assert lay.ghost_ptr == [0, plane, plane, 2 * plane]
    # interior rows first: owned offsets of plane 4 (offsets 20..39), then 3 and 5
    assert torch.equal(torch.sort(lay.perm[:plane]).values, torch.arange(plane, 2 * plane))
    # every rank's send list to a peer = exactly what that peer asked for
    for r, lr in enumerate(lays):
        for q, idx in lr.send_idx.items():
            sent = lr.perm[idx.long()] + lr.lo
            want = lays[q].ghost_gid[lays[q].ghost_ptr[r]:lays[q].ghost_ptr[r + 1]]
            assert torch.equal(sent, want)
    # local edge ids point at the right global nodes
    glob = torch.cat([lay.perm + lay.lo, lay.ghost_gid])
    assert torch.equal(glob[lay.edge_index], edges[1])


def test_layout_rejects_foreign_destinations():
    x, ei = _graph(False)
    b = range_bounds(x.shape[0], 2)
    with pytest.raises(ValueError):
        build_local_layouts([ei, ei], b)
