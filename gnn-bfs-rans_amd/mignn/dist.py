"""Node-range (k-slab) partitioning of a mesh across GPUs with a 1-hop halo
exchange per layer.  One process per GPU; the exchange is
point-to-point `torch.distributed` (backend "nccl" == RCCL over xGMI on
MI355X, "gloo" on the CPU test path).

Layout per rank (natural node order, i fastest, k slowest):
    rows [0, n_own)                 owned nodes: k-planes [r*nzl, (r+1)*nzl)
    rows [n_own, n_own+plane)       lower ghost plane  (global plane r*nzl - 1)
    rows [n_own+plane, n_own+2pl)   upper ghost plane  (global plane (r+1)*nzl)
A slab's halo is one contiguous i-j plane per side, so nothing is packed: the
sends are x[0:plane] (to the lower peer, its upper ghost) and
x[n_own-plane:n_own] (to the upper peer, its lower ghost).  The grid is
periodic in k, so every rank has exactly two peers (one peer, twice, at P=2).

Per layer: post the exchange, run the interior rows [plane, n_own-plane) --
which read no ghost row -- on the compute stream while RCCL moves the planes,
wait, then run the two boundary planes.  GCN additionally needs the ghost
nodes' deg^-1/2, exchanged once when the graph is set up.  Eval-mode
BatchNorm needs no communication.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

TAG_TO_LOWER = 11   # my first plane -> lower peer's upper ghost
TAG_TO_UPPER = 12   # my last plane  -> upper peer's lower ghost


@dataclass
class SlabPartition:
    nx: int
    ny: int
    nz_local: int
    rank: int
    world: int

    @property
    def plane(self) -> int:
        return self.nx * self.ny

    @property
    def nz_total(self) -> int:
        return self.nz_local * self.world

    @property
    def n_own(self) -> int:
        return self.plane * self.nz_local

    @property
    def n_total(self) -> int:
        return self.n_own + (2 * self.plane if self.world > 1 else 0)

    @property
    def lower_peer(self) -> int:
        return (self.rank - 1) % self.world

    @property
    def upper_peer(self) -> int:
        return (self.rank + 1) % self.world

    @property
    def z_begin(self) -> int:
        return self.rank * self.nz_local

    def interior(self):
        return (self.plane, self.n_own - self.plane)

    def boundary(self):
        return [(0, self.plane), (self.n_own - self.plane, self.n_own)]

    def localize(self, edge_index_global: torch.Tensor) -> torch.Tensor:
        """Map global node ids of this slab's edges to local rows (own, then
        lower ghost plane, then upper ghost plane)."""
        if self.world == 1:
            return edge_index_global
        pl = self.plane
        base = self.z_begin * pl
        g = edge_index_global
        lo_plane = ((self.z_begin - 1) % self.nz_total) * pl
        up_plane = ((self.z_begin + self.nz_local) % self.nz_total) * pl
        local = g - base
        own = (g >= base) & (g < base + self.n_own)
        lo = (g >= lo_plane) & (g < lo_plane + pl) & ~own
        up = (g >= up_plane) & (g < up_plane + pl) & ~own
        local = torch.where(lo, g - lo_plane + self.n_own, local)
        local = torch.where(up, g - up_plane + self.n_own + pl, local)
        bad = ~(own | lo | up)
        if bool(bad.any()):
            raise ValueError("edge references a node outside the slab and its 1-hop halo")
        return local


def halo_exchange(buf: torch.Tensor, part: SlabPartition, group=None) -> List:
    """Post the two-plane exchange on `buf` ([n_total, F]); returns works to wait on."""
    if part.world == 1:
        return []
    pl, n = part.plane, part.n_own
    ops = [
        dist.P2POp(dist.isend, buf[0:pl], part.lower_peer, group, TAG_TO_LOWER),
        dist.P2POp(dist.irecv, buf[n + pl:n + 2 * pl], part.upper_peer, group, TAG_TO_LOWER),
        dist.P2POp(dist.isend, buf[n - pl:n], part.upper_peer, group, TAG_TO_UPPER),
        dist.P2POp(dist.irecv, buf[n:n + pl], part.lower_peer, group, TAG_TO_UPPER),
    ]
    return dist.batch_isend_irecv(ops)


class LayerExecutor:
    """What the sharded driver needs from a compute backend."""

    num_layers: int
    hidden_dim: int
    overlap_ok: bool = True

    def input_proj(self, x_own: torch.Tensor, out: torch.Tensor) -> None: ...
    def layer(self, i: int, x: torch.Tensor, out: torch.Tensor, rb: int, re: int) -> None: ...
    def output(self, x_own: torch.Tensor) -> torch.Tensor: ...


def sharded_forward(ex: LayerExecutor, part: SlabPartition, x_own: torch.Tensor, group=None,
                    timing_hook: Optional[Callable] = None) -> torch.Tensor:
    """Forward of one rank's slab; returns the rank's [n_own, out] rows."""
    H = ex.hidden_dim
    dev = x_own.device
    a = torch.empty((part.n_total, H), dtype=x_own.dtype, device=dev)
    b = torch.empty_like(a)
    ex.input_proj(x_own, a[:part.n_own])
    cur, nxt = a, b
    for i in range(ex.num_layers):
        works = halo_exchange(cur, part, group)
        if part.world > 1 and ex.overlap_ok:
            rb, re = part.interior()
            ex.layer(i, cur, nxt, rb, re)
            for w in works:
                w.wait()
            for rb, re in part.boundary():
                ex.layer(i, cur, nxt, rb, re)
        else:
            for w in works:
                w.wait()
            ex.layer(i, cur, nxt, 0, part.n_own)
        cur, nxt = nxt, cur
    return ex.output(cur[:part.n_own])


class FlowGNNExecutor(LayerExecutor):
    """GPU executor: FlowGNN's native layers on a rank-local CSR."""

    def __init__(self, model, part: SlabPartition, edge_index_local: torch.Tensor, group=None):
        self.model = model
        self.part = part
        self.group = group
        self.edge_index_local = edge_index_local
        self.num_layers = model.num_layers
        self.hidden_dim = model.hidden_dim
        self.overlap_ok = model.layer_type != "GAT"   # GAT logits read ghost rows
        self.build_graph()

    def build_graph(self):
        """Rank-local CSR (+ GCN norm with the ghost rows' true degrees)."""
        from ._lib import CSR_ONE_SELF_LOOP, CSR_VERBATIM
        from .gnn_model import build_csr

        part = self.part
        mode = CSR_ONE_SELF_LOOP if self.model.layer_type in ("GCN", "GAT") else CSR_VERBATIM
        self.csr = build_csr(self.edge_index_local, part.n_total, mode)
        if self.csr.dinv is not None and part.world > 1:
            # ghost rows' true deg^-1/2 comes from their owner
            d = self.csr.dinv[:part.n_total].view(-1, 1)
            for w in halo_exchange(d, part, self.group):
                w.wait()
            self.csr.compute_gcn_weights(0, part.n_own)   # entries of owned rows, true ghost dinv

    def input_proj(self, x_own, out):
        self.model._input_proj(x_own.contiguous(), out)

    def layer(self, i, x, out, rb, re):
        self.model._layer(i, self.model.gnn_layers[i], self.csr, x, out, rb, re)

    def output(self, x_own):
        out = torch.empty((x_own.shape[0], self.model.output_dim), dtype=torch.float32,
                          device=x_own.device)
        tmp = torch.empty_like(x_own)
        self.model._output_mlp(x_own, tmp, out)   # x_own is scratch after the last layer
        return out
