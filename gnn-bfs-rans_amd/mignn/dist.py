"""Node-range partitioning of any graph across GPUs with a 1-hop halo
exchange per layer (north star: "large meshes shard by
contiguous node-range across the 8 GPUs ... with RCCL halo exchange of
boundary node features").  One process per GPU; the exchange is
point-to-point `torch.distributed` (backend "nccl" == RCCL over xGMI on
MI355X, "gloo" on the CPU test path).

Partition: rank r owns the global node ids [bounds[r], bounds[r+1]) and the
in-edges of those nodes (the CSR rows it computes).  `RangeLayout` derives,
from this rank's edges alone plus one exchange of requests:
  * ghosts  : the sources of its in-edges owned by other ranks, sorted by
              global id (so grouped by owner rank: one contiguous slice of the
              activation buffer per peer -- received rows land in place);
  * send lists: the owned rows each peer asked for (packed with
              mignn_rows_gather on the GPU);
  * a local order of the owned rows: interior rows (no ghost source) first,
    boundary rows last, each group in the mesh locality order
    (mignn_locality_order on the cell centres) when one is given -- so the
    interior rows run while RCCL moves the halo, as one contiguous launch.
Activation buffers are [n_own + n_ghost, H]: owned rows (local order), then
the ghosts.  Static per-graph data crosses once: GCN's ghost deg^-1/2 and the
ghost cell centres (the fused input_proj + GCN layer 0 reads coordinates, so
layer 0 needs no feature exchange at all).

`sharded_forward` drives any list of shards with a halo-exchange object:
`DistExchange` (this rank's shard, torch.distributed P2P) or `LocalExchange`
(several shards in one process, the halo filled by device-to-device row
copies) -- the same per-layer code either way, which is what the
single-process multi-shard GPU tests exercise.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

TAG_HALO = 17
TAG_EXTRA = 18          # the second per-layer exchange (sharded GAT: ghost logits)


# ---------------------------------------------------------------------------
# layout
# ---------------------------------------------------------------------------

def range_bounds(num_nodes: int, world: int) -> List[int]:
    """Contiguous node ranges [r*N/P, (r+1)*N/P)."""
    return [(r * num_nodes) // world for r in range(world + 1)]


def _nonzero_known(t: torch.Tensor, count: int) -> torch.Tensor:
    """Indices of the nonzero entries of a 1-D tensor whose count is already
    known on the host (no second device->host sync)."""
    try:
        return torch.nonzero_static(t, size=count).flatten()
    except (RuntimeError, NotImplementedError):
        return torch.nonzero(t).flatten()


class RangeLayout:
    """One rank's part of a contiguous node-range partition (see the module
    docstring).  `edge_index` [2, E_r] holds global ids of the edges whose
    destination this rank owns (int64, any device); `pos` [n_own, >=3]
    optional cell centres of the owned nodes (caller order = global id
    order), used only to pick the locality order via `order_fn(pos, ei)`
    -> perm (local position -> owned offset), or (perm, info) for the
    column order (mignn_locality_order_cols' info, kept as `order_info`: the
    window GCN kernel's route on the rank-local CSR).

    The `ei` handed to `order_fn` is NOT this rank's adjacency: it is a
    strided sample of at most 2^18 of its edges ([2, <= 2^18], int64, local
    owned offsets), and an edge whose source is a ghost has its source set to
    -1.  The locality orders only estimate the mesh spacing from it
    (mignn_locality_order skips the -1 entries).  An order_fn that needs the
    full owned-to-owned adjacency (RCM, a graph partitioner) must not rely on
    it: build that from `edge_index` before constructing the layout."""

    def __init__(self, edge_index: torch.Tensor, bounds: Sequence[int], rank: int,
                 requests: "RequestExchange", pos: Optional[torch.Tensor] = None,
                 order_fn: Optional[Callable] = None):
        dev = edge_index.device
        self.rank, self.world = rank, len(bounds) - 1
        self.bounds = [int(b) for b in bounds]
        lo, hi = self.bounds[rank], self.bounds[rank + 1]
        N = self.bounds[-1]
        self.lo, self.hi, self.n_own = lo, hi, hi - lo
        src, dst = edge_index[0].long(), edge_index[1].long()
        E = int(src.numel())
        if self.n_own <= 0 and E > 0:
            # (checked before any device indexing: a rank that owns no rows
            # cannot own a destination either)
            raise ValueError("edge_index holds an edge whose destination this rank does not own")
        # ghost marks over the global ids (+1 dummy slot), boundary marks over
        # the owned rows, id checks: one native pass on the device
        mark = torch.zeros(N + 1, dtype=torch.int32, device=dev)
        bmark = torch.zeros(self.n_own + 1, dtype=torch.int8, device=dev)
        if dev.type == "cuda":
            from . import _lib
            bad = torch.zeros(2, dtype=torch.int32, device=dev)
            if E:
                ei64 = edge_index if (edge_index.dtype == torch.int64 and edge_index.is_contiguous()) \
                    else torch.stack([src, dst])
                _lib.check(_lib.lib().mignn_range_mark(
                    _lib.ptr(ei64), E, lo, hi, N, _lib.ptr(mark), _lib.ptr(bmark), _lib.ptr(bad),
                    _lib.stream(dev)), "mignn_range_mark")
            bad_dst, bad_src = bad[0].bool(), bad[1].bool()
        else:
            own_src = (src >= lo) & (src < hi)
            if E:
                mark.index_fill_(0, torch.where(own_src, torch.full_like(src, N), src.clamp(0, N)), 1)
                # (a flag fill through a dummy slot: an index_add over every
                # edge serialised on a mesh's runs of equal destinations)
                bmark.index_fill_(0, torch.where(own_src, torch.full_like(dst, self.n_own),
                                                 (dst - lo).clamp(0, max(self.n_own, 0))), 1)
                dmin, dmax = torch.aminmax(dst)
                smin, smax = torch.aminmax(src)
                bad_dst, bad_src = (dmin < lo) | (dmax >= hi), (smin < 0) | (smax >= N)
            else:
                bad_dst = bad_src = torch.zeros((), dtype=torch.bool, device=dev)
        mark[N] = 0
        csum = torch.cumsum(mark, 0)
        b = torch.tensor(self.bounds, dtype=torch.int64, device=dev)
        ends = torch.where(b > 0, csum[(b - 1).clamp(min=0)], torch.zeros_like(b))
        counts = ends[1:] - ends[:-1]                        # ghosts per owner rank
        # boundary rows: owned destinations with a ghost source
        boundary = bmark[:self.n_own] > 0
        # every host-side size in ONE device->host transfer
        host = torch.cat([torch.stack([bad_dst.long(), bad_src.long(), (~boundary).sum()]),
                          counts]).cpu().tolist()
        if host[0]:
            raise ValueError("edge_index holds an edge whose destination this rank does not own")
        if host[1]:
            raise ValueError("edge_index holds a source outside [0, N)")
        self.n_int = int(host[2])
        counts = [int(c) for c in host[3:]]
        self.ghost_ptr = [0]
        for c in counts:
            self.ghost_ptr.append(self.ghost_ptr[-1] + c)
        self.n_ghost = self.ghost_ptr[-1]
        self.n_total = self.n_own + self.n_ghost
        # ghosts: sorted global ids == grouped by owner rank (contiguous ranges)
        ghost = _nonzero_known(mark[:N], self.n_ghost)
        self.ghost_gid = ghost
        self.order_info = None
        # local order of the owned rows: interior first, boundary last
        if order_fn is not None and pos is not None and self.n_own > 0:
            # the locality order reads edges only for its spacing estimate, a
            # strided sample of <= 2^18 of them (mignn_locality_order): that
            # sample of this rank's edges in local ids, the ghost-source ones
            # marked invalid (-1, skipped by the estimate)
            ns = min(E, 1 << 18)
            idx = (torch.arange(ns, device=dev) * E) // max(ns, 1)
            s_i = src[idx]
            s_loc = torch.where((s_i >= lo) & (s_i < hi), s_i - lo, torch.full_like(idx, -1))
            got = order_fn(pos, torch.stack([s_loc, dst[idx] - lo]))
            if isinstance(got, tuple):
                got, self.order_info = got
            base = got.long()
        else:
            base = torch.arange(self.n_own, device=dev)
        # interior first, boundary last, each in the base order: a stable
        # partition by prefix sums (a stable sort of the 0/1 keys cost 0.7 ms)
        bnd = boundary[base]
        ci = torch.cumsum(~bnd, 0, dtype=torch.int32)
        perm = torch.empty_like(base)
        self.inv = torch.empty_like(base)
        if dev.type == "cuda" and self.n_own > 0:
            # (one pass: destination, perm and inv scatters -- mignn_range_partition)
            from . import _lib
            base = base.contiguous()
            _lib.check(_lib.lib().mignn_range_partition(
                _lib.ptr(base), _lib.ptr(boundary.contiguous()), _lib.ptr(ci), self.n_own, self.n_int,
                _lib.ptr(perm), _lib.ptr(self.inv), _lib.stream(dev)), "mignn_range_partition")
        else:
            cb = torch.arange(1, self.n_own + 1, device=dev, dtype=torch.int32) - ci
            dest = torch.where(bnd, self.n_int + cb - 1, ci - 1).long()
            perm[dest] = base                                      # local position -> owned offset
            self.inv[perm] = torch.arange(self.n_own, device=dev)
        self.perm = perm
        # local edge list: owned -> local position, ghost -> n_own + ghost
        # index (the ghost's rank among the marked ids: the prefix sum above).
        # On the device it is not written here: build_csr maps the global ids
        # inside the CSR build (mignn_csr_build_range); `edge_index`
        # materialises it on first use (mignn_range_relabel)
        self._ei_global = self._ghost_rank = None
        self._edge_index: Optional[torch.Tensor] = None
        if dev.type == "cuda" and E > 0:
            self._ei_global = edge_index if (edge_index.dtype == torch.int64
                                             and edge_index.is_contiguous()) \
                else torch.stack([src, dst])
            self._ghost_rank = csum
        else:
            own_src = (src >= lo) & (src < hi)
            lsrc = torch.where(own_src, self.inv[(src - lo).clamp(0, max(self.n_own - 1, 0))],
                               self.n_own - 1 + csum[src.clamp(0, N)])
            self._edge_index = torch.stack([lsrc, self.inv[dst - lo]])
        # send lists: every peer's ghost requests, answered with my local rows
        req = {q: ghost[self.ghost_ptr[q]:self.ghost_ptr[q + 1]]
               for q in range(self.world) if q != rank and counts[q] > 0}
        got = requests.exchange(rank, req)
        self.send_idx: Dict[int, torch.Tensor] = {
            q: self.inv[ids.to(dev).long() - lo].to(torch.int32) for q, ids in got.items()
            if ids.numel() > 0}

    @property
    def edge_index(self) -> torch.Tensor:
        """The rank-local edge list [2, E_r] (int64): a source in [lo, hi) ->
        its local position, a ghost -> n_own + its ghost index; a destination
        -> its local position."""
        if self._edge_index is None:
            from . import _lib
            ei = self._ei_global
            E = int(ei.shape[1])
            out = torch.empty((2, E), dtype=torch.int64, device=ei.device)
            _lib.check(_lib.lib().mignn_range_relabel(
                _lib.ptr(ei), E, self.lo, self.hi, _lib.ptr(self.inv), _lib.ptr(self._ghost_rank),
                self.n_own, _lib.ptr(out), _lib.stream(ei.device)), "mignn_range_relabel")
            self._edge_index = out
        return self._edge_index

    def build_csr(self, mode: int):
        """This rank's local CSR (mignn.gnn_model.build_csr of `edge_index`,
        n_total nodes); on the device straight from the global-id in-edges
        (mignn_csr_build_range: the local list is never written)."""
        from .gnn_model import build_csr, build_csr_range
        if self._edge_index is None and self._ei_global is not None:
            return build_csr_range(self._ei_global, self.bounds[-1], self.lo, self.hi, self.inv,
                                   self._ghost_rank, self.n_total, mode)
        return build_csr(self.edge_index, self.n_total, mode)

    def ghost_slice(self, q: int) -> slice:
        return slice(self.n_own + self.ghost_ptr[q], self.n_own + self.ghost_ptr[q + 1])

    def peers(self) -> List[int]:
        return sorted(set(self.send_idx) | {q for q in range(self.world)
                                            if q != self.rank and self.ghost_ptr[q + 1] > self.ghost_ptr[q]})


class RequestExchange:
    """Setup-time exchange of ghost id lists (who needs which of my rows)."""

    def exchange(self, rank: int, req: Dict[int, torch.Tensor]) -> Dict[int, torch.Tensor]:
        raise NotImplementedError


def _comm_device(group=None, device=None) -> torch.device:
    """Where a process group's tensors must live: the given device, else the
    current ROCm device for nccl (RCCL), else the CPU (gloo)."""
    if device is not None:
        return torch.device(device)
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class DistRequests(RequestExchange):
    """torch.distributed: counts by all_gather, id lists by P2P (on the
    group's device: the current ROCm device under nccl, the CPU under gloo)."""

    def __init__(self, group=None, device=None):
        self.group, self.device = group, device

    def exchange(self, rank, req):
        world = dist.get_world_size(self.group)
        dev = _comm_device(self.group, self.device)
        mine = torch.zeros(world, dtype=torch.int64, device=dev)
        for q, ids in req.items():
            mine[q] = ids.numel()
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine, group=self.group)
        ops, got = [], {}
        for q in range(world):
            if q == rank:
                continue
            if q in req and req[q].numel():
                ops.append(dist.P2POp(dist.isend, req[q].to(dev).contiguous(), q, self.group, TAG_HALO))
            n = int(allc[q][rank])
            if n:
                got[q] = torch.empty(n, dtype=torch.int64, device=dev)
                ops.append(dist.P2POp(dist.irecv, got[q], q, self.group, TAG_HALO))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return got


class LocalRequests(RequestExchange):
    """Several ranks' layouts built in one process: requests are handed over
    directly (build rank 0..P-1 in order with the same object, then call
    `resolve` -- see build_local_layouts)."""

    def __init__(self):
        self.posted: Dict[int, Dict[int, torch.Tensor]] = {}

    def exchange(self, rank, req):
        self.posted[rank] = req
        return {}


def build_local_layouts(edge_lists: Sequence[torch.Tensor], bounds: Sequence[int],
                        pos: Optional[Sequence[torch.Tensor]] = None,
                        order_fn: Optional[Callable] = None) -> List[RangeLayout]:
    """All P layouts of a partition in one process (LocalExchange shards)."""
    reqs = LocalRequests()
    lays = [RangeLayout(ei, bounds, r, reqs, None if pos is None else pos[r], order_fn)
            for r, ei in enumerate(edge_lists)]
    for r, lay in enumerate(lays):          # answer the requests posted to each rank
        lay.send_idx = {q: lay.inv[reqs.posted[q][r].long() - lay.lo].to(torch.int32)
                        for q in range(len(lays)) if q != r and r in reqs.posted.get(q, {})
                        and reqs.posted[q][r].numel() > 0}
    return lays


# ---------------------------------------------------------------------------
# halo exchange
# ---------------------------------------------------------------------------

def _gather_rows(src: torch.Tensor, idx: torch.Tensor, dst: torch.Tensor):
    """dst[r] = src[idx[r]] (mignn_rows_gather on a ROCm device)."""
    if src.is_cuda:
        from . import _lib
        _lib.check(_lib.lib().mignn_rows_gather(
            _lib.ptr(src), src.stride(0), _lib.ptr(idx), idx.numel(), src.shape[1],
            _lib.ptr(dst), dst.stride(0), _lib.stream(src.device)), "mignn_rows_gather")
    else:
        torch.index_select(src, 0, idx.long(), out=dst)


class DistExchange:
    """This rank's halo over torch.distributed P2P: pack each peer's rows,
    isend; irecv straight into the peer's ghost slice.  Under a backend
    whose P2P takes host tensors only (gloo) with device activations, the
    packed rows and the ghost slices are staged through host memory (the
    multi-process GPU test on a one-GPU box); under nccl (RCCL) the device
    tensors go straight to the transport."""

    def __init__(self, group=None):
        self.group = group
        self._staged = None
        # per-peer pack buffers, one per (peer, width, dtype, device), grown
        # when a layout needs more rows and handed out as a view of the first
        # n rows -- reused by every layer (a layer's sends complete -- wait()
        # -- before the next layer packs), and by rebuilt layouts of other
        # sizes without a buffer per distinct ghost count
        self._pack: Dict[tuple, torch.Tensor] = {}

    def _stage(self, buf) -> bool:
        if self._staged is None:
            self._staged = dist.get_backend(self.group) != "nccl"
        return self._staged and buf.is_cuda

    def _pack_buf(self, q, n, buf):
        key = (q, buf.shape[1], buf.dtype, str(buf.device))
        pk = self._pack.get(key)
        if pk is None or pk.shape[0] < n:
            pk = self._pack[key] = torch.empty((n, buf.shape[1]), dtype=buf.dtype, device=buf.device)
        return pk[:n]

    def start(self, shards, bufs, tag: int = TAG_HALO):
        (sh,), (buf,) = shards, bufs
        lay = sh.layout
        stage = self._stage(buf)
        ops, unstage = [], []
        for q in lay.peers():
            if q in lay.send_idx:
                idx = lay.send_idx[q]
                pk = self._pack_buf(q, idx.numel(), buf)
                _gather_rows(buf, idx, pk)
                ops.append(dist.P2POp(dist.isend, pk.cpu() if stage else pk, q, self.group, tag))
            sl = lay.ghost_slice(q)
            if sl.stop > sl.start:
                dst = buf[sl]
                if stage:
                    host = torch.empty(dst.shape, dtype=dst.dtype)
                    unstage.append((dst, host))
                    dst = host
                ops.append(dist.P2POp(dist.irecv, dst, q, self.group, tag))
        return (dist.batch_isend_irecv(ops) if ops else [], unstage)

    def wait(self, handle):
        works, unstage = handle
        for w in works:
            w.wait()
        for dst, host in unstage:
            dst.copy_(host)


class LocalExchange:
    """All shards in one process: every send list is copied device-to-device
    into the receiving shard's ghost slice (the stream orders the copies
    before the boundary rows' launches)."""

    def start(self, shards, bufs, tag: int = TAG_HALO):
        for r, sh in enumerate(shards):
            for q, idx in sh.layout.send_idx.items():
                dst = bufs[q][shards[q].layout.ghost_slice(r)]
                _gather_rows(bufs[r], idx, dst)
        return None

    def wait(self, handle):
        pass


def exchange_static(shards, exchange, tensors: List[torch.Tensor]):
    """One-off halo fill of per-row static data (owned rows already written)."""
    exchange.wait(exchange.start(shards, tensors))


# ---------------------------------------------------------------------------
# driver
# ---------------------------------------------------------------------------

class Shard:
    """What sharded_forward needs from a compute backend for one rank."""

    layout: RangeLayout
    num_layers: int
    hidden_dim: int

    def first_layer(self, x_own: torch.Tensor, buf: torch.Tensor) -> int:
        """Write layer-0 input (or, fused, layer 0's output) rows [0, n_own)
        of buf; return the index of the first layer still to run."""
        raise NotImplementedError

    def layer(self, i: int, x: torch.Tensor, out: torch.Tensor, rb: int, re: int) -> None: ...

    def halo_rows(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """The rows layer i reads from the ghosts (default: its input x)."""
        return x

    def halo_extra(self, i: int) -> Optional[torch.Tensor]:
        """A second per-row tensor whose ghost rows travel with layer i's
        feature halo (sharded GAT: the logits the previous layer's epilogue
        formed), or None.  Must be decided by the model configuration and i
        alone -- the same on every rank -- since every rank posts (or skips)
        the second exchange on its own (tag TAG_EXTRA)."""
        return None

    def end_layer(self, i: int) -> None:
        """Layer i's rows are all written."""

    def before_halo(self, i: int, x: torch.Tensor) -> None:
        """Work of layer i that needs only owned rows (before the halo lands)."""

    def after_halo(self, i: int, x: torch.Tensor) -> None:
        """Work of layer i on the ghost rows once they have landed."""

    def output(self, x_own: torch.Tensor) -> torch.Tensor: ...


def sharded_forward(shards: List[Shard], exchange, xs_own: List[torch.Tensor]) -> List[torch.Tensor]:
    """Forward of every shard in `shards` (one for DistExchange); returns each
    shard's [n_own, out] rows in its owned-node (global id) order.
    Per layer: post the halo exchange, run the interior rows, wait, run the
    ghost-dependent work and the boundary rows."""
    bufs_a, bufs_b, starts = [], [], []
    for sh, x in zip(shards, xs_own):
        lay = sh.layout
        a = torch.empty((lay.n_total, sh.hidden_dim), dtype=torch.float32 if x.is_cuda else x.dtype,
                        device=x.device)
        bufs_a.append(a)
        bufs_b.append(torch.empty_like(a))
        starts.append(sh.first_layer(x, a))
    first = starts[0]
    assert all(s == first for s in starts)
    cur, nxt = bufs_a, bufs_b
    for i in range(first, shards[0].num_layers):
        h = exchange.start(shards, [sh.halo_rows(i, x) for sh, x in zip(shards, cur)])
        extra = [sh.halo_extra(i) for sh in shards]
        if any(e is not None for e in extra) and not all(e is not None for e in extra):
            raise RuntimeError(f"layer {i}: halo_extra differs between shards")
        h2 = exchange.start(shards, extra, tag=TAG_EXTRA) if extra[0] is not None else None
        for sh, x, o in zip(shards, cur, nxt):
            sh.before_halo(i, x)
            sh.layer(i, x, o, 0, sh.layout.n_int)
        exchange.wait(h)
        if h2 is not None:
            exchange.wait(h2)
        for sh, x, o in zip(shards, cur, nxt):
            sh.after_halo(i, x)
            sh.layer(i, x, o, sh.layout.n_int, sh.layout.n_own)
            sh.end_layer(i)
        cur, nxt = nxt, cur
    return [sh.output(x[:sh.layout.n_own]) for sh, x in zip(shards, cur)]


class FlowGNNShard(Shard):
    """GPU shard: FlowGNN's native layers on the rank-local CSR (owned rows
    in the interior/boundary locality order, then the ghosts).  Layer 0 is
    composed with input_proj from the coordinates as on one GPU (GCN, GIN
    H=256, GAT, TransformerConv: FlowGNN._layer0_kind), with the ghost
    coordinates exchanged once per layout, so layer 0 moves no feature halo.
    One difference from the 1-GPU route: sharded GAT forms every next
    layer's logits in the layer's epilogue -- layer 0's collapsed kernel
    included (mignn_gat_layer0_coords with logits_next) -- and the ghost
    rows' logits travel in a second exchange (tag TAG_EXTRA), so no rank runs
    a logit GEMV on ghost rows; the 1-GPU forward forms layer 1's logits by
    a GEMV (measured faster there).  The two routes agree up to fp32
    summation order."""

    def __init__(self, model, layout: RangeLayout, x_own: torch.Tensor):
        self.model, self.layout = model, layout
        self.num_layers, self.hidden_dim = model.num_layers, model.hidden_dim
        self.x_own = x_own
        self.csr = None
        self.pos = None
        self.kind0 = model._layer0_kind()
        self.chain = (model.layer_type == "GAT" and model.precision == "f16x3"
                      and model.gat_next_logits)
        self.lg = None          # [n_total, 2 heads] logits of the layer about to run
        self.lg_ready = False   # its owned rows written by the previous layer
        self.lg_next = None
        self.codes = None       # layer 0's row codes [n_total, 8] when layer 1 reads them

    def setup(self, exchange, shards: List["FlowGNNShard"]):
        """Per-graph setup of every shard in `shards` (collective over them):
        setup_graph (local CSRs, GCN ghost degrees + edge weights) and
        setup_static (ghost cell centres for the composed layer 0)."""
        self.setup_graph(exchange, shards)
        self.setup_static(exchange, shards)

    def setup_graph(self, exchange, shards: List["FlowGNNShard"]):
        """The rank-local CSRs on the device, GCN's ghost deg^-1/2 from their
        owners and the gcn_norm edge weights -- what FlowGNN.forward rebuilds
        from edge_index when its CSR cache is off (the bench's per-step graph
        setup)."""
        from ._lib import CSR_ONE_SELF_LOOP, CSR_VERBATIM
        m = self.model
        mode = CSR_ONE_SELF_LOOP if m.layer_type in ("GCN", "GAT") else CSR_VERBATIM
        for sh in shards:
            sh.csr = sh.layout.build_csr(mode)
            # (the column order: the window kernel's route; its plans cover
            # row ranges -- interior, boundary -- so they take the contiguous
            # chunk schedule, the info only marks the order)
            sh.csr.order_info = sh.layout.order_info
        if shards[0].csr.dinv is not None:
            # ghost rows' true deg^-1/2 comes from their owners
            exchange_static(shards, exchange, [sh.csr.dinv[:sh.layout.n_total].view(-1, 1)
                                               for sh in shards])
            for sh in shards:
                sh.csr.compute_gcn_weights(0, sh.layout.n_own)

    def setup_static(self, exchange, shards: List["FlowGNNShard"]):
        """Static per-layout data: the ghost rows' cell centres (the composed
        layer 0 reads coordinates, so layer 0 needs no feature exchange)."""
        m = self.model
        if self.kind0 is not None:
            D = m.input_dim
            poss = []
            for sh in shards:
                p = torch.zeros((sh.layout.n_total, D), dtype=torch.float32, device=sh.x_own.device)
                p[:sh.layout.n_own] = sh.x_own.float()[sh.layout.perm]
                poss.append(p)
            exchange_static(shards, exchange, poss)
            for sh, p in zip(shards, poss):
                sh.pos = p

    def _logits_buf(self):
        return torch.empty((self.layout.n_total, 2 * _heads()), dtype=torch.float32,
                           device=self.x_own.device)

    def first_layer(self, x_own, buf):
        m, lay = self.model, self.layout
        self.lg, self.lg_ready, self.lg_next = None, False, None
        self.codes = None
        if self.kind0 == "gcn" and m._use_gcn_codes(self.csr):
            # layer 0 as row codes (the 1-GPU route, FlowGNN._gcn_layers01_codes):
            # layer 1's halo moves the ghosts' 32-B codes instead of their rows
            self.codes = torch.zeros((lay.n_total, 8), dtype=torch.float32, device=buf.device)
            m._gcn_layer0_codes(self.csr, self.pos, 0, lay.n_own, self.codes)
            return 1
        if self.kind0 is not None:
            lg = None
            if self.kind0 == "gat" and self.chain and self.num_layers > 1:
                lg = self._logits_buf()
            m._layer0(self.kind0, self.csr, self.pos, 0, lay.n_own, buf, logits_next=lg)
            self.lg, self.lg_ready = lg, lg is not None
            return 1
        xo = x_own.contiguous().float()
        m._input_proj(xo, buf[:lay.n_own], rows=lay.perm.to(torch.int32))
        return 0

    def halo_rows(self, i, x):
        return self.codes if (i == 1 and self.codes is not None) else x

    def halo_extra(self, i):
        return self.lg if self.lg_ready else None

    def _wlog(self, i):
        layer = self.model.gnn_layers[i]
        return self.model._cached("gat", i, (layer.lin.weight, layer.att_src, layer.att_dst),
                                  lambda: self.model._gat_weights(layer))[0]

    def before_halo(self, i, x):
        """GAT without logits from the previous layer: the owned rows'
        logits, computed while the features move."""
        if self.model.layer_type == "GAT" and not self.lg_ready:
            from .gnn_model import linear
            self.lg = self._logits_buf()
            linear(x[:self.layout.n_own], self._wlog(i), out=self.lg[:self.layout.n_own])

    def after_halo(self, i, x):
        """GAT without exchanged logits: the ghost rows' logits, from their
        rows that just landed."""
        if self.model.layer_type == "GAT" and self.layout.n_ghost and not self.lg_ready:
            from .gnn_model import linear
            linear(x[self.layout.n_own:], self._wlog(i), out=self.lg[self.layout.n_own:])

    def layer(self, i, x, out, rb, re):
        if i == 1 and self.codes is not None:
            self.model._gcn_layer1_codes(self.csr, self.codes, rb, re, out)
            return
        lg_next = None
        if self.chain and i + 1 < self.num_layers:
            if self.lg_next is None:
                self.lg_next = self._logits_buf()
            lg_next = self.lg_next
        self.model._layer(i, self.model.gnn_layers[i], self.csr, x, out, rb, re,
                          logits=self.lg, logits_next=lg_next)

    def end_layer(self, i):
        if i == 1:
            self.codes = None
        if self.chain and i + 1 < self.num_layers:
            self.lg, self.lg_next = self.lg_next, self.lg
            self.lg_ready = True
        else:
            self.lg_ready = False

    def output(self, x_own):
        m = self.model
        out = torch.empty((x_own.shape[0], m.output_dim), dtype=torch.float32,
                          device=x_own.device)
        tmp = torch.empty_like(x_own)
        # local order -> owned (global id) order
        m._output_mlp(x_own, tmp, out, rows=self.layout.perm.to(torch.int32),
                      inv=self.layout.inv.to(torch.int32))
        return out


def _heads() -> int:
    from .gnn_model import HEADS
    return HEADS
