"""The sharded forward on the GPU without a second GPU: P = 2 and 4 shards of
one graph in one process, each a FlowGNNShard (the native layers on its
rank-local CSR, owned rows in the interior/boundary locality order, layer 0
composed with input_proj from exchanged ghost coordinates for GCN, GAT, GIN
H=256 and TransformerConv, GAT logits from the previous layer's epilogue
with their ghost rows in the halo), the halo filled by
device-to-device row copies through the same sharded_forward code the
multi-process RCCL path runs.  Must equal the unsharded forward up to fp32
summation order, for all four layer types, on k-slabs (natural order) and on
arbitrary node ranges (shuffled order)."""

import pytest
import torch

from helpers import khop_subgraph
from mignn import FlowGNN
from mignn.dist import FlowGNNShard, LocalExchange, build_local_layouts, range_bounds, sharded_forward
from mignn.gnn_model import locality_order
from mignn.synthetic import grid_graph, seeded_state_dict
from oracle import flowgnn_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from mignn import _lib
    _lib.lib()


def _sharded(model, x, ei, P, ordered=True, cols=False):
    n = x.shape[0]
    b = range_bounds(n, P)
    edges = [ei[:, (ei[1] >= b[r]) & (ei[1] < b[r + 1])] for r in range(P)]
    pos = [x[b[r]:b[r + 1]] for r in range(P)]
    order = (lambda p, e: locality_order(p, e)[0]) if ordered else None
    if ordered and cols:     # the column order: the window kernel on the shards
        order = lambda p, e: (lambda r: (r[0], r[2]))(locality_order(p, e, cols=True))  # noqa: E731
    lays = build_local_layouts(edges, b, pos=pos, order_fn=order)
    shards = [FlowGNNShard(model, lay, p) for lay, p in zip(lays, pos)]
    ex = LocalExchange()
    shards[0].setup(ex, shards)
    with torch.no_grad():
        ys = sharded_forward(shards, ex, pos)
    return torch.cat(ys, 0), lays


@pytest.mark.parametrize("shuffle", [None, 2])
@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("lt,H", [("GCN", 128), ("GCN", 64), ("GAT", 64), ("GAT", 128),
                                  ("GAT", 256), ("GIN", 64), ("GIN", 256), ("Transformer", 64),
                                  ("Transformer", 256)])
def test_sharded_matches_unsharded(lt, H, P, shuffle):
    cfg = dict(hidden_dim=H, num_layers=3, layer_type=lt)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=4)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, ei = grid_graph(24, 20, 16, device=DEV, permute_seed=shuffle)
    with torch.no_grad():
        y = m(x, ei)
    ys, lays = _sharded(m, x, ei, P)
    scale = max(1.0, y.abs().max().item())
    err = (ys - y).abs().max().item()
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    e64 = (ys.cpu().double() - ref).abs().max().item()
    print(f"{lt} H{H} P={P} shuffle={shuffle}: ghosts/rank {[l.n_ghost for l in lays]}, "
          f"interior {[l.n_int for l in lays]}, max|sharded-unsharded| {err:.2e}, "
          f"max|sharded-fp64| {e64:.2e}")
    if shuffle is None:
        plane = 24 * 20
        assert all(l.n_ghost == 2 * plane for l in lays)      # k-slabs: two halo planes
    assert err <= 2e-6 * scale
    assert e64 <= 1e-5 * scale


@pytest.mark.parametrize("lt,H,kind", [("GCN", 128, "gcn"), ("GAT", 128, "gat"),
                                       ("GAT", 256, "gat"), ("GIN", 256, "gin"),
                                       ("Transformer", 128, "transformer")])
def test_sharded_route_matches_one_gpu(lt, H, kind, monkeypatch):
    """The shards take FlowGNN.forward's route: layer 0 composed from the
    coordinates (the kind the 1-GPU forward runs), and sharded GAT forms
    every later layer's logits in the previous layer's epilogue, their ghost
    rows travelling with the halo -- no logit GEMV (mignn.gnn_model.linear)
    is launched."""
    import mignn.gnn_model as gm
    cfg = dict(hidden_dim=H, num_layers=3, layer_type=lt)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=8))
    m = m.to(DEV).eval()
    assert m._layer0_kind() == kind
    x, ei = grid_graph(24, 20, 16, device=DEV)
    with torch.no_grad():
        y = m(x, ei)
    calls = []
    real = gm.linear

    def counting(*a, **k):
        calls.append(a[0].shape)
        return real(*a, **k)
    monkeypatch.setattr(gm, "linear", counting)
    ys, lays = _sharded(m, x, ei, 4)
    assert all(l.n_ghost > 0 for l in lays)
    if lt == "GAT":
        assert calls == [], f"logit GEMVs in the sharded GAT forward: {calls}"
    scale = max(1.0, y.abs().max().item())
    assert (ys - y).abs().max().item() <= 2e-6 * scale


def test_sharded_single_shard_is_plain_forward():
    """P = 1: no ghosts, every row interior; identical to FlowGNN.forward
    without the internal reorder (same CSR, same kernels)."""
    cfg = dict(hidden_dim=128, num_layers=4, layer_type="GCN")
    m = FlowGNN(input_dim=3, output_dim=7, **cfg)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=1))
    m = m.to(DEV).eval()
    m.reorder = "0"
    x, ei = grid_graph(30, 20, 10, device=DEV)
    with torch.no_grad():
        y = m(x, ei)
    ys, lays = _sharded(m, x, ei, 1, ordered=False)
    assert lays[0].n_ghost == 0 and lays[0].n_int == x.shape[0]
    assert torch.equal(ys, y)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_config4_gin_h256_l8_partitioned(P):
    """configs[4]'s model (GIN, hidden 256, 8 layers) as the bench runs it at
    N GPUs -- k-slab node ranges with a halo exchange per layer -- here as P
    in-process FlowGNNShards of a 500 x 400 x 16 mesh (3.2M nodes; P = 8
    gives each shard two k-planes and two ghost planes).  Must equal the
    unsharded forward up to fp32 summation order, and the fp64 oracle on the
    receptive field of a seeded row sample (helpers.khop_subgraph)."""
    cfg = dict(hidden_dim=256, num_layers=8, layer_type="GIN")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=6)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, ei = grid_graph(500, 400, 16, device=DEV)
    n = x.shape[0]
    with torch.no_grad():
        y = m(x, ei)
    ys, lays = _sharded(m, x, ei, P)
    plane = 500 * 400
    assert all(l.n_ghost == 2 * plane for l in lays)
    scale = max(1.0, y.abs().max().item())
    err = (ys - y).abs().max().item()
    g = torch.Generator().manual_seed(77 + P)
    # seeds on the shard boundaries (first / last plane of each shard) and inside
    b = range_bounds(n, P)
    seeds = torch.cat([torch.tensor([b[r], b[r + 1] - 1]) for r in range(P)]
                      + [torch.randint(0, n, (8,), generator=g)]).unique().to(DEV)
    nodes, sub = khop_subgraph(ei, n, seeds, cfg["num_layers"])
    xs, subc = x[nodes].cpu(), sub.cpu()
    got = ys[seeds].cpu().double()
    del y, ys
    torch.cuda.empty_cache()
    r64 = orc.flowgnn_forward(sd, cfg, xs, subc, None, dtype=torch.float64)[:seeds.numel()]
    r32 = orc.flowgnn_forward(sd, cfg, xs, subc, None, dtype=torch.float32)[:seeds.numel()]
    e64 = (got - r64).abs().max().item()
    ref = (r32.double() - r64).abs().max().item()
    print(f"GIN H256 L8 P={P}: {n} nodes, interior {[l.n_int for l in lays]}, "
          f"max|sharded-unsharded| {err:.2e} (|y| <= {scale:.2f}), max|sharded-fp64| {e64:.2e} "
          f"on {seeds.numel()} rows ({nodes.numel()}-node field), fp32 oracle {ref:.2e}")
    assert err <= 2e-6 * scale
    assert e64 <= max(1e-5, 2.0 * ref)


@pytest.mark.parametrize("P", [2, 3])
def test_range_layout_device_matches_host(P):
    """RangeLayout on the device (the local edge list by mignn_range_relabel)
    equals the same layout built from host tensors by the torch path: local
    edges, order, ghosts, boundary split and send lists, on a graph with
    duplicate edges, self-loops and ranks without ghosts from some peers."""
    g = torch.Generator().manual_seed(P)
    n = 3000
    ei = torch.randint(0, n, (2, 40000), generator=g)
    ei = torch.cat([ei, torch.stack([torch.arange(n), torch.arange(n)])], 1)
    b = range_bounds(n, P)
    edges = [ei[:, (ei[1] >= b[r]) & (ei[1] < b[r + 1])] for r in range(P)]
    host = build_local_layouts(edges, b)
    dev = build_local_layouts([e.to(DEV) for e in edges], b)
    for lh, ld in zip(host, dev):
        assert (lh.n_int, lh.n_ghost, lh.ghost_ptr) == (ld.n_int, ld.n_ghost, ld.ghost_ptr)
        assert torch.equal(lh.edge_index, ld.edge_index.cpu())
        assert torch.equal(lh.perm, ld.perm.cpu())
        assert torch.equal(lh.ghost_gid, ld.ghost_gid.cpu())
        assert sorted(lh.send_idx) == sorted(ld.send_idx)
        for q in lh.send_idx:
            assert torch.equal(lh.send_idx[q], ld.send_idx[q].cpu())


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("P", [2, 3])
def test_range_csr_matches_relabelled_list(P, mode):
    """A shard's CSR built straight from its global-id in-edges
    (RangeLayout.build_csr -> mignn_csr_build_range, the ids mapped inside the
    build) equals build_csr of the materialised local list
    (mignn_range_relabel) bit for bit -- row_ptr, col, dinv, gcn_norm ew, the
    kept / invalid counts -- with duplicate edges and self-loops, in both CSR
    modes (VERBATIM, ONE_SELF_LOOP)."""
    from mignn.gnn_model import build_csr
    g = torch.Generator().manual_seed(10 + P)
    n = 3000
    ei = torch.randint(0, n, (2, 40000), generator=g)
    ei = torch.cat([ei, torch.stack([torch.arange(n), torch.arange(n)]), ei[:, :500]], 1)
    b = range_bounds(n, P)
    edges = [ei[:, (ei[1] >= b[r]) & (ei[1] < b[r + 1])].to(DEV) for r in range(P)]
    for lay in build_local_layouts(edges, b):
        assert lay._edge_index is None            # the device layout writes no local list
        c1 = lay.build_csr(mode)
        c2 = build_csr(lay.edge_index, lay.n_total, mode)
        torch.cuda.synchronize()
        assert torch.equal(c1.row_ptr, c2.row_ptr)
        nnz = int(c2.row_ptr[-1])
        assert torch.equal(c1.col[:nnz], c2.col[:nnz])
        assert torch.equal(c1.info, c2.info)
        if mode == 1:
            assert torch.equal(c1.dinv, c2.dinv)
            assert torch.equal(c1.ew[:nnz], c2.ew[:nnz])


@pytest.mark.parametrize("shuffle", [None, 2])
@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("H", [64, 128])
def test_sharded_column_order_window_route(H, P, shuffle):
    """Shards in the column order take the window kernel (their CSRs carry
    the order info; plans over the interior / boundary row ranges in the
    chunk schedule): equal to the unsharded forward up to fp32 summation
    order and to fp64 within the usual bound."""
    cfg = dict(hidden_dim=H, num_layers=3, layer_type="GCN")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=6)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, ei = grid_graph(40, 32, 24, device=DEV, permute_seed=shuffle)
    with torch.no_grad():
        y = m(x, ei)
    ys, lays = _sharded(m, x, ei, P, cols=True)
    assert all(l.order_info is not None for l in lays)
    assert m._gcn_kernel(H) == "win"
    scale = max(1.0, y.abs().max().item())
    assert (ys - y).abs().max().item() <= 2e-6 * scale
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    assert (ys.cpu().double() - ref).abs().max().item() <= 1e-5 * scale
