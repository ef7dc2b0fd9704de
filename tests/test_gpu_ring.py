"""GPU parity of the ring GCN kernel (csrc/gcn_ring.hip: the route of a
block-ordered H = 64 row range) against fp64 and against the producer /
consumer kernel (mignn_gcn_layer_f16x3), its aggregate alone, many-step
launches (every workgroup walks several tiles: the slot refill, the records
two steps ahead, the ring parity), and the model's GCN kernel routes.
Reference op: PyG GCNConv (gnn_model.py:63, :166) + residual / BatchNorm /
ReLU (:184-191)."""

import pytest
import torch

from mignn import _lib
from mignn.gnn_model import build_csr, locality_order
from mignn.synthetic import grid_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


def _graph(case, dims=(40, 30, 20)):
    x0, ei = grid_graph(*dims, device=DEV, permute_seed=3 if case == "shuffled" else None)
    n = x0.shape[0]
    if case == "hub":   # node 5 receives from 300 nodes (its wave takes the row-per-wave path)
        src = torch.arange(100, 400, device=DEV)
        ei = torch.cat([ei, torch.stack([src, torch.full_like(src, 5)])], 1)
    if case == "locality":
        _, inv = locality_order(x0, ei)
        return build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv), n
    return build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP), n


def _gcn_layer_ref(csr, X, W, b, sc, sh):
    n = csr.num_nodes
    nnz = int(csr.row_ptr[-1].item())
    rows = torch.repeat_interleave(torch.arange(n), (csr.row_ptr[1:] - csr.row_ptr[:-1]).cpu().long())
    Xd = X.cpu().double()
    agg = torch.zeros(n, X.shape[1], dtype=torch.float64)
    agg.index_add_(0, rows, csr.ew[:nnz].cpu().double()[:, None] * Xd[csr.col[:nnz].cpu().long()])
    y = Xd[:n] + b.cpu().double() + agg @ W.cpu().double().t()
    return agg, torch.relu(y * sc.cpu().double() + sh.cpu().double())


def _ring_plan(csr, rb, re, h):
    L = _lib.lib()
    nb = L.mignn_gcn_ring_plan_bytes(rb, re, h)
    plan = torch.zeros(max(nb, 16), dtype=torch.uint8, device=DEV)
    stats = torch.zeros(4, dtype=torch.int64, device=DEV)
    _lib.check(L.mignn_gcn_ring_plan(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col), _lib.ptr(csr.ew), rb,
                                     re, h, _lib.ptr(plan), nb, _lib.ptr(stats), _lib.stream()),
               "gcn_ring_plan")
    return plan, stats


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "locality", "small", "strided"])
def test_gcn_layer_ring(H, case):
    """The ring kernel vs fp64 and vs the producer / consumer kernel: in-tile,
    ext-area and far (past the ext capacity: the shuffled order) entries, hub
    rows (the row-per-wave path), row ranges, partial tiles, strides."""
    dims = {"small": (13, 11, 3), "strided": (23, 7, 5)}.get(case, (40, 30, 20))
    csr, n = _graph("natural" if case in ("small", "strided") else case, dims)
    g = torch.Generator().manual_seed(H + 3)
    ld = H + 12 if case == "strided" else H
    X = torch.randn(n, ld, generator=g).to(DEV)[:, :H]
    W = (torch.randn(H, H, generator=g) * 0.05).to(DEV)
    b = (torch.randn(H, generator=g) * 0.05).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    _, ref = _gcn_layer_ref(csr, X, W, b, sc, sh)
    out = torch.full((n, ld), float("nan"), device=DEV)
    old = torch.full((n, ld), float("nan"), device=DEV)
    P = _lib.ptr
    L = _lib.lib()
    for rb, re in ((0, n), (7, n - 3), (64, 64 + min(n - 64, 1000))):
        plan, stats = _ring_plan(csr, rb, re, H)
        out.fill_(float("nan"))
        _lib.check(L.mignn_gcn_layer_ring(
            P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc),
            P(sh), 15, P(out), ld, _lib.stream()), "gcn_layer_ring")
        _lib.check(L.mignn_gcn_layer_f16x3(
            P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc), P(sh),
            15, P(old), ld, _lib.stream()), "gcn_layer_f16x3")
        got = out[:, :H].cpu().double()
        err = (got[rb:re] - ref[rb:re]).abs().max().item()
        assert err < 1e-5, (rb, re, err, stats.tolist())
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
        assert torch.isnan(out[:, H:]).all()
        d = (out[rb:re, :H] - old[rb:re, :H]).abs().max().item()
        assert d < 2e-6, (rb, re, d)
        # the aggregate alone by the ring kernel: fp32 sums in CSR order
        agg = torch.full((n, ld), float("nan"), device=DEV)
        _lib.check(L.mignn_gcn_aggregate_ring(
            P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(agg), ld,
            _lib.stream()), "gcn_aggregate_ring")
        rp = csr.row_ptr.long().cpu()
        cl, ew, Xd = csr.col.long().cpu(), csr.ew.cpu().double(), X.cpu().double()
        rows = torch.unique(torch.cat([torch.arange(rb, min(re, rb + 70)),
                                       torch.randint(rb, re, (500,), generator=g)]))
        aref = torch.stack([(ew[rp[r]:rp[r + 1], None] * Xd[cl[rp[r]:rp[r + 1]]]).sum(0)
                            for r in rows.tolist()])
        ag = agg[:, :H].cpu().double()
        assert (ag[rows] - aref).abs().max().item() < 2e-6 * max(1.0, aref.abs().max().item())
        assert torch.isnan(ag[:rb]).all() and torch.isnan(ag[re:]).all()
        assert not torch.isnan(ag[rb:re]).any()
        assert torch.isnan(agg[:, H:]).all()
        st = stats.tolist()
        if case == "shuffled":
            assert st[1] > 0          # far entries exercised
        if case == "hub" and rb <= 5 < re:
            assert st[2] > 0          # a row-per-wave wave exercised


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["locality", "shuffled"])
def test_gcn_ring_many_steps(H, case):
    """>= 4 G 64 rows (G = the ring grid: 512 workgroups at H = 64 on 256 CUs),
    so every workgroup runs several steps; row ranges off a tile boundary;
    layer vs the producer / consumer kernel, layer and aggregate vs fp64 on
    sampled rows."""
    dims = (64, 48, 48)                      # 147,456 rows
    x0, ei = grid_graph(*dims, device=DEV, permute_seed=5 if case == "shuffled" else None)
    n = x0.shape[0]
    if case == "locality":
        _, inv = locality_order(x0, ei)
        csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
    else:
        csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator().manual_seed(H + 21)
    X = torch.randn(n, H, generator=g).to(DEV)
    W = (torch.randn(H, H, generator=g) * 0.05).to(DEV)
    b = (torch.randn(H, generator=g) * 0.05).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    P = _lib.ptr
    L = _lib.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rp, cl = csr.row_ptr.long().cpu(), csr.col.long().cpu()
    ew, Xd = csr.ew.cpu().double(), X.cpu().double()
    Wd, bd, scd, shd = W.cpu().double(), b.cpu().double(), sc.cpu().double(), sh.cpu().double()
    for rb, re in ((0, n), (37, n - 11)):
        assert re - rb >= 4 * (cus * 2) * 64 or H == 128
        plan, stats = _ring_plan(csr, rb, re, H)
        Y, Y0, A = (torch.full_like(X, float("nan")) for _ in range(3))
        _lib.check(L.mignn_gcn_layer_ring(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb,
                                          re, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H,
                                          _lib.stream()), "ring")
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb, re, H,
                                           P(W), P(b), P(sc), P(sh), 15, P(Y0), H, _lib.stream()), "pc")
        _lib.check(L.mignn_gcn_aggregate_ring(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                              rb, re, H, P(A), H, _lib.stream()), "ring_agg")
        torch.cuda.synchronize()
        assert torch.isnan(Y[:rb]).all() and torch.isnan(Y[re:]).all()
        assert not torch.isnan(Y[rb:re]).any() and not torch.isnan(A[rb:re]).any()
        scale = max(1.0, Y0[rb:re].abs().max().item())
        assert (Y[rb:re] - Y0[rb:re]).abs().max().item() < 2e-6 * scale
        rows = torch.randint(rb, re, (400,), generator=g).tolist()
        agg = torch.stack([(ew[rp[r]:rp[r + 1], None] * Xd[cl[rp[r]:rp[r + 1]]]).sum(0) for r in rows])
        ref = torch.relu((Xd[rows] + bd + agg @ Wd.t()) * scd + shd)
        assert (A[rows].cpu().double() - agg).abs().max().item() < 2e-6 * max(1.0, agg.abs().max().item())
        assert (Y[rows].cpu().double() - ref).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("reorder", ["0", "1"])
def test_model_gcn_kernel_routes_agree(H, reorder):
    """FlowGNN with each split-fp16 GCN layer kernel (pc, ring, win): the same
    model output up to fp32 summation order, and within the fp64 oracle's
    tolerance; the plan is built with the CSR (before the layers); the window
    kernel's graphs are in the column order when reordering is on."""
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    from oracle import flowgnn_oracle as orc
    cfg = dict(hidden_dim=H, num_layers=4, layer_type="GCN")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=5)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    m.reorder = reorder
    x, ei = grid_graph(36, 28, 20, device=DEV, permute_seed=3)
    ys = {}
    for kern in ("pc", "ring", "win"):
        m.gcn_kernel = kern
        m._csr.entries.clear()
        with torch.no_grad():
            ys[kern] = m(x, ei)
        csr = next(iter(m._csr.entries.values()))
        kinds = {k[0] for k in csr.plans}
        assert kinds == (set() if kern == "pc" else {kern})
        assert (csr.order_info is not None) == (kern == "win" and reorder == "1")
    scale = max(1.0, ys["pc"].abs().max().item())
    for kern in ("ring", "win"):
        assert (ys[kern] - ys["pc"]).abs().max().item() <= 2e-6 * scale, kern
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    for kern in ("ring", "win"):
        assert (ys[kern].cpu().double() - ref).abs().max().item() <= 1e-5 * scale, kern


def test_ring_plan_header_mismatch():
    """A ring plan built for another row range (or grid) is refused by the
    kernel: MIGNN_DEVERR_PLAN in the device error word, the launch's output
    rows set to NaN, rows outside its range untouched."""
    csr, n = _graph("locality")
    H = 64
    X = torch.randn(n, H, device=DEV)
    W = torch.randn(H, H, device=DEV) * 0.05
    z = torch.zeros(H, device=DEV)
    plan, _ = _ring_plan(csr, 0, n, H)
    out = torch.zeros_like(X)
    P = _lib.ptr
    _lib.device_errors(clear=True)
    _lib.check(_lib.lib().mignn_gcn_layer_ring(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H,
                                                0, n - 1, H, P(W), P(z), P(z), P(z), 11, P(out), H,
                                                _lib.stream()), "ring")
    assert _lib.device_errors(clear=True) & _lib.DEVERR_PLAN
    assert torch.isnan(out[:n - 1]).all() and torch.count_nonzero(out[n - 1:]).item() == 0


def test_forward_device_error_check_opt_in():
    """FlowGNN.check_device_errors (MIGNN_CHECK_ERRORS=1): the forward reads
    the device's sticky error word after the last kernel and raises on a
    nonzero word; a clean forward returns normally and leaves the word clear."""
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=128, num_layers=3, layer_type="GCN")
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=2))
    m = m.to(DEV).eval()
    m.check_device_errors = True
    x, ei = grid_graph(20, 16, 12, device=DEV)
    with torch.no_grad():
        y = m(x, ei)
    assert torch.isfinite(y).all()
    assert _lib.device_errors(clear=True) == 0
