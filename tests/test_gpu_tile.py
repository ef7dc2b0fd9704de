"""GPU parity of the tile-plan GCN kernels (csrc/gcn_tile.hip): the plan
builder bit-exact against a Python restatement, the fused split-fp16 layer
(mignn_gcn_layer_planned) against fp64 and against the producer / consumer
kernel it replaces (mignn_gcn_layer_f16x3: same arithmetic and sum order, so
rows on the plan's fast path agree bit for bit), and the aggregate alone
(mignn_gcn_aggregate_planned) against fp64.  Reference op: PyG GCNConv
(gnn_model.py:63, :166) + residual / BatchNorm / ReLU (:184-191)."""

import numpy as np
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


def _plan_ref(row_ptr, col, ew, rb, re, h):
    """Python restatement of gcn_plan_kernel: [ntiles*64, 16] uint32."""
    ntiles = (re - rb + 63) // 64
    out = np.zeros((ntiles * 64, 16), dtype=np.uint32)
    ewb = ew.view(np.uint32)
    rowb = 4 * h
    for t in range(ntiles):
        t0 = rb + 64 * t
        nloc = min(64, re - t0)
        cnts = []
        for lr in range(64):
            r = t0 + lr
            rec = out[t * 64 + lr]
            nin = nex = 0
            if r < re:
                for e in range(row_ptr[r], row_ptr[r + 1]):
                    c = int(col[e])
                    off = c - t0
                    inside = 0 <= off < nloc
                    if nin + nex < 7:
                        s = nin if inside else 6 - nex
                        rec[2 * s] = (off * rowb) | ((off & 7) << 4) if inside else c
                        rec[2 * s + 1] = ewb[e]
                    if inside:
                        nin += 1
                    else:
                        nex += 1
            slow = 1 if nin + nex > 7 else 0
            cin, cex = (0, 0) if slow else (nin, nex)
            rec[14] = cin | (cex << 8) | (slow << 16)
            cnts.append((cin, cex, slow))
        for w in range(4):
            grp = cnts[16 * w:16 * w + 16]
            s = (max(c[0] for c in grp) | (max(c[1] for c in grp) << 8)
                 | (max(c[2] for c in grp) << 16))
            out[t * 64 + 16 * w:t * 64 + 16 * w + 16, 15] = s
    return out


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


def _plan(csr, rb, re, h):
    L = _lib.lib()
    nb = L.mignn_gcn_plan_bytes(rb, re)
    plan = torch.zeros(max(nb, 16), dtype=torch.uint8, device=DEV)
    _lib.check(L.mignn_gcn_plan(_lib.ptr(csr.row_ptr), _lib.ptr(csr.col), _lib.ptr(csr.ew), rb, re,
                                h, _lib.ptr(plan), nb, _lib.stream()), "gcn_plan")
    return plan


@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "locality"])
@pytest.mark.parametrize("h", [64, 128])
def test_gcn_plan_bit_exact(case, h):
    csr, n = _graph(case, (13, 11, 7))
    rp, col, ew = (t.cpu().numpy() for t in (csr.row_ptr, csr.col, csr.ew))
    for rb, re in ((0, n), (5, n - 9), (64, 64 + 100)):
        got = _plan(csr, rb, re, h)[:_lib.lib().mignn_gcn_plan_bytes(rb, re)].cpu().numpy()
        ref = _plan_ref(rp, col, ew, rb, re, h)
        assert np.array_equal(got.view(np.uint32).reshape(-1, 16), ref), (case, rb, re)


def _gcn_layer_ref(csr, X, W, b, sc, sh):
    n = csr.num_nodes
    nnz = int(csr.row_ptr[-1].item())
    rows = torch.repeat_interleave(torch.arange(n), (csr.row_ptr[1:] - csr.row_ptr[:-1]).cpu().long())
    Xd = X.cpu().double()
    agg = torch.zeros(n, X.shape[1], dtype=torch.float64)
    agg.index_add_(0, rows, csr.ew[:nnz].cpu().double()[:, None] * Xd[csr.col[:nnz].cpu().long()])
    y = Xd[:n] + b.cpu().double() + agg @ W.cpu().double().t()
    return agg, torch.relu(y * sc.cpu().double() + sh.cpu().double())


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "locality", "small", "strided"])
def test_gcn_layer_planned(H, case):
    """vs fp64 (the split-fp16 bound of the producer / consumer kernel's test)
    and vs that kernel (bitwise on most rows: same sum order and split)."""
    dims = {"small": (13, 11, 3), "strided": (23, 7, 5)}.get(case, (40, 30, 20))
    csr, n = _graph("natural" if case in ("small", "strided") else case, dims)
    g = torch.Generator().manual_seed(H + 7)
    ld = H + 12 if case == "strided" else H
    Xs = torch.randn(n, ld, generator=g).to(DEV)
    X = Xs[:, :H]
    W = (torch.randn(H, H, generator=g) * 0.05).to(DEV)
    b = (torch.randn(H, generator=g) * 0.05).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    _, ref = _gcn_layer_ref(csr, X, W, b, sc, sh)
    out = torch.full((n, ld), float("nan"), device=DEV)
    old = torch.full((n, ld), float("nan"), device=DEV)
    P = _lib.ptr
    L = _lib.lib()
    for rb, re in ((0, n), (7, n - 3), (64, 64 + min(n - 64, 1000))):
        plan = _plan(csr, rb, re, H)
        out.fill_(float("nan"))
        _lib.check(L.mignn_gcn_layer_planned(
            P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc),
            P(sh), 15, P(out), ld, _lib.stream()), "gcn_layer_planned")
        _lib.check(L.mignn_gcn_layer_f16x3(
            P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc), P(sh),
            15, P(old), ld, _lib.stream()), "gcn_layer_f16x3")
        got = out[:, :H].cpu().double()
        err = (got[rb:re] - ref[rb:re]).abs().max().item()
        assert err < 1e-5, (rb, re, err)
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
        assert torch.isnan(out[:, H:]).all()   # stride padding untouched
        d = (out[rb:re, :H] - old[rb:re, :H]).abs().max().item()
        assert d < 2e-6, (rb, re, d)
        if case == "locality":
            same = (out[rb:re, :H] == old[rb:re, :H]).all(1).float().mean().item()
            assert same > 0.99, same


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "locality"])
def test_gcn_aggregate_planned(H, case):
    csr, n = _graph(case)
    g = torch.Generator().manual_seed(H + 11)
    X = torch.randn(n, H, generator=g).to(DEV)
    agg, _ = _gcn_layer_ref(csr, X, torch.zeros(H, H, device=DEV), torch.zeros(H, device=DEV),
                            torch.ones(H, device=DEV), torch.zeros(H, device=DEV))
    out = torch.full((n, H), float("nan"), device=DEV)
    P = _lib.ptr
    for rb, re in ((0, n), (3, n - 70)):
        plan = _plan(csr, rb, re, H)
        out.fill_(float("nan"))
        _lib.check(_lib.lib().mignn_gcn_aggregate_planned(
            P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb, re, H, P(out), H,
            _lib.stream()), "gcn_aggregate_planned")
        got = out.cpu().double()
        err = (got[rb:re] - agg[rb:re]).abs().max().item()
        assert err < 2e-6 * max(1.0, agg[rb:re].abs().max().item()), err
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()


@pytest.mark.parametrize("H", [64, 128])
def test_gcn_planned_mesh_10m_properties(H):
    """The bench mesh (10M nodes, locality order): the planned layer is
    deterministic run to run and agrees with the producer / consumer kernel
    (max |diff| at the split-fp16 bound); the planned aggregate matches the
    fp64 sums on sampled rows."""
    x0, ei = grid_graph(250, 200, 200, device=DEV)
    n = x0.shape[0]
    _, inv = locality_order(x0, ei)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
    del ei, x0
    g = torch.Generator(device=DEV).manual_seed(1)
    X = torch.randn(n, H, device=DEV, generator=g)
    W = torch.randn(H, H, device=DEV, generator=g) * 0.05
    b = torch.randn(H, device=DEV, generator=g) * 0.05
    sc = torch.rand(H, device=DEV, generator=g) + 0.5
    sh = torch.randn(H, device=DEV, generator=g) * 0.1
    plan = _plan(csr, 0, n, H)
    P = _lib.ptr
    L = _lib.lib()
    Y1, Y2, Y0 = (torch.empty_like(X) for _ in range(3))
    for Y in (Y1, Y2):
        _lib.check(L.mignn_gcn_layer_planned(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X),
                                             H, 0, n, H, P(W), P(b), P(sc), P(sh), 15, P(Y), H,
                                             _lib.stream()), "planned")
    _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                       P(W), P(b), P(sc), P(sh), 15, P(Y0), H, _lib.stream()), "pc")
    assert torch.equal(Y1, Y2)
    assert (Y1 - Y0).abs().max().item() < 2e-6 * max(1.0, Y0.abs().max().item())
    A = torch.empty_like(X)
    _lib.check(L.mignn_gcn_aggregate_planned(P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X),
                                             H, 0, n, H, P(A), H, _lib.stream()), "agg")
    rows = torch.randint(0, n, (2048,), generator=torch.Generator().manual_seed(2)).to(DEV)
    rp = csr.row_ptr.long()
    ref = []
    for r in rows.tolist():
        e = slice(int(rp[r]), int(rp[r + 1]))
        ref.append((csr.ew[e].double()[:, None] * X[csr.col[e].long()].double()).sum(0))
    ref = torch.stack(ref)
    assert (A[rows].double() - ref).abs().max().item() < 2e-6 * max(1.0, ref.abs().max().item())


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
@pytest.mark.parametrize("reorder", ["0", "1"])
def test_model_gcn_kernel_routes_agree(H, reorder):
    """FlowGNN with each split-fp16 GCN layer kernel (ring, tile, pc): the
    same model output up to fp32 summation order, and within the fp64
    oracle's tolerance; the plan is built with the CSR (before the layers)."""
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
    for kern in ("pc", "tile", "ring"):
        m.gcn_kernel = kern
        m._csr.entries.clear()
        with torch.no_grad():
            ys[kern] = m(x, ei)
        csr = next(iter(m._csr.entries.values()))
        kinds = {k[0] for k in csr.plans}
        assert kinds == ({"ring"} if kern == "ring" else {"tile"} if kern == "tile" else set())
    scale = max(1.0, ys["pc"].abs().max().item())
    for kern in ("tile", "ring"):
        assert (ys[kern] - ys["pc"]).abs().max().item() <= 2e-6 * scale, kern
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    assert (ys["ring"].cpu().double() - ref).abs().max().item() <= 1e-5 * scale


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
