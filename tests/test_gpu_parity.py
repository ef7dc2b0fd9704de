"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden vectors made from the reference's own code.

Tolerance: the north star's 1e-5 max-abs error on the raw [N, 7] forward
output (BASELINE.json).  The exact-fp32 path (MFMA f32 / VALU fp32) shows
~1e-7; the split-fp16 ("f16x3") GCN transform ~1e-6; integer work (grid
graph, CSR) is bit-exact.  Model-level tests run at both precisions.
"""

import math

import numpy as np
import pytest
import torch

from helpers import (bfs_graph, csr_np, grid_graph_np, model_fixture, model_names, parity_tol,
                     surrogate_fixture, surrogate_names, tiny_fixture, tiny_names)
import mignn
from mignn import _lib
from mignn.gnn_model import FlowGNN, build_csr, linear
from mignn.synthetic import grid_graph, seeded_state_dict
from oracle import flowgnn_oracle as orc

pytestmark = pytest.mark.gpu
TOL = 1e-5  # BASELINE.json north star: <= 1e-5 max-abs vs the CPU reference


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()  # loud failure if libmignn.so is missing
    torch.set_num_threads(min(16, torch.get_num_threads()))


DEV = "cuda"


def make_model(cfg, sd, precision="f16x3"):
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    m.load_state_dict(sd)
    m.precision = precision
    return m.to(DEV).eval()


PRECISIONS = ["f32", "f16x3"]


# ------------------------------------------------------------------ integer work
def test_grid_graph_bit_exact():
    for dims, slab in (((5, 4, 3), None), ((7, 3, 6), (2, 3)), ((1, 2, 2), None)):
        zb, zc = slab if slab else (0, None)
        x, ei = grid_graph(*dims, device=DEV, z_begin=zb, z_count=zc)
        xn, ein = grid_graph_np(*dims, z_begin=zb, z_count=zc)
        assert np.array_equal(ei.cpu().numpy(), ein)
        assert np.array_equal(x.cpu().numpy(), xn)


def _edge_sets():
    g = torch.Generator().manual_seed(0)
    sets = {name: (tiny_fixture(name, "GCN")[1], tiny_fixture(name, "GCN")[0].shape[0])
            for name in tiny_names()}
    x, ei, _ = bfs_graph("train")
    sets["bfs_train"] = (ei, x.shape[0])
    x, ei, _ = bfs_graph("infer")
    sets["bfs_infer"] = (ei, x.shape[0])
    ei = torch.randint(-3, 1003, (2, 20000), generator=g)
    sets["random_invalid"] = (ei, 1000)
    ei = torch.randint(0, 50, (2, 5000), generator=g)   # heavy duplicates, hub rows
    sets["dense_dups"] = (ei, 60)
    # rows of ~30 entries from scattered edges (in-memory insertion-sort path),
    # many waves / blocks per row
    ei = torch.randint(0, 5000, (2, 150000), generator=g)
    sets["mid_degree"] = (ei, 5000)
    # a mesh edge list (a node's edges consecutive: one run per row) with every
    # 7th edge moved to the end (rows split over runs and waves)
    ei = torch.from_numpy(grid_graph_np(12, 10, 9)[1])
    sel = torch.arange(ei.shape[1]) % 7 == 3
    sets["mesh_split_runs"] = (torch.cat([ei[:, ~sel], ei[:, sel]], 1), 12 * 10 * 9)
    return sets


@pytest.mark.parametrize("mode", [_lib.CSR_VERBATIM, _lib.CSR_ONE_SELF_LOOP])
def test_csr_build_bit_exact(mode):
    for name, (ei, n) in _edge_sets().items():
        csr = build_csr(ei.to(DEV), n, mode)
        rp, col = csr_np(ei.numpy(), n, mode == _lib.CSR_ONE_SELF_LOOP)
        got_rp = csr.row_ptr.cpu().numpy()
        assert np.array_equal(got_rp, rp), name
        assert np.array_equal(csr.col[: rp[-1]].cpu().numpy(), col), name
        info = csr.info.cpu().numpy()
        assert info[2] == rp[-1]
        if mode == _lib.CSR_ONE_SELF_LOOP:
            deg = np.diff(rp)
            np.testing.assert_allclose(csr.dinv.cpu().numpy()[:n], 1 / np.sqrt(deg), rtol=2e-7)
            _check_gcn_weights(csr, name)


def _check_gcn_weights(csr, name):
    """the build's ew (written by csr_scatter, rewritten after a split row's
    sort) equals mignn_gcn_norm's dinv[col] * dinv[row] bitwise"""
    nnz = int(csr.row_ptr[-1].item())
    ew = csr.ew[:nnz].clone()
    csr.compute_gcn_weights()
    assert torch.equal(ew, csr.ew[:nnz]), name
    rp = csr.row_ptr.cpu().numpy()
    rows = np.repeat(np.arange(csr.num_nodes), np.diff(rp))
    dinv = csr.dinv.cpu().numpy()[: csr.num_nodes].astype(np.float64)
    want = dinv[csr.col[:nnz].cpu().numpy()] * dinv[rows]
    np.testing.assert_allclose(ew.cpu().numpy(), want, rtol=1e-6, err_msg=name)


@pytest.mark.parametrize("rb,re", [(0, 5000), (37, 4100), (1000, 1001), (64, 128)])
def test_gcn_norm_row_ranges(rb, re):
    """mignn_gcn_norm over rows [rb, re) of a CSR with empty rows, long rows
    and ragged chunk ends: every entry of those rows = dinv[col] * dinv[row]
    (fp32 product, bitwise), every other entry untouched."""
    g = np.random.default_rng(rb + 7 * re)
    n = 5000
    deg = g.integers(0, 12, n)
    deg[g.random(n) < 0.2] = 0
    deg[g.integers(0, n, 5)] = 200
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = g.integers(0, n, rp[-1]).astype(np.int32)
    dinv = g.random(n).astype(np.float32) + np.float32(0.5)
    d = torch.device("cuda", 0)
    t_rp, t_col, t_dinv = (torch.from_numpy(a).to(d) for a in (rp, col, dinv))
    ew = torch.full((max(int(rp[-1]), 1),), float("nan"), device=d)
    _lib.check(_lib.lib().mignn_gcn_norm(_lib.ptr(t_rp), _lib.ptr(t_col), _lib.ptr(t_dinv), rb, re,
                                         _lib.ptr(ew), _lib.stream(d)), "mignn_gcn_norm")
    got = ew.cpu().numpy()[: rp[-1]]
    rows = np.repeat(np.arange(n), deg)
    inside = (rows >= rb) & (rows < re)
    want = dinv[col] * dinv[rows]
    assert np.array_equal(got[inside].view(np.uint32), want[inside].view(np.uint32))
    assert np.isnan(got[~inside]).all()


@pytest.mark.parametrize("mode", [_lib.CSR_VERBATIM, _lib.CSR_ONE_SELF_LOOP])
def test_csr_build_relabeled_and_transposed(mode):
    """relabel (a permutation of the node ids) and the transposed build equal
    the CPU restatement on the mapped / reversed edge list."""
    g = torch.Generator().manual_seed(7)
    n = 3000
    ei = torch.randint(-2, n + 2, (2, 40000), generator=g)
    perm = torch.randperm(n, generator=g).to(torch.int32)
    valid = (ei >= 0).all(0) & (ei < n).all(0)
    mapped = ei.clone()
    mapped[:, valid] = perm[ei[:, valid]].long()
    csr = build_csr(ei.to(DEV), n, mode, relabel=perm.to(DEV))
    rp, col = csr_np(mapped.numpy(), n, mode == _lib.CSR_ONE_SELF_LOOP)
    assert np.array_equal(csr.row_ptr.cpu().numpy(), rp)
    assert np.array_equal(csr.col[: rp[-1]].cpu().numpy(), col)
    csr_t = build_csr(ei.to(DEV), n, mode | _lib.CSR_TRANSPOSE)
    rp, col = csr_np(ei.flip(0).numpy(), n, mode == _lib.CSR_ONE_SELF_LOOP)
    assert np.array_equal(csr_t.row_ptr.cpu().numpy(), rp)
    assert np.array_equal(csr_t.col[: rp[-1]].cpu().numpy(), col)
    if mode == _lib.CSR_ONE_SELF_LOOP:
        _check_gcn_weights(csr, "relabeled")


# ------------------------------------------------------------------ dense transforms
@pytest.mark.parametrize("M,K,K2,N", [(1, 4, 0, 1), (37, 12, 0, 7), (300, 64, 0, 64),
                                      (1000, 128, 0, 128), (513, 260, 64, 64), (129, 128, 8, 200)])
def test_linear_vs_fp64(M, K, K2, N):
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g)
    A2 = torch.randn(M, K2, generator=g) if K2 else None
    W = torch.randn(N, K + K2, generator=g) * 0.1
    b, r = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    sc, sh = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
    d = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    got = linear(d(A), d(W), d(b), relu=True, residual=d(r), scale=d(sc), shift=d(sh), a2=d(A2))
    Af = A.double() if A2 is None else torch.cat([A, A2], 1).double()
    ref = torch.relu(((Af @ W.double().T + b.double()) + r.double()) * sc.double() + sh.double())
    assert (got.cpu().double() - ref).abs().max().item() < 1e-5
    plain = linear(d(A), d(W[:, :K].contiguous()))
    assert (plain.cpu().double() - A.double() @ W[:, :K].double().T).abs().max().item() < 1e-5


@pytest.mark.parametrize("M,K,N", [(1, 64, 1), (1000, 128, 8), (777, 64, 7), (513, 256, 3),
                                   (4099, 128, 8)])
def test_narrow_linear_vs_fp64(M, K, N):
    """n <= 8 outputs at k in {64, 128, 256}: the streaming row-dot kernel of
    mignn_linear (bias + ReLU epilogue; a residual falls back to the tiles)."""
    g = torch.Generator().manual_seed(7 * M + K + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.1
    b = torch.randn(N, generator=g)
    got = linear(A.to(DEV), W.to(DEV), b.to(DEV), relu=True).cpu().double()
    ref = torch.relu(A.double() @ W.double().T + b.double())
    assert (got - ref).abs().max().item() < 1e-5
    plain = linear(A.to(DEV), W.to(DEV)).cpu().double()
    assert (plain - A.double() @ W.double().T).abs().max().item() < 1e-5
    # strided rows and a strided output
    Ab = torch.randn(M, K + 8, generator=g)
    out = torch.full((M, 12), float("nan"))
    o = out.to(DEV)
    linear(Ab.to(DEV)[:, :K], W.to(DEV), b.to(DEV), out=o[:, :N])
    o = o.cpu()
    assert (o[:, :N].double() - (Ab[:, :K].double() @ W.double().T + b.double())).abs().max() < 1e-5
    assert torch.isnan(o[:, N:]).all()


def test_linear_identity_asymmetric():
    # A = I with an asymmetric W catches a transposed C-write
    n = 48
    A = torch.eye(n)
    W = torch.arange(n * n, dtype=torch.float32).view(n, n) / 100.0
    got = linear(A.to(DEV), W.to(DEV)).cpu()
    assert torch.equal(got, W.T.contiguous())


# ------------------------------------------------------------------ fused GCN layer
@pytest.mark.parametrize("H", [64, 128])
def test_gcn_fused_layer_vs_fp64(H):
    nx, ny, nz = 20, 15, 11
    x0, ei = grid_graph(nx, ny, nz, device=DEV, permute_seed=5)
    n = x0.shape[0]
    g = torch.Generator().manual_seed(H)
    X = torch.randn(n, H, generator=g).to(DEV)
    W = (torch.rand(H, H, generator=g) * 0.2 - 0.1).to(DEV)
    b = (torch.rand(H, generator=g) * 0.2 - 0.1).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    L = _lib.lib()
    out = torch.full((n, H), float("nan"), device=DEV)
    P = _lib.ptr
    for rb, re in ((0, n), (17, n - 100)):
        out.fill_(float("nan"))
        _lib.check(L.mignn_gcn_layer(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb, re, H,
                                     P(W), P(b), P(sc), P(sh), 15, P(out), H, _lib.stream()),
                   "gcn_layer")
        Xd = X.double().cpu()
        ref = orc.gcn_conv(Xd, ei.cpu(), W.double().cpu(), b.double().cpu())
        ref = torch.relu((Xd + ref) * sc.double().cpu() + sh.double().cpu())
        got = out.cpu().double()
        assert (got[rb:re] - ref[rb:re]).abs().max().item() < 1e-5
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()


def _gcn_layer_ref(csr, X, W, b, sc, sh):
    """fp64 evaluation of the fused layer on the CSR the kernel reads."""
    rp = csr.row_ptr.cpu().long()
    n = csr.num_nodes
    nnz = int(rp[-1])
    rows = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    Xd = X.cpu().double()
    agg = torch.zeros(n, X.shape[1], dtype=torch.float64)
    agg.index_add_(0, rows, csr.ew[:nnz].cpu().double()[:, None] * Xd[csr.col[:nnz].cpu().long()])
    y = Xd[:n] + b.cpu().double() + agg @ W.cpu().double().t()
    return torch.relu(y * sc.cpu().double() + sh.cpu().double())


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "small", "strided"])
def test_gcn_f16x3_layer_vs_fp64(H, case):
    """Split-fp16 fused GCN layer: row ranges, partial tiles, in-/out-of-tile
    entries in any mix (natural vs shuffled order), hub rows (> 64 entries per
    producer wave: the slow path), one-step grids, strided x / out."""
    dims = {"natural": (40, 30, 20), "shuffled": (40, 30, 20), "hub": (40, 30, 20),
            "small": (13, 11, 3), "strided": (23, 7, 5)}[case]
    x0, ei = grid_graph(*dims, device=DEV, permute_seed=3 if case == "shuffled" else None)
    n = x0.shape[0]
    if case == "hub":   # node 5 receives from 300 nodes
        src = torch.arange(100, 400, device=DEV)
        ei = torch.cat([ei, torch.stack([src, torch.full_like(src, 5)])], 1)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator().manual_seed(H)
    ld = H + 12 if case == "strided" else H
    Xs = torch.randn(n, ld, generator=g).to(DEV)
    X = Xs[:, :H]
    W = (torch.randn(H, H, generator=g) * 0.05).to(DEV)
    b = (torch.randn(H, generator=g) * 0.05).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    ref = _gcn_layer_ref(csr, X, W, b, sc, sh)
    out = torch.full((n, ld), float("nan"), device=DEV)
    P = _lib.ptr
    for rb, re in ((0, n), (7, n - 3), (64, 64 + min(n - 64, 1000))):
        out.fill_(float("nan"))
        _lib.check(_lib.lib().mignn_gcn_layer_f16x3(
            P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc), P(sh),
            15, P(out), ld, _lib.stream()), "gcn_layer_f16x3")
        got = out[:, :H].cpu().double()
        err = (got[rb:re] - ref[rb:re]).abs().max().item()
        assert err < 1e-5, err
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
        assert torch.isnan(out[:, H:]).all()   # stride padding untouched


def _head_ref(x, ws, bs):
    """fp64 output_proj: Lin-ReLU-Lin-ReLU-Lin-ReLU-Lin (gnn_model.py:90-100)."""
    h = x.cpu().double()
    for i, (w, b) in enumerate(zip(ws, bs)):
        h = h @ w.cpu().double().t() + b.cpu().double()
        if i < 3:
            h = torch.relu(h)
    return h


@pytest.mark.parametrize("H", [64, 128, 256])
@pytest.mark.parametrize("case", [(1000, 7, 0, 0), (37, 8, 0, 1), (1, 3, 4, 0), (20011, 7, 12, 5),
                                  (64, 1, 0, 0), (4096, 7, 0, 0, "wide")])
def test_mlp_head_f16x3_vs_fp64(H, case):
    """Fused split-fp16 output head: partial row blocks, 1..8 outputs,
    strided x / out (padding left untouched), inputs spanning 2^+-8 in
    magnitude ("wide": per-row exponents matter); H = 256 is the chained
    three-transform kernel of agg_gemm.hip."""
    n, od, padx, pado = case[:4]
    g = torch.Generator().manual_seed(n + H + od)
    ld = H + padx
    xs = torch.randn(n, ld, generator=g)
    if len(case) > 4:
        xs = xs * torch.exp2(torch.randint(-8, 9, (n, 1), generator=g).double()).float()
    x = xs.to(DEV)[:, :H]
    dims = [(H, H), (H, H), (H // 2, H), (od, H // 2)]
    ws = [(torch.randn(o, i, generator=g) / math.sqrt(i)).to(DEV) for o, i in dims]
    bs = [(torch.randn(o, generator=g) * 0.1).to(DEV) for o, _ in dims]
    L, P = _lib.lib(), _lib.ptr
    img = torch.empty(L.mignn_mlp_head_prep_bytes(H), dtype=torch.uint8, device=DEV)
    wb = [P(t) for pair in zip(ws, bs) for t in pair]
    _lib.check(L.mignn_mlp_head_prep(*wb, H, od, P(img), img.numel(), _lib.stream()),
               "mlp_head_prep")
    out = torch.full((n, od + pado), float("nan"), device=DEV)
    _lib.check(L.mignn_mlp_head(P(x), ld, n, H, P(img), od, P(out), od + pado, None,
                                _lib.stream()), "mlp_head")
    ref = _head_ref(x, ws, bs)
    got = out.cpu().double()
    scale = max(1.0, ref.abs().max().item())
    err = (got[:, :od] - ref).abs().max().item()
    assert err < 1e-5 * scale, (err, scale)
    assert torch.isnan(got[:, od:]).all()


@pytest.mark.parametrize("H", [128, 256])
def test_mlp_head_scatter_rows(H):
    """out_rows: result row r lands in out row out_rows[r] (locality order ->
    caller order); identical values to the unscattered launch."""
    n, od = 777, 7
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, H, generator=g).to(DEV)
    dims = [(H, H), (H, H), (H // 2, H), (od, H // 2)]
    ws = [(torch.randn(o, i, generator=g) / math.sqrt(i)).to(DEV) for o, i in dims]
    bs = [(torch.randn(o, generator=g) * 0.1).to(DEV) for o, _ in dims]
    L, P = _lib.lib(), _lib.ptr
    img = torch.empty(L.mignn_mlp_head_prep_bytes(H), dtype=torch.uint8, device=DEV)
    wb = [P(t) for pair in zip(ws, bs) for t in pair]
    _lib.check(L.mignn_mlp_head_prep(*wb, H, od, P(img), img.numel(), _lib.stream()), "prep")
    rows = torch.randperm(n, generator=g).to(torch.int32).to(DEV)
    a = torch.full((n, od), float("nan"), device=DEV)
    b = torch.full((n, od), float("nan"), device=DEV)
    _lib.check(L.mignn_mlp_head(P(x), H, n, H, P(img), od, P(a), od, None, _lib.stream()), "a")
    _lib.check(L.mignn_mlp_head(P(x), H, n, H, P(img), od, P(b), od, P(rows), _lib.stream()), "b")
    assert torch.equal(b[rows.long()], a)


def test_mlp_head_rejects_bad_shapes():
    L, P = _lib.lib(), _lib.ptr
    x = torch.zeros(4, 96, device=DEV)
    img = torch.zeros(1 << 18, dtype=torch.uint8, device=DEV)
    out = torch.zeros(4, 8, device=DEV)
    rc = L.mignn_mlp_head(P(x), 96, 4, 96, P(img), 7, P(out), 8, None, _lib.stream())
    assert rc == 1 and "h must be 64, 128 or 256" in _lib.last_error()
    rc = L.mignn_mlp_head(P(x), 96, 4, 64, P(img), 9, P(out), 8, None, _lib.stream())
    assert rc == 1
    rc = L.mignn_mlp_head(P(x) + 4, 96, 4, 64, P(img), 7, P(out), 8, None, _lib.stream())
    assert rc == 1 and "16-B" in _lib.last_error()


# ------------------------------------------------------------------ locality order
def _block_panel_order_np(nx, ny, nz):
    """numpy restatement of the locality key on the natural grid labels:
    4x4x4-cell blocks in panels of 4x4 block columns swept along z
    (csrc/reorder.hip order_keys_kernel)."""
    v = np.arange(nx * ny * nz)
    i, j, k = v % nx, (v // nx) % ny, v // (nx * ny)
    ti, tj, tk = i // 4, j // 4, k // 4
    npx = ((nx + 3) // 4 + 3) // 4
    ntz = (nz + 3) // 4
    blk = (((tj // 4) * npx + ti // 4) * ntz + tk) * 16 + (tj % 4) * 4 + ti % 4
    key = blk * 64 + (k % 4) * 16 + (j % 4) * 4 + i % 4
    return np.argsort(key, kind="stable")


@pytest.mark.parametrize("dims", [(12, 8, 10), (10, 9, 7), (250, 20, 6)])
def test_locality_order_grid(dims):
    from mignn.gnn_model import locality_order
    x, ei = grid_graph(*dims, device=DEV)
    perm, inv = locality_order(x, ei)
    n = x.shape[0]
    p = perm.cpu().numpy()
    assert np.array_equal(np.sort(p), np.arange(n))
    assert np.array_equal(inv.cpu().numpy()[p], np.arange(n))
    assert np.array_equal(p, _block_panel_order_np(*dims))


def test_locality_order_shuffled_and_degenerate():
    """A relabelled grid gets the same cells in the same order (by position);
    no edges / coincident points / a flat mesh still give a permutation."""
    from mignn.gnn_model import locality_order
    x0, ei0 = grid_graph(12, 8, 10, device=DEV)
    x1, ei1 = grid_graph(12, 8, 10, device=DEV, permute_seed=3)
    p0, _ = locality_order(x0, ei0)
    p1, _ = locality_order(x1, ei1)
    assert torch.equal(x0[p0.long()], x1[p1.long()])
    for x, ei in ((torch.rand(1000, 3, device=DEV), torch.zeros(2, 0, dtype=torch.int64, device=DEV)),
                  (torch.zeros(50, 3, device=DEV), torch.randint(0, 50, (2, 200), device=DEV)),
                  (torch.cat([torch.rand(300, 2), torch.zeros(300, 1)], 1).to(DEV),
                   torch.randint(0, 300, (2, 900), device=DEV)),
                  # NaN rows, 1e+-30 magnitudes, invalid edge ids
                  (torch.where(torch.rand(400, 1) < 0.1, torch.tensor(float("nan")),
                               torch.randn(400, 3) * 10.0 ** torch.randint(-30, 31, (400, 3)))
                   .to(DEV), torch.randint(-5, 405, (2, 1200), device=DEV))):
        perm, inv = locality_order(x, ei)
        n = x.shape[0]
        assert torch.equal(perm.sort().values.cpu(), torch.arange(n, dtype=torch.int32))
        assert torch.equal(inv[perm.long()].cpu(), torch.arange(n, dtype=torch.int32))


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("layer_type", ["GCN", "GAT", "GIN", "Transformer"])
def test_flowgnn_reorder_matches_natural(layer_type, precision):
    """The internal locality order changes only the summation order: forward
    with MIGNN_REORDER=1 equals the unreordered forward to fp32 rounding, on
    the natural and the shuffled grid."""
    H = 64
    cfg = dict(hidden_dim=H, num_layers=2, layer_type=layer_type)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=1))
    m = m.to(DEV).eval()
    m.precision = precision
    for seed in (None, 4):
        x, ei = grid_graph(14, 9, 11, device=DEV, permute_seed=seed)
        with torch.no_grad():
            m.reorder = "0"
            y0 = m(x, ei)
            m.reorder = "1"
            y1 = m(x, ei)
        err = (y0 - y1).abs().max().item()
        # summation order only: a few fp32 ulps of the output scale
        assert err < 2e-6 * max(1.0, y0.abs().max().item()), (layer_type, precision, seed, err)


@pytest.mark.parametrize("H,bn,reorder", [(64, True, "0"), (128, True, "1"), (128, False, "0"),
                                         (32, True, "1")])
def test_gcn_layer0_fusion_matches(H, bn, reorder, monkeypatch):
    """input_proj + GCN layer 0 composed into one pass over the coordinates
    (mignn_gcn_layer0_coords) equals the two-step path to fp32 rounding."""
    cfg = dict(hidden_dim=H, num_layers=2, layer_type="GCN", use_batch_norm=bn)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=2))
    m = m.to(DEV).eval()
    m.reorder = reorder
    x, ei = grid_graph(13, 10, 9, device=DEV, permute_seed=2)
    with torch.no_grad():
        m.fuse_layer0 = False
        y0 = m(x, ei)
        m.fuse_layer0 = True
        y1 = m(x, ei)
    assert (y0 - y1).abs().max().item() < 2e-6 * max(1.0, y0.abs().max().item())


# ------------------------------------------------------------------ end-to-end parity
@pytest.mark.parametrize("reorder", ["0", "1"])
@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", model_names())
def test_flowgnn_bfs_parity(name, precision, reorder):
    """Every fixture model (configs[0..4]'s architectures among them) on the
    reference-built BFS graphs vs the reference wrapper's fp32 CPU output and
    the fp64 oracle; outputs are O(1)..O(10) (fan-in weights)."""
    cfg, sd, outs, err = model_fixture(name)
    m = make_model(cfg, sd, precision)
    m.reorder = reorder
    for gname, (y32, y64) in outs.items():
        x, ei, ea = bfs_graph(gname)
        ea_in = None if cfg["layer_type"] == "Transformer" else ea.to(DEV)
        with torch.no_grad():
            y = m(x.to(DEV), ei.to(DEV), ea_in).cpu()
        e32 = (y - y32).abs().max().item()
        e64 = (y.double() - y64).abs().max().item()
        tol = parity_tol(name, gname)
        print(f"{name} {gname} {precision} reorder={reorder}: |y| <= {y64.abs().max():.2f}  "
              f"max|gpu-cpu32| {e32:.2e}  max|gpu-fp64| {e64:.2e}  (tol {tol:.1e})")
        assert e64 <= tol and e32 <= tol + (y32.double() - y64).abs().max().item()
    if err is not None:
        x, ei, ea = bfs_graph("train")
        with pytest.raises(RuntimeError) as exc:
            m(x.to(DEV), ei.to(DEV), ea.to(DEV))
        assert str(exc.value).split("\n")[0] == err


@pytest.mark.parametrize("reorder", ["0", "1"])
@pytest.mark.parametrize("name", tiny_names())
@pytest.mark.parametrize("lt", ["GCN", "GAT", "GIN", "Transformer"])
def test_flowgnn_tiny_edge_cases(name, lt, reorder):
    x, ei, sd, y32, y64 = tiny_fixture(name, lt)
    m = make_model(dict(hidden_dim=8, num_layers=2, layer_type=lt), sd)
    m.reorder = reorder
    with torch.no_grad():
        y = m(x.to(DEV), ei.to(DEV)).cpu()
    assert (y.double() - y64).abs().max().item() <= TOL
    assert (y - y32).abs().max().item() <= TOL


@pytest.mark.parametrize("lt,H,precision", [("GCN", 128, "f32"), ("GCN", 128, "f16x3"),
                                            ("GCN", 64, "f16x3"), ("GCN", 256, "f16x3"),
                                            ("GAT", 64, "f32"), ("GIN", 64, "f32"),
                                            ("Transformer", 64, "f32")])
def test_synthetic_grid_vs_oracle(lt, H, precision):
    """Mid-size synthetic mesh (shuffled node order) vs the fp64 CPU oracle."""
    x, ei = grid_graph(40, 30, 25, device=DEV, permute_seed=1)
    cfg = dict(hidden_dim=H, num_layers=2, layer_type=lt)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=11)
    m = make_model(cfg, sd, precision)
    with torch.no_grad():
        y = m(x, ei).cpu()
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    err = (y.double() - ref).abs().max().item()
    print(f"{lt} H={H} {precision}: max err {err:.2e}")
    assert err <= TOL


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", surrogate_names())
def test_flowgnn_surrogate_parity(name, precision):
    """FlowGNNSurrogate (gnn_model.py:223-291): encoder -> + boundary
    conditions -> decoder (output_dim 8), with and without bc, vs the
    reference's own module run (fp32 CPU) and the fp64 oracle."""
    from mignn import FlowGNNSurrogate
    cfg, sd, bc, outs = surrogate_fixture(name)
    m = FlowGNNSurrogate(input_dim=3, dropout=0.1, **cfg)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    m.encoder.precision = m.decoder.precision = precision
    x, ei, ea = bfs_graph("train")
    for tag, b in (("nobc", None), ("bc", bc.to(DEV))):
        y32, y64 = outs[tag]
        with torch.no_grad():
            y = m(x.to(DEV), ei.to(DEV), ea.to(DEV), boundary_conditions=b).cpu()
        assert y.shape == (x.shape[0], 8)
        assert (y.double() - y64).abs().max().item() <= TOL
        assert (y - y32).abs().max().item() <= TOL
