"""GPU parity of the window GCN kernel (csrc/gcn_win.hip), the product route
of the split-fp16 GCN layer at H = 64 and 128: the fused layer
(mignn_gcn_layer_win) against fp64 and against the producer / consumer
kernel (mignn_gcn_layer_f16x3: same arithmetic, a different fp32 sum order
for the next-tile entry), the aggregate alone (mignn_gcn_aggregate_win)
against fp64, the column order (mignn_locality_order_cols), the plan's
schedule (every tile exactly once) and its header check.  Sizes reach many
steps per workgroup (>= 4 G 64 rows), ranges start off a tile boundary.
Reference op: PyG GCNConv (gnn_model.py:63, :166) + residual / BatchNorm /
ReLU (:184-191)."""

import numpy as np
import pytest
import torch

from mignn import _lib
from mignn.gnn_model import build_csr, locality_order
from mignn.synthetic import grid_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"
P = _lib.ptr


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


def _graph(case, dims=(40, 30, 20)):
    """CSR (GCN mode) of a periodic grid in the named node order, and the
    column-order info where the order is the column order."""
    x0, ei = grid_graph(*dims, device=DEV, permute_seed=3 if case == "shuffled" else None)
    n = x0.shape[0]
    if case in ("hub", "hub_cols"):   # node 5 receives from 300 nodes (its wave: the CSR path)
        src = torch.arange(100, 400, device=DEV)
        ei = torch.cat([ei, torch.stack([src, torch.full_like(src, 5)])], 1)
    if case == "blocks":
        _, inv = locality_order(x0, ei)
        return build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv), n, None
    if case in ("cols", "hub_cols"):
        _, inv, info = locality_order(x0, ei, cols=True)
        return build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv), n, info
    return build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP), n, None


def _plan(csr, rb, re, h, info=None):
    L = _lib.lib()
    nb = L.mignn_gcn_win_plan_bytes(rb, re, h)
    plan = torch.zeros(max(nb, 16), dtype=torch.uint8, device=DEV)
    stats = torch.zeros(4, dtype=torch.int64, device=DEV)
    _lib.check(L.mignn_gcn_win_plan(P(csr.row_ptr), P(csr.col), P(csr.ew), rb, re, h, P(info),
                                    P(plan), nb, P(stats), _lib.stream()), "gcn_win_plan")
    return plan, stats


def _header(plan):
    h = plan[:256].cpu().numpy()
    i32 = h[:32].view(np.int32)
    i64 = h[32:64].view(np.int64)
    return dict(magic=int(i32[0]) & 0xffffffff, G=int(i32[1]), h=int(i32[2]), L=int(i32[3]),
                R1=int(i32[4]), chunk=int(i32[5]), nsteps=int(i32[6]), Z=int(i32[7]),
                ntiles=int(i64[0]), t2=int(i64[1]), rb=int(i64[2]), re=int(i64[3]))


def _sched_tiles(hd):
    """Python restatement of win_tile over every (position, step): tile ids."""
    G, L, R1, chunk, T, t2 = hd["G"], hd["L"], hd["R1"], hd["chunk"], hd["ntiles"], hd["t2"]
    out = []
    p = np.arange(G)[:, None]
    if R1 > 0:
        s = np.arange(R1 * L)[None, :]
        out.append((((s // L) * G + p) * L + s % L).ravel())
    j = np.arange(chunk)[None, :]
    t = t2 + p * chunk + j
    out.append(t[t < T].ravel())
    return np.concatenate(out)


def _ref(csr, X, W, b, sc, sh):
    n = csr.num_nodes
    nnz = int(csr.row_ptr[-1].item())
    rows = torch.repeat_interleave(torch.arange(n), (csr.row_ptr[1:] - csr.row_ptr[:-1]).cpu().long())
    Xd = X.cpu().double()
    agg = torch.zeros(n, X.shape[1], dtype=torch.float64)
    agg.index_add_(0, rows, csr.ew[:nnz].cpu().double()[:, None] * Xd[csr.col[:nnz].cpu().long()])
    y = Xd[:n] + b.cpu().double() + agg @ W.cpu().double().t()
    return agg, torch.relu(y * sc.cpu().double() + sh.cpu().double())


def _layer(csr, plan, X, ld, rb, re, H, W, b, sc, sh, out, flags=15):
    _lib.check(_lib.lib().mignn_gcn_layer_win(
        P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc),
        P(sh), flags, P(out), ld, _lib.stream()), "gcn_layer_win")


def _weights(H, seed):
    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(H, H, generator=g) * 0.05).to(DEV)
    b = (torch.randn(H, generator=g) * 0.05).to(DEV)
    sc, sh = (torch.rand(H, generator=g) + 0.5).to(DEV), (torch.randn(H, generator=g) * 0.1).to(DEV)
    return g, W, b, sc, sh


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["natural", "shuffled", "hub", "blocks", "cols", "hub_cols",
                                  "small", "strided"])
def test_gcn_layer_win(H, case):
    """vs fp64 and vs the producer / consumer kernel: in-window, ext-area,
    next-tile and CSR-path (shuffled order, hub rows) entries, row ranges,
    partial tiles, strides, every node order."""
    # (the column orders: a grid whose workgroups walk 4 tiles -- next-tile entries)
    dims = {"small": (13, 11, 3), "strided": (23, 7, 5), "cols": (64, 48, 40),
            "hub_cols": (64, 48, 40)}.get(case, (40, 30, 20))
    csr, n, info = _graph("natural" if case in ("small", "strided") else case, dims)
    g, W, b, sc, sh = _weights(H, H + 3)
    ld = H + 12 if case == "strided" else H
    X = torch.randn(n, ld, generator=g).to(DEV)[:, :H]
    _, ref = _ref(csr, X, W, b, sc, sh)
    out = torch.full((n, ld), float("nan"), device=DEV)
    old = torch.full((n, ld), float("nan"), device=DEV)
    L = _lib.lib()
    for rb, re in ((0, n), (7, n - 3), (64, 64 + min(n - 64, 1000))):
        plan, stats = _plan(csr, rb, re, H, info if rb == 0 and re == n else None)
        out.fill_(float("nan"))
        _layer(csr, plan, X, ld, rb, re, H, W, b, sc, sh, out)
        _lib.check(L.mignn_gcn_layer_f16x3(
            P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(W), P(b), P(sc), P(sh),
            15, P(old), ld, _lib.stream()), "gcn_layer_f16x3")
        got = out[:, :H].cpu().double()
        err = (got[rb:re] - ref[rb:re]).abs().max().item()
        assert err < 1e-5, (rb, re, err, stats.tolist())
        assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
        assert torch.isnan(out[:, H:]).all()
        # (the kernels round the residual / bias in a different order: a few
        # ulps of the output apart, both within the fp64 bound above)
        d = (out[rb:re, :H] - old[rb:re, :H]).abs().max().item()
        assert d < 2e-6 * max(1.0, old[rb:re, :H].abs().max().item()), (rb, re, d)
        # the aggregate alone by the window kernel
        agg = torch.full((n, ld), float("nan"), device=DEV)
        _lib.check(L.mignn_gcn_aggregate_win(
            P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), ld, rb, re, H, P(agg), ld,
            _lib.stream()), "gcn_aggregate_win")
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
        if case in ("shuffled", "hub", "hub_cols") and rb == 0:
            assert st[1] > 0          # CSR-path rows exercised
        if case == "cols" and rb == 0:
            assert st[2] > 0          # next-tile entries exercised


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("case", ["cols", "shuffled"])
def test_gcn_layer_win_many_steps(H, case):
    """~1M rows (>= 4 G 64: every workgroup walks many steps, the slot ring
    and record ring wrap, the column schedule's rounds and its chunk phase),
    a range starting off a tile boundary: vs the producer / consumer kernel
    on every row, vs fp64 on sampled rows, bitwise deterministic."""
    csr, n, info = _graph(case, (100, 100, 100))
    g, W, b, sc, sh = _weights(H, 17)
    X = torch.randn(n, H, generator=torch.Generator(device=DEV).manual_seed(5), device=DEV)
    L = _lib.lib()
    for rb, re in ((0, n), (37, n - 5)):
        plan, stats = _plan(csr, rb, re, H, info if rb == 0 else None)
        hd = _header(plan)
        assert hd["magic"] == 0x4E495747 and hd["ntiles"] == (re - rb + 63) // 64
        assert hd["nsteps"] >= 4, hd                 # many steps per workgroup
        t = np.sort(_sched_tiles(hd))
        assert np.array_equal(t, np.arange(hd["ntiles"])), hd
        Y1, Y2, Y0 = (torch.full_like(X, float("nan")) for _ in range(3))
        for Y in (Y1, Y2):
            _layer(csr, plan, X, H, rb, re, H, W, b, sc, sh, Y)
        _lib.check(L.mignn_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, rb, re,
                                           H, P(W), P(b), P(sc), P(sh), 15, P(Y0), H,
                                           _lib.stream()), "pc")
        assert torch.equal(Y1[rb:re], Y2[rb:re])
        assert torch.isnan(Y1[:rb]).all() and torch.isnan(Y1[re:]).all()
        scale = max(1.0, Y0[rb:re].abs().max().item())
        assert (Y1[rb:re] - Y0[rb:re]).abs().max().item() < 2e-6 * scale
        rows = torch.randint(rb, re, (256,), generator=torch.Generator().manual_seed(2))
        rp = csr.row_ptr.long()
        Xd = X.double()
        for r in rows.tolist():
            e = slice(int(rp[r]), int(rp[r + 1]))
            a = (csr.ew[e].double()[:, None] * Xd[csr.col[e].long()]).sum(0)
            y = torch.relu((Xd[r] + b.double() + W.double() @ a) * sc.double() + sh.double())
            assert (Y1[r].double() - y).abs().max().item() < 1e-5 * scale


def test_column_order_info_and_permutation():
    """mignn_locality_order_cols: a permutation; info = {1, planes per
    column, full 8x8 columns, full columns per row}; every full column's 64-row
    tiles are its z-planes, in z order."""
    for dims in ((250, 24, 10), (40, 32, 20), (13, 11, 3)):
        x0, ei = grid_graph(*dims, device=DEV)
        perm, inv, info = locality_order(x0, ei, cols=True)
        n = x0.shape[0]
        assert torch.equal(torch.sort(perm.long()).values, torch.arange(n, device=DEV))
        assert torch.equal(inv.long()[perm.long()], torch.arange(n, device=DEV))
        nx, ny, nz = dims
        fx, fy = nx // 8, ny // 8
        assert info.tolist() == [1, nz, fx * fy, fx], (dims, info.tolist())
        if fx * fy == 0:
            continue
        # cell coordinates of the internal rows of the first full column
        c = (x0[perm.long()[:64 * nz]] * torch.tensor(dims, device=DEV) - 0.5).round().long()
        assert bool((c[:, 0] < 8).all() and (c[:, 1] < 8).all())
        z = c[:, 2].view(nz, 64)
        assert torch.equal(z, torch.arange(nz, device=DEV)[:, None].expand(nz, 64))


def test_bench_mesh_column_schedule():
    """The bench mesh (250 x 200 x 200, column order): info {1, 200, 775, 31};
    at H = 128 the column schedule walks whole columns (L = 200) and leaves a
    short chunk phase; the plan's ext capacity holds every full-column plane
    (tiles over capacity only at column ends and the 2-wide x remainder)."""
    x0, ei = grid_graph(250, 200, 200, device=DEV)
    n = x0.shape[0]
    _, inv, info = locality_order(x0, ei, cols=True)
    assert info.tolist() == [1, 200, 775, 31]
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
    del ei, x0
    for H in (64, 128):
        plan, stats = _plan(csr, 0, n, H, info)
        hd = _header(plan)
        assert hd["L"] in (200, 100), hd
        assert hd["chunk"] <= 16, hd
        t = np.sort(_sched_tiles(hd))
        assert np.array_equal(t, np.arange(hd["ntiles"]))
        st = stats.tolist()
        # over-capacity tiles: the first / last tile of every segment and
        # chunk (periodic z, another column before / after), the remainder
        # columns' tiles
        assert st[0] <= 2 * (hd["R1"] * hd["G"] + hd["G"]) + 25 * 50, (st, hd)
        del plan


def test_win_plan_header_mismatch_flags_device_error():
    """A launch whose row range does not match its plan's header: the kernel
    sets MIGNN_DEVERR_PLAN and writes NaN over the launch's output rows (no
    stale buffer contents pass for layer output); rows outside the launch's
    range are untouched."""
    csr, n, _ = _graph("natural", (20, 16, 12))
    H = 64
    g, W, b, sc, sh = _weights(H, 4)
    X = torch.randn(n, H, generator=g).to(DEV)
    plan, _ = _plan(csr, 0, n, H)
    out = torch.zeros((n, H), device=DEV)
    _lib.device_errors(clear=True)
    _layer(csr, plan, X, H, 0, n - 64, H, W, b, sc, sh, out)
    bits = _lib.device_errors(clear=True)
    assert bits & _lib.DEVERR_PLAN
    assert torch.isnan(out[:n - 64]).all() and torch.count_nonzero(out[n - 64:]).item() == 0


@pytest.mark.parametrize("H", [64, 128])
def test_model_gcn_win_1m(H):
    """FlowGNN GCN L4 at 1M nodes (the locality order on, the column order
    for the window route): the window route against the producer / consumer
    route (block order) and the fp64 oracle on a receptive-field sample."""
    from helpers import khop_subgraph
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    from oracle import flowgnn_oracle as orc
    cfg = dict(hidden_dim=H, num_layers=4, layer_type="GCN")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=7)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    m.reorder = "1"
    x, ei = grid_graph(100, 100, 100, device=DEV)
    ys = {}
    for kern in ("win", "pc"):
        m.gcn_kernel = kern
        m._csr.entries.clear()
        with torch.no_grad():
            ys[kern] = m(x, ei)
        csr = next(iter(m._csr.entries.values()))
        assert (csr.order_info is not None) == (kern == "win")
    scale = max(1.0, ys["pc"].abs().max().item())
    assert (ys["win"] - ys["pc"]).abs().max().item() <= 2e-6 * scale
    seeds = torch.randint(0, x.shape[0], (24,), generator=torch.Generator().manual_seed(3))
    nodes, sub = khop_subgraph(ei, x.shape[0], seeds.to(DEV), 4)
    ref = orc.flowgnn_forward(sd, cfg, x[nodes].cpu(), sub.cpu(), None, dtype=torch.float64)
    err = (ys["win"][seeds.to(DEV)].cpu().double() - ref[:24]).abs().max().item()
    assert err <= 1e-5 * scale, err


def _layer0_rows_and_codes(csr, n, H, seed):
    """Layer 0 both ways: its [n, H] rows (mignn_gcn_layer0_coords) and its
    row codes (mignn_gcn_layer0_codes), from random 3-D positions and a
    random [H][8] coefficient table."""
    g = torch.Generator().manual_seed(seed)
    pos = (torch.rand(n, 3, generator=g) * 4 - 1).to(DEV)
    coef = (torch.randn(H, 8, generator=g) * 0.5).to(DEV)
    L = _lib.lib()
    rows = torch.full((n, H), float("nan"), device=DEV)
    _lib.check(L.mignn_gcn_layer0_coords(P(csr.row_ptr), P(csr.col), P(csr.ew), P(pos), 3, 3, 0, n,
                                         P(coef), H, P(rows), H, _lib.stream()), "layer0_coords")
    codes = torch.full((n, 8), float("nan"), device=DEV)
    _lib.check(L.mignn_gcn_layer0_codes(P(csr.row_ptr), P(csr.col), P(csr.ew), P(pos), 3, 3, 0, n,
                                        P(codes), 8, _lib.stream()), "layer0_codes")
    return rows, codes, coef


@pytest.mark.parametrize("case,dims", [("cols", (64, 48, 40)), ("hub_cols", (64, 48, 40)),
                                       ("shuffled", (40, 30, 20)), ("natural", (13, 11, 3)),
                                       ("cols", (100, 100, 100))])
def test_gcn_layer_win_codes(case, dims):
    """The codes form (mignn_gcn_layer0_codes + mignn_gcn_layer_win_codes)
    equals layer 0's rows through mignn_gcn_layer_win bitwise: in-window,
    ext, next-tile and CSR-path entries (the hub / shuffled graphs) expanded
    from codes, row ranges off tile boundaries, compile-time and run-time
    epilogue flags, 1M rows (many steps per workgroup)."""
    H = 128
    csr, n, info = _graph(case, dims)
    X, codes, coef = _layer0_rows_and_codes(csr, n, H, 11)
    assert not torch.isnan(codes).any()
    assert torch.equal(codes[:, 7], torch.zeros(n, device=DEV))
    _, W, b, sc, sh = _weights(H, 23)
    L = _lib.lib()
    for rb, re in ((0, n), (37, n - 5)):
        plan, stats = _plan(csr, rb, re, H, info if rb == 0 else None)
        for flags in (15, 11, 3):
            ref = torch.full((n, H), float("nan"), device=DEV)
            _layer(csr, plan, X, H, rb, re, H, W, b, sc, sh, ref, flags=flags)
            got = torch.full((n, H), float("nan"), device=DEV)
            _lib.check(L.mignn_gcn_layer_win_codes(
                P(plan), P(csr.row_ptr), P(csr.col), P(csr.ew), P(codes), 8, rb, re, H, P(coef),
                P(W), P(b), P(sc), P(sh), flags, P(got), H, _lib.stream()), "win_codes")
            assert torch.equal(got[rb:re], ref[rb:re]), (rb, re, flags,
                                                         (got[rb:re] - ref[rb:re]).abs().max().item())
            assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
        if case in ("hub_cols", "shuffled") and rb == 0:
            assert stats.tolist()[1] > 0          # CSR-path rows exercised


def test_model_gcn_codes_bitwise():
    """FlowGNN GCN H = 128 (window route): layers 0 and 1 through the row
    codes give the same output, bitwise, as layer 0's rows written and read."""
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, hidden_dim=128, num_layers=4,
                layer_type="GCN")
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=9))
    m = m.to(DEV).eval()
    m.reorder = "1"
    x, ei = grid_graph(64, 48, 40, device=DEV)
    ys = {}
    for codes in (True, False):
        m.gcn_codes = codes
        with torch.no_grad():
            ys[codes] = m(x, ei)
        csr = next(iter(m._csr.entries.values()))
        assert m._use_gcn_codes(csr) == codes
    assert torch.equal(ys[True], ys[False])


@pytest.mark.parametrize("H", [64, 128])
def test_win_plan_weight_classes(H):
    """The 16-B plan record carries degree classes, not weights: the kernel
    rebuilds w_ij = dv[c_j] dv[c_i] and the plan admits a row only if that
    equals its ew bitwise.  A one-ulp change of one entry's weight moves
    exactly that row to the CSR path (stats[1] + 1) and the layer still
    follows ew; a graph with arbitrary weights runs every row through the CSR
    path, correct against fp64."""
    csr, n, info = _graph("cols", (64, 48, 40))
    g, W, b, sc, sh = _weights(H, 31)
    X = torch.randn(n, H, generator=g).to(DEV)
    _, st0 = _plan(csr, 0, n, H, info)
    base_far = st0.tolist()[1]
    # a row of a wave that takes the planned path (its summary word's CSR-path
    # bit clear; plan layout per tile: per wave its 16-B codes, then its list
    # -- EPW ext columns, the summary, the row classes): bump its first weight
    plan0, _ = _plan(csr, 0, n, H, info)
    rpw, epw, recg = (16, 8, 304) if H == 64 else (8, 4, 160)
    nw = 64 // rpw
    tabs = plan0[256:].cpu().numpy()
    ntiles = (n + 63) // 64
    summ = np.frombuffer(tabs.tobytes(), dtype=np.uint32).reshape(ntiles, nw, recg // 4)[:, :, rpw * 4 + epw]
    ok = np.argwhere((summ >> 8) & 1 == 0)
    t, w = map(int, ok[len(ok) // 2])
    row = 64 * t + rpw * w + 3
    rp = csr.row_ptr.long()
    e = int(rp[row])
    ew2 = csr.ew.clone()
    ew2[e] = torch.nextafter(ew2[e], torch.tensor(2.0, device=DEV))
    csr2 = copy_with_ew(csr, ew2)
    plan2, st2 = _plan(csr2, 0, n, H, info)
    assert st2.tolist()[1] == base_far + 1, (base_far, st2.tolist())
    out = torch.full((n, H), float("nan"), device=DEV)
    _layer(csr2, plan2, X, H, 0, n, H, W, b, sc, sh, out)
    _, ref = _ref(csr2, X, W, b, sc, sh)
    assert (out.cpu().double() - ref).abs().max().item() < 1e-5
    # arbitrary weights: every row with entries takes the CSR path
    csr3 = copy_with_ew(csr, (torch.rand(csr.ew.shape[0], generator=g) + 0.1).to(DEV))
    plan3, st3 = _plan(csr3, 0, n, H, info)
    assert st3.tolist()[1] == n, st3.tolist()
    out.fill_(float("nan"))
    _layer(csr3, plan3, X, H, 0, n, H, W, b, sc, sh, out)
    _, ref3 = _ref(csr3, X, W, b, sc, sh)
    assert (out.cpu().double() - ref3).abs().max().item() < 1e-5 * max(1.0, ref3.abs().max().item())


def copy_with_ew(csr, ew):
    import copy
    c = copy.copy(csr)
    c.ew = ew
    return c
