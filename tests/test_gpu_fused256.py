"""Fused H = 256 layers (mignn_gin_layer_fused / mignn_gcn_layer_fused,
csrc/agg_gemm.hip) against a float64 torch restatement of the same layer on
the same CSR, and against the unfused launches they replace (aggregate +
split-fp16 GEMM(s)).

Graphs: random destination-major edge lists with degrees 0..12 (rows past the
kernel's 8 register slots take its one-at-a-time path) and hub rows of 40-60
entries, a row sub-range [rb, re) written at out + rb * ldo, rows scaled over
2^+-20 (the online row exponent), every epilogue flag combination.  Bound:
the split arithmetic's ~2^-22 per product, taken as 4e-6 of the magnitude of
the chain computed on |values| (plus fp32 rounding of the result)."""

import pytest
import torch

from mignn import _lib
from mignn.gnn_model import build_csr, f16x3_image, gin_fused_image, linear_f16x3

GAT_LAUNCHES = 64   # include/mignn.h MIGNN_GAT_LAUNCHES
pytestmark = pytest.mark.gpu
DEV = "cuda"
H = 256


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


def _graph(n, seed):
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, 13, (n,), generator=g)
    hub = torch.randperm(n, generator=g)[:5]
    deg[hub] = torch.randint(40, 61, (5,), generator=g)
    dst = torch.repeat_interleave(torch.arange(n), deg)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    perm = torch.randperm(dst.numel(), generator=g)
    return torch.stack([src[perm], dst[perm]]).to(DEV)


def _csr_edges(csr, n):
    rp = csr.row_ptr.cpu().long()
    col = csr.col.cpu().long()[: int(rp[-1])]
    dst = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    return col, dst


def _params(seed, scaled_rows=True, n=3000):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(n, H, device=DEV, generator=g)
    if scaled_rows:
        x *= torch.pow(2.0, torch.randint(-20, 21, (n, 1), device=DEV, generator=g).float())
        x[:7] = 0.0
    w1 = torch.randn(H, H, device=DEV, generator=g) / 16
    w2 = torch.randn(H, H, device=DEV, generator=g) / 16
    b1 = torch.randn(H, device=DEV, generator=g) * 0.1
    b2 = torch.randn(H, device=DEV, generator=g) * 0.1
    sc = torch.rand(H, device=DEV, generator=g) + 0.5
    sh = torch.randn(H, device=DEV, generator=g) * 0.1
    return x, w1, w2, b1, b2, sc, sh


def _epi64(c, mag, x, b, sc, sh, flags):
    if flags & _lib.EPI_BIAS:
        c = c + b.double()
        mag = mag + b.double().abs()
    if flags & _lib.EPI_RESIDUAL:
        c = x + c
        mag = mag + x.abs()
    if flags & _lib.EPI_AFFINE:
        c = c * sc.double() + sh.double()
        mag = mag * sc.double() + sh.double().abs()
    if flags & _lib.EPI_RELU:
        c = c.clamp_min(0)
    return c, mag


def _check(got, ref, mag, what):
    err = (got.double() - ref).abs()
    bound = 4e-6 * mag + 2 * torch.finfo(torch.float32).eps * ref.abs() + 1e-35
    worst = float((err / bound).max())
    assert worst <= 1.0, (what, float(err.max()), worst)


FLAGS = [15, 0, 1 | 8, 2 | 4]


@pytest.mark.parametrize("flags", FLAGS)
@pytest.mark.parametrize("rb,re", [(0, 3000), (123, 2701)])
def test_gin_fused_vs_fp64(flags, rb, re):
    n = 3000
    ei = _graph(n, 11)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    x, w1, w2, b1, b2, sc, sh = _params(5)
    eps = 0.3
    out = torch.full((n, H), float("nan"), device=DEV)
    L = _lib.lib()
    P = _lib.ptr
    img1, img2 = f16x3_image(w1), gin_fused_image(w2)
    _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(x), H, rb, re, H, eps,
                                       P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), flags,
                                       P(out), H, _lib.stream()), "gin_fused")
    torch.cuda.synchronize()
    col, dst = _csr_edges(csr, n)
    X = x.double().cpu()
    a = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, X[col]) + (1 + eps) * X
    am = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, X[col].abs()) + (1 + eps) * X.abs()
    W1, W2 = w1.double().cpu(), w2.double().cpu()
    h = (a @ W1.T + b1.double().cpu()).clamp_min(0)
    hm = am @ W1.T.abs() + b1.double().cpu().abs()
    c = h @ W2.T
    cm = hm @ W2.T.abs()
    ref, mag = _epi64(c, cm, X, b2.cpu(), sc.cpu(), sh.cpu(), flags)
    got = out.cpu()
    _check(got[rb:re], ref[rb:re], mag[rb:re], f"gin flags={flags}")
    assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()


@pytest.mark.parametrize("flags", FLAGS)
def test_gcn_fused_vs_fp64(flags):
    n = 3000
    rb, re = 57, 2999
    ei = _graph(n, 12)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    x, w1, _, b1, _, sc, sh = _params(6)
    out = torch.full((n, H), float("nan"), device=DEV)
    L = _lib.lib()
    P = _lib.ptr
    img = f16x3_image(w1)
    _lib.check(L.mignn_gcn_layer_fused(P(csr.row_ptr), P(csr.col), P(csr.ew), P(x), H, rb, re, H,
                                       P(img), P(b1), P(sc), P(sh), flags, P(out), H,
                                       _lib.stream()), "gcn_fused")
    torch.cuda.synchronize()
    col, dst = _csr_edges(csr, n)
    ew = csr.ew.cpu().double()[: col.numel()]
    X = x.double().cpu()
    a = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, ew[:, None] * X[col])
    am = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, (ew[:, None] * X[col]).abs())
    W = w1.double().cpu()
    ref, mag = _epi64(a @ W.T, am @ W.T.abs(), X, b1.cpu(), sc.cpu(), sh.cpu(), flags)
    got = out.cpu()
    _check(got[rb:re], ref[rb:re], mag[rb:re], f"gcn flags={flags}")
    assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()


def test_gin_fused_matches_unfused_launches():
    """The fused kernel against the launch sequence it replaces (sum aggregate
    + two split-fp16 GEMMs): the same arithmetic up to the hidden layer's
    exponent (one per row over all 256 columns vs the GEMM's online one) and
    fp32 summation order."""
    n = 20000
    g = torch.Generator(device=DEV).manual_seed(3)
    ei = torch.stack([torch.randint(0, n, (6 * n,), device=DEV, generator=g),
                      torch.arange(n, device=DEV).repeat_interleave(6)])
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    x, w1, w2, b1, b2, sc, sh = _params(7, scaled_rows=False, n=n)
    L = _lib.lib()
    P = _lib.ptr
    out = torch.empty(n, H, device=DEV)
    img1, img2 = f16x3_image(w1), gin_fused_image(w2)
    _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(x), H, 0, n, H, 0.0,
                                       P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), 15, P(out),
                                       H, _lib.stream()), "gin_fused")
    agg = torch.empty(n, H, device=DEV)
    _lib.check(L.mignn_sum_aggregate(P(csr.row_ptr), P(csr.col), P(x), H, 1.0, 0, n, H, P(agg), H,
                                     _lib.stream()), "sum_aggregate")
    h1 = linear_f16x3(agg, img1, H, b1, relu=True)
    ref = linear_f16x3(h1, f16x3_image(w2), H, b2, relu=True, residual=x, scale=sc, shift=sh)
    torch.cuda.synchronize()
    d = (out - ref).abs().max().item()
    assert d <= 2e-6 * max(1.0, ref.abs().max().item()), d


def test_fused_deterministic():
    """Two launches give bitwise the same rows (fixed sum order, no atomics)."""
    n = 5000
    ei = _graph(n, 13)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    x, w1, w2, b1, b2, sc, sh = _params(8, n=n)
    L = _lib.lib()
    P = _lib.ptr
    img1, img2 = f16x3_image(w1), gin_fused_image(w2)
    outs = []
    for _ in range(2):
        o = torch.empty(n, H, device=DEV)
        _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(x), H, 0, n, H, 0.1,
                                           P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), 15, P(o),
                                           H, _lib.stream()), "gin_fused")
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def _gat_layer(csr, x, n_x, rb, re, h, wlog, wcat, img, bias, sc, sh, flags, out):
    L = _lib.lib()
    P = _lib.ptr
    nb = L.mignn_gat_layer_scratch_bytes(n_x, re - rb, h, 4)
    scratch = torch.empty(max(nb, 1), dtype=torch.uint8, device=DEV)
    _lib.check(L.mignn_gat_layer(P(csr.row_ptr), P(csr.col), P(x), x.stride(0), n_x, rb, re, h, 4,
                                 0.2, P(wlog), None, 8, P(wcat), P(img), P(bias), P(sc), P(sh),
                                 flags, P(scratch), nb, P(out), out.stride(0), _lib.stream()),
               "gat_layer")


@pytest.mark.parametrize("h", [64, 128])
@pytest.mark.parametrize("flags", [15, 1 | 2])
def test_gat_fused_vs_launches_and_fp64(h, flags):
    """mignn_gat_layer's fused kernel (split-fp16 image given, 4 heads) against
    its aggregate + transform launch sequence (flag MIGNN_GAT_LAUNCHES)
    and against a float64 restatement (PyG GATConv semantics on the CSR:
    LeakyReLU(0.2) logits, softmax + 1e-16, head mean, bias) on a graph with
    hub rows (the kernel's past-the-slots path) and a row sub-range."""
    n = 4000
    rb, re = 33, 3967
    ei = _graph(n, 21)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator(device=DEV).manual_seed(h + flags)
    x = torch.randn(n, h, device=DEV, generator=g)
    wlog = torch.randn(8, h, device=DEV, generator=g) / h ** 0.5
    wcat = torch.randn(h, 4 * h, device=DEV, generator=g) / (2 * h) ** 0.5
    bias = torch.randn(h, device=DEV, generator=g) * 0.1
    sc = torch.rand(h, device=DEV, generator=g) + 0.5
    sh = torch.randn(h, device=DEV, generator=g) * 0.1
    img = f16x3_image(wcat)
    outs = []
    for fused in (1, 0):
        o = torch.full((n, h), float("nan"), device=DEV)
        _gat_layer(csr, x, n, rb, re, h, wlog, wcat, img, bias, sc, sh,
                   flags | (0 if fused else GAT_LAUNCHES), o)
        outs.append(o)
    torch.cuda.synchronize()
    got, launches = outs[0].cpu(), outs[1].cpu()
    assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
    # float64 restatement on the same CSR
    col, dst = _csr_edges(csr, n)
    X = x.double().cpu()
    lg = X @ wlog.double().cpu().T                                   # [n, 8]
    s = lg[col, :4] + lg[dst, 4:]
    s = torch.where(s > 0, s, 0.2 * s)
    mx = torch.full((n, 4), -float("inf"), dtype=torch.float64).scatter_reduce(
        0, dst[:, None].expand_as(s), s, "amax", include_self=True)
    pexp = torch.exp(s - mx[dst])
    sm = torch.zeros((n, 4), dtype=torch.float64).index_add_(0, dst, pexp) + 1e-16
    alpha = pexp / sm[dst]                                          # [E, 4]
    agg = torch.zeros((n, 4, h), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col][:, None, :]).reshape(n, 4 * h)
    aggm = torch.zeros((n, 4, h), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col].abs()[:, None, :]).reshape(n, 4 * h)
    W = wcat.double().cpu()
    ref, mag = _epi64(agg @ W.T, aggm @ W.T.abs(), X, bias.cpu(), sc.cpu(), sh.cpu(), flags)
    _check(got[rb:re], ref[rb:re], mag[rb:re], f"gat fused h={h}")
    _check(launches[rb:re], ref[rb:re], mag[rb:re], f"gat launches h={h}")


@pytest.mark.parametrize("h", [64, 128])
def test_gat_fused_coresident_blocks(h):
    """The fused GAT kernel runs two 4-wave blocks per CU; the small-graph
    tests above launch fewer blocks than there are CUs.  Here 200k rows
    (3125 blocks) of the irregular graph (degrees 0-12, hubs) put two blocks
    on every CU: fused == the launch sequence on every row."""
    n = 200_000
    ei = _graph(n, 21)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator(device=DEV).manual_seed(h)
    x = torch.randn(n, h, device=DEV, generator=g)
    wlog = torch.randn(8, h, device=DEV, generator=g) / h ** 0.5
    wcat = torch.randn(h, 4 * h, device=DEV, generator=g) / (2 * h) ** 0.5
    bias = torch.randn(h, device=DEV, generator=g) * 0.1
    sc = torch.rand(h, device=DEV, generator=g) + 0.5
    sh = torch.randn(h, device=DEV, generator=g) * 0.1
    img = f16x3_image(wcat)
    outs = []
    for fused in (1, 0):
        o = torch.full((n, h), float("nan"), device=DEV)
        _gat_layer(csr, x, n, 0, n, h, wlog, wcat, img, bias, sc, sh,
                   15 | (0 if fused else GAT_LAUNCHES), o)
        outs.append(o)
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max(1).values
    scale = max(1.0, outs[1].abs().max().item())
    assert torch.isfinite(outs[0]).all()
    assert int((d > 2e-5 * scale).sum()) == 0, (int((d > 2e-5 * scale).sum()), d.max().item())


def _tf_layer(fused, csr, x, rb, re, wqk, bqk, wout, bout, sc, sh, flags, out):
    L = _lib.lib()
    P = _lib.ptr
    nb = L.mignn_transformer_layer_scratch_bytes(re - rb, H, 4)
    scratch = torch.empty(max(nb, 1), dtype=torch.uint8, device=DEV)
    img_q = f16x3_image(wqk)
    if fused:
        fimg = torch.empty(L.mignn_transformer_fused_prep_bytes(H, 4), dtype=torch.uint8,
                           device=DEV)
        _lib.check(L.mignn_transformer_fused_prep(P(wout), H, 4, P(fimg), fimg.numel(),
                                                  _lib.stream()), "tf_fused_prep")
        _lib.check(L.mignn_transformer_layer_fused(
            P(csr.row_ptr), P(csr.col), P(x), H, rb, re, H, 4, 1.0 / 16, P(img_q), P(bqk), P(fimg),
            P(bout), P(sc), P(sh), flags, P(scratch), nb, P(out), H, _lib.stream()), "tf_fused")
    else:
        _lib.check(L.mignn_transformer_layer(
            P(csr.row_ptr), P(csr.col), P(x), H, rb, re, H, 4, 1.0 / 16, P(wqk), P(img_q), P(bqk),
            P(wout), P(f16x3_image(wout)), P(bout), P(sc), P(sh), flags, P(scratch), nb, P(out), H,
            _lib.stream()), "tf_layer")


@pytest.mark.parametrize("flags", [15, 1 | 2])
def test_transformer_fused_vs_launches_and_fp64(flags):
    """mignn_transformer_layer_fused (scores, softmax, weighted sums and the
    output transform in one kernel) against mignn_transformer_layer's launch
    sequence and a float64 restatement (PyG TransformerConv on the CSR, 4
    heads, concat=False, root weight: softmax + 1e-16 of q_i . k_j / sqrt(C),
    head mean of the weighted values, + lin_skip) in the re-associated weights
    the layer takes (wqk = Wk^T Wq, wout = [Wv / 4 | bv / 4 | W_skip]).  The
    graph has empty rows and hub rows of 40-60 entries (past the kernel's 8
    register slots and 16 LDS-kept scores: the recompute path); a row range."""
    n = 3000
    rb, re = 45, 2980
    ei = _graph(n, 31)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    g = torch.Generator(device=DEV).manual_seed(flags)
    x = torch.randn(n, H, device=DEV, generator=g)
    x *= torch.pow(2.0, torch.randint(-3, 4, (n, 1), device=DEV, generator=g).float())
    wqk = torch.randn(4 * H, H, device=DEV, generator=g) / 16
    bqk = torch.randn(4 * H, device=DEV, generator=g) * 0.1
    wout = torch.randn(H, 4 * H + 4 + H, device=DEV, generator=g) / (4 * H + 4 + H) ** 0.5
    bout = torch.randn(H, device=DEV, generator=g) * 0.1
    sc = torch.rand(H, device=DEV, generator=g) + 0.5
    sh = torch.randn(H, device=DEV, generator=g) * 0.1
    outs = []
    for fused in (True, False):
        o = torch.full((n, H), float("nan"), device=DEV)
        _tf_layer(fused, csr, x, rb, re, wqk, bqk, wout, bout, sc, sh, flags, o)
        outs.append(o)
    torch.cuda.synchronize()
    got, launches = outs[0].cpu(), outs[1].cpu()
    assert torch.isnan(got[:rb]).all() and torch.isnan(got[re:]).all()
    col, dst = _csr_edges(csr, n)
    X = x.double().cpu()
    qt = X @ wqk.double().cpu().T + bqk.double().cpu()              # [n, 4H]
    s = (qt[dst].view(-1, 4, H) * X[col][:, None, :]).sum(-1) / 16   # [E, 4]
    mx = torch.full((n, 4), -float("inf"), dtype=torch.float64).scatter_reduce(
        0, dst[:, None].expand_as(s), s, "amax", include_self=True)
    pexp = torch.exp(s - mx[dst])
    sm = torch.zeros((n, 4), dtype=torch.float64).index_add_(0, dst, pexp) + 1e-16
    alpha = pexp / sm[dst]
    agg = torch.zeros((n, 4, H), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col][:, None, :]).reshape(n, 4 * H)
    asum = torch.zeros((n, 4), dtype=torch.float64).index_add_(0, dst, alpha)
    aggm = torch.zeros((n, 4, H), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col].abs()[:, None, :]).reshape(n, 4 * H)
    W = wout.double().cpu()
    c = torch.cat([agg, asum, X], 1) @ W.T
    cm = torch.cat([aggm, asum, X.abs()], 1) @ W.T.abs()
    ref, mag = _epi64(c, cm, X, bout.cpu(), sc.cpu(), sh.cpu(), flags)
    # the scores carry the Q~K transform's split-fp16 error into the softmax:
    # bound scaled by 4 (|score| <~ 10 here)
    err_f = ((got[rb:re].double() - ref[rb:re]).abs() / (mag[rb:re] + 1e-30)).max().item()
    err_l = ((launches[rb:re].double() - ref[rb:re]).abs() / (mag[rb:re] + 1e-30)).max().item()
    assert err_f <= 1.6e-5 and err_l <= 1.6e-5, (err_f, err_l)
    d = (got[rb:re] - launches[rb:re]).abs().max().item()
    assert d <= 2e-5 * max(1.0, ref[rb:re].abs().max().item()), d


def test_transformer_fused_many_blocks():
    """The fused TransformerConv layer against its launch sequence on every
    row of a 200k-row irregular graph (degrees 0-12, hubs): 1563 blocks,
    several per CU over the launch -- the small-graph test above launches
    fewer blocks than there are CUs (a two-blocks-per-CU variant of this
    kernel went wrong only here)."""
    n = 200_000
    ei = _graph(n, 31)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    g = torch.Generator(device=DEV).manual_seed(15)
    x = torch.randn(n, H, device=DEV, generator=g)
    wqk = torch.randn(4 * H, H, device=DEV, generator=g) / 16
    bqk = torch.randn(4 * H, device=DEV, generator=g) * 0.1
    wout = torch.randn(H, 4 * H + 4 + H, device=DEV, generator=g) / (4 * H + 4 + H) ** 0.5
    bout = torch.randn(H, device=DEV, generator=g) * 0.1
    sc = torch.rand(H, device=DEV, generator=g) + 0.5
    sh = torch.randn(H, device=DEV, generator=g) * 0.1
    outs = []
    for fused in (True, False):
        o = torch.full((n, H), float("nan"), device=DEV)
        _tf_layer(fused, csr, x, 0, n, wqk, bqk, wout, bout, sc, sh, 15, o)
        outs.append(o)
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max(1).values
    scale = max(1.0, outs[1].abs().max().item())
    assert torch.isfinite(outs[0]).all()
    assert int((d > 2e-5 * scale).sum()) == 0, (int((d > 2e-5 * scale).sum()), d.max().item())


def test_transformer_fused_prep_rejects():
    L = _lib.lib()
    assert L.mignn_transformer_fused_prep_bytes(128, 4) == 0
    assert L.mignn_transformer_fused_prep_bytes(256, 4) == 41 * 16 * 2 * 1024 + 1024
    img = torch.empty(16, dtype=torch.uint8, device=DEV)
    w = torch.zeros(H, 4 * H + 4 + H, device=DEV)
    assert L.mignn_transformer_fused_prep(_lib.ptr(w), 128, 4, _lib.ptr(img), 16, None) == 1
    assert L.mignn_transformer_fused_prep(_lib.ptr(w), 256, 4, _lib.ptr(img), 16, None) == 1


@pytest.mark.parametrize("flags", [15, 1 | 2])
def test_gin_layer0_fused_vs_fp64_and_two_step(flags):
    """mignn_gin_layer0_fused (input_proj composed into GIN layer 0's
    aggregate: a_i = W_in (sum_j pos_j + (1+eps) pos_i) + (deg_i+1+eps) b_in,
    residual recomputed from pos_i) against a float64 restatement of
    input_proj -> GINConv -> epilogue, and against the two-step route it
    replaces (input_proj, then mignn_gin_layer_fused); hub rows, empty rows,
    a row range."""
    n = 3000
    rb, re = 77, 2950
    ei = _graph(n, 51)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    g = torch.Generator(device=DEV).manual_seed(flags + 3)
    pos = torch.rand(n, 3, device=DEV, generator=g) * 10
    w_in = torch.randn(H, 3, device=DEV, generator=g) / 3 ** 0.5
    b_in = torch.randn(H, device=DEV, generator=g) * 0.1
    _, w1, w2, b1, b2, sc, sh = _params(9, scaled_rows=False)
    eps = 0.2
    L = _lib.lib()
    P = _lib.ptr
    img1, img2 = f16x3_image(w1), gin_fused_image(w2)
    got = torch.full((n, H), float("nan"), device=DEV)
    _lib.check(L.mignn_gin_layer0_fused(P(csr.row_ptr), P(csr.col), P(pos), 3, 3, rb, re, H, eps,
                                        P(w_in), P(b_in), P(img1), P(b1), P(img2), P(b2), P(sc),
                                        P(sh), flags, P(got), H, _lib.stream()), "gin0_fused")
    x0 = (pos @ w_in.T + b_in).contiguous()
    two = torch.full((n, H), float("nan"), device=DEV)
    _lib.check(L.mignn_gin_layer_fused(P(csr.row_ptr), P(csr.col), P(x0), H, rb, re, H, eps,
                                       P(img1), P(b1), P(img2), P(b2), P(sc), P(sh), flags, P(two),
                                       H, _lib.stream()), "gin_fused")
    torch.cuda.synchronize()
    col, dst = _csr_edges(csr, n)
    X = pos.double().cpu() @ w_in.double().cpu().T + b_in.double().cpu()
    a = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, X[col]) + (1 + eps) * X
    am = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, X[col].abs()) + (1 + eps) * X.abs()
    W1, W2 = w1.double().cpu(), w2.double().cpu()
    h = (a @ W1.T + b1.double().cpu()).clamp_min(0)
    hm = am @ W1.T.abs() + b1.double().cpu().abs()
    ref, mag = _epi64(h @ W2.T, hm @ W2.T.abs(), X, b2.cpu(), sc.cpu(), sh.cpu(), flags)
    g_cpu, t_cpu = got.cpu(), two.cpu()
    _check(g_cpu[rb:re], ref[rb:re], mag[rb:re], f"gin0 flags={flags}")
    _check(t_cpu[rb:re], ref[rb:re], mag[rb:re], f"gin two-step flags={flags}")
    assert torch.isnan(g_cpu[:rb]).all() and torch.isnan(g_cpu[re:]).all()
    d = (g_cpu[rb:re] - t_cpu[rb:re]).abs().max().item()
    assert d <= 4e-6 * max(1.0, ref[rb:re].abs().max().item()), d


@pytest.mark.parametrize("h", [64, 128])
@pytest.mark.parametrize("flags", [15, 1 | 2])
def test_gat_layer0_fused_vs_fp64_and_two_step(h, flags):
    """mignn_gat_layer0_fused (input_proj composed into GAT layer 0: logits
    through [wlog W_in | wlog b_in], weighted sums W_in P + S b_in, residual
    recomputed) against a float64 restatement of input_proj -> GATConv ->
    epilogue and against the two-step route (input_proj, then
    mignn_gat_layer's fused kernel); hub rows, empty rows, a row range."""
    n = 4000
    rb, re = 29, 3981
    ei = _graph(n, 61)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator(device=DEV).manual_seed(h + flags + 5)
    pos = torch.rand(n, 3, device=DEV, generator=g) * 4
    w_in = torch.randn(h, 3, device=DEV, generator=g) / 3 ** 0.5
    b_in = torch.randn(h, device=DEV, generator=g) * 0.1
    wlog = torch.randn(8, h, device=DEV, generator=g) / h ** 0.5
    wcat = torch.randn(h, 4 * h, device=DEV, generator=g) / (2 * h) ** 0.5
    bias = torch.randn(h, device=DEV, generator=g) * 0.1
    sc = torch.rand(h, device=DEV, generator=g) + 0.5
    sh = torch.randn(h, device=DEV, generator=g) * 0.1
    img = f16x3_image(wcat)
    lw = torch.zeros(8, 4, dtype=torch.float64, device=DEV)
    lw[:, :3] = wlog.double() @ w_in.double()
    lw[:, 3] = wlog.double() @ b_in.double()
    lw = lw.float().contiguous()
    L = _lib.lib()
    P = _lib.ptr
    got = torch.full((n, h), float("nan"), device=DEV)
    _lib.check(L.mignn_gat_layer0_fused(P(csr.row_ptr), P(csr.col), P(pos), 3, 3, rb, re, h, 0.2,
                                        P(w_in), P(b_in), P(lw), P(img), P(bias), P(sc), P(sh),
                                        flags, P(got), h, _lib.stream()), "gat0_fused")
    x0 = (pos @ w_in.T + b_in).contiguous()
    two = torch.full((n, h), float("nan"), device=DEV)
    _gat_layer(csr, x0, n, rb, re, h, wlog, wcat, img, bias, sc, sh, flags, two)
    torch.cuda.synchronize()
    col, dst = _csr_edges(csr, n)
    X = pos.double().cpu() @ w_in.double().cpu().T + b_in.double().cpu()
    lg = X @ wlog.double().cpu().T
    s = lg[col, :4] + lg[dst, 4:]
    s = torch.where(s > 0, s, 0.2 * s)
    mx = torch.full((n, 4), -float("inf"), dtype=torch.float64).scatter_reduce(
        0, dst[:, None].expand_as(s), s, "amax", include_self=True)
    pexp = torch.exp(s - mx[dst])
    sm = torch.zeros((n, 4), dtype=torch.float64).index_add_(0, dst, pexp) + 1e-16
    alpha = pexp / sm[dst]
    agg = torch.zeros((n, 4, h), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col][:, None, :]).reshape(n, 4 * h)
    aggm = torch.zeros((n, 4, h), dtype=torch.float64).index_add_(
        0, dst, alpha[:, :, None] * X[col].abs()[:, None, :]).reshape(n, 4 * h)
    W = wcat.double().cpu()
    ref, mag = _epi64(agg @ W.T, aggm @ W.T.abs(), X, bias.cpu(), sc.cpu(), sh.cpu(), flags)
    g_cpu, t_cpu = got.cpu(), two.cpu()
    _check(g_cpu[rb:re], ref[rb:re], mag[rb:re], f"gat0 h={h}")
    _check(t_cpu[rb:re], ref[rb:re], mag[rb:re], f"gat two-step h={h}")
    assert torch.isnan(g_cpu[:rb]).all() and torch.isnan(g_cpu[re:]).all()


@pytest.mark.parametrize("hidden", [64, 128, 256])
def test_transformer_layer0_coords_matches_two_step(hidden, monkeypatch):
    """TransformerConv layer 0 collapsed to 3-vectors (mignn_transformer_layer0_coords:
    input_proj, Q~K, softmax, value / skip transforms, residual and BN composed
    in fp64) against the model's own two-step route (input_proj, then the
    layer) on a graph with empty and hub rows, 2-layer model with BN; and the
    whole model against the fp64 oracle."""
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    from oracle import flowgnn_oracle as orc
    n = 3000
    ei = _graph(n, 71)
    g = torch.Generator(device=DEV).manual_seed(hidden)
    x = torch.rand(n, 3, device=DEV, generator=g) * 2 - 1
    cfg = dict(hidden_dim=hidden, num_layers=2, layer_type="Transformer")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=hidden)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    with torch.no_grad():
        m.fuse_layer0 = True
        y1 = m(x, ei)
        m.fuse_layer0 = False
        y0 = m(x, ei)
    scale = max(1.0, y0.abs().max().item())
    assert (y1 - y0).abs().max().item() <= 2e-5 * scale
    r64 = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    err = (y1.cpu().double() - r64).abs().max().item()
    assert err <= 2e-5 * max(1.0, r64.abs().max().item()), err


@pytest.mark.parametrize("hidden", [64, 128, 256])
def test_gat_layer0_coords_matches_two_step(hidden, monkeypatch):
    """GATConv layer 0 collapsed to 3-vectors (mignn_gat_layer0_coords) against
    the model's two-step route (input_proj, then the fused layer) on a graph
    with empty and hub rows, and the model against the fp64 oracle."""
    from mignn import FlowGNN
    from mignn.synthetic import seeded_state_dict
    from oracle import flowgnn_oracle as orc
    n = 3000
    ei = _graph(n, 81)
    g = torch.Generator(device=DEV).manual_seed(hidden + 1)
    x = torch.rand(n, 3, device=DEV, generator=g) * 2 - 1
    cfg = dict(hidden_dim=hidden, num_layers=2, layer_type="GAT")
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=hidden + 1)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    m.gat_coords = True
    with torch.no_grad():
        m.fuse_layer0 = True
        y1 = m(x, ei)
        m.fuse_layer0 = False
        y0 = m(x, ei)
    scale = max(1.0, y0.abs().max().item())
    assert (y1 - y0).abs().max().item() <= 2e-5 * scale
    r64 = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    err = (y1.cpu().double() - r64).abs().max().item()
    assert err <= 2e-5 * max(1.0, r64.abs().max().item()), err


@pytest.mark.parametrize("hidden", [64, 128, 256])
def test_gat_layer0_coords_next_logits(hidden):
    """The shard-only route of GAT layer 0 (FlowGNNShard, mignn.dist): the
    collapsed layer 0 (mignn_gat_layer0_coords) with logits_next forms layer
    1's logits in its epilogue.  Direct parity on a row range: the output rows
    equal the launch without logits_next (bitwise), and the logits match the
    GEMV out . wlog_next^T (fp64) of those rows; rows outside stay unwritten."""
    from mignn import FlowGNN
    from mignn.gnn_model import CSR_ONE_SELF_LOOP
    from mignn.synthetic import seeded_state_dict
    n = 3000
    rb, re = 37, 2950
    ei = _graph(n, 83)
    g = torch.Generator(device=DEV).manual_seed(hidden + 9)
    x = torch.rand(n, 3, device=DEV, generator=g) * 2 - 1
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, hidden_dim=hidden, num_layers=2,
                layer_type="GAT")
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=hidden + 9))
    m = m.to(DEV).eval()
    m.gat_coords = True
    csr = m._csr.get(ei, n, CSR_ONE_SELF_LOOP, None)
    pos = m._coords(x, csr)
    with torch.no_grad():
        out0 = torch.full((n, hidden), float("nan"), device=DEV)
        m._gat_layer0(csr, pos, rb, re, out0)
        out1 = torch.full_like(out0, float("nan"))
        lg = torch.full((n, 8), float("nan"), device=DEV)
        m._gat_layer0(csr, pos, rb, re, out1, logits_next=lg)
        wlog_n, _ = m._gat_weights(m.gnn_layers[1])
    torch.cuda.synchronize()
    assert torch.equal(out0[rb:re], out1[rb:re])
    assert torch.isnan(out1[:rb]).all() and torch.isnan(out1[re:]).all()
    assert torch.isnan(lg[:rb]).all() and torch.isnan(lg[re:]).all()
    ref = out1[rb:re].double() @ wlog_n.double().t()
    err = (lg[rb:re].double() - ref).abs().max().item()
    assert err <= 2e-6 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("h", [64, 128, 256])
@pytest.mark.parametrize("fused", [1, 0])
def test_gat_layer_next_logits(h, fused):
    """mignn_gat_layer_next: the same output rows as mignn_gat_layer, plus the
    next layer's logits of those rows (out . wlog_next^T), from the fused
    kernel's epilogue (fused) or a GEMV after the launch sequence (0)."""
    n = 3000
    rb, re = 40, 2960
    ei = _graph(n, 91)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    g = torch.Generator(device=DEV).manual_seed(h + 3 * fused)
    x = torch.randn(n, h, device=DEV, generator=g)
    wlog = torch.randn(8, h, device=DEV, generator=g) / h ** 0.5
    wnext = torch.randn(8, h, device=DEV, generator=g) / h ** 0.5
    wcat = torch.randn(h, 4 * h, device=DEV, generator=g) / (2 * h) ** 0.5
    bias = torch.randn(h, device=DEV, generator=g) * 0.1
    sc = torch.rand(h, device=DEV, generator=g) + 0.5
    sh = torch.randn(h, device=DEV, generator=g) * 0.1
    img = f16x3_image(wcat)
    L = _lib.lib()
    P = _lib.ptr
    lf = 0 if fused else GAT_LAUNCHES
    if True:
        ref = torch.full((n, h), float("nan"), device=DEV)
        _gat_layer(csr, x, n, rb, re, h, wlog, wcat, img, bias, sc, sh, 15 | lf, ref)
        out = torch.full((n, h), float("nan"), device=DEV)
        lg = torch.full((n, 8), float("nan"), device=DEV)
        nb = L.mignn_gat_layer_scratch_bytes(n, re - rb, h, 4)
        scratch = torch.empty(max(nb, 1), dtype=torch.uint8, device=DEV)
        _lib.check(L.mignn_gat_layer_next(P(csr.row_ptr), P(csr.col), P(x), h, n, rb, re, h, 4, 0.2,
                                          P(wlog), None, 8, P(wcat), P(img), P(bias), P(sc), P(sh),
                                          15 | lf, P(scratch), nb, P(out), h, P(wnext), P(lg),
                                          _lib.stream()), "gat_layer_next")
        torch.cuda.synchronize()
    assert torch.equal(out[rb:re], ref[rb:re])
    want = out[rb:re].double() @ wnext.double().T
    err = (lg[rb:re].double() - want).abs().max().item()
    assert err <= 1e-5 * max(1.0, want.abs().max().item()), err
    assert torch.isnan(lg[:rb]).all() and torch.isnan(lg[re:]).all()


