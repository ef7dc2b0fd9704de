"""Aggregation kernels (mignn_{gcn,sum,gat,transformer}_aggregate) against a
float64 torch restatement of the PyG message/aggregate steps on the same CSR.

Graphs: random destination-major edge lists with degrees 0..20 and hub rows
of 40-90 entries (several 8-entry batches per row, the batched kernels'
online-softmax path), both CSR modes, and a row sub-range [rb, re) written at
out + rb * ldo.  The batched kernels (4 heads, the FlowGNN widths) and the
entry-at-a-time kernels (any other head count / width: h = 20 / 48 / 40
below) are held to the same bound: fp32 accumulation error relative to the
sum of |terms| of each output.
"""

import math

import pytest
import torch

from mignn import _lib
from mignn.gnn_model import build_csr

pytestmark = pytest.mark.gpu
DEV = "cuda"
HEADS = 4


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


def _graph(n, seed, hubs=True):
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, 21, (n,), generator=g)
    if hubs:
        hub = torch.randperm(n, generator=g)[:6]
        deg[hub] = torch.randint(40, 91, (6,), generator=g)
    dst = torch.repeat_interleave(torch.arange(n), deg)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    perm = torch.randperm(dst.numel(), generator=g)          # edge order != CSR order
    return torch.stack([src[perm], dst[perm]]).to(DEV)


def _edges(csr, n):
    rp = csr.row_ptr.cpu().long()
    col = csr.col.cpu().long()[: int(rp[-1])]
    dst = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    return col, dst


def _seg_softmax(s, dst, n):
    """PyG utils.softmax over rows: exp(s - max) / (sum + 1e-16), float64."""
    mx = torch.full((n, s.shape[1]), -math.inf, dtype=s.dtype)
    mx = mx.scatter_reduce(0, dst[:, None].expand_as(s), s, "amax", include_self=True)
    p = torch.exp(s - mx[dst])
    sm = torch.zeros((n, s.shape[1]), dtype=s.dtype).index_add_(0, dst, p) + 1e-16
    return p / sm[dst]


def _check(got, ref, mag, what, deg=None):
    """|err| <= 4e-7 |terms|; softmax aggregations: 1e-6 |terms| (fp32 exp
    of scores up to ~30 in magnitude) plus the rounding of the row's exp-sum
    (~deg ulps of every alpha)"""
    err = (got.double() - ref).abs()
    rel = 4e-7 if deg is None else 1e-6 + 1.2e-7 * deg.double()[:, None]
    bound = rel * mag + 1e-30
    bad = (err > bound)
    assert not bool(bad.any()), (what, float(err.max()), float((err / bound).max()))


def _run(fn):
    out = fn()
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("h", [32, 64, 128, 256, 20])
def test_sum_and_gcn_aggregate(h):
    n = 3000
    ei = _graph(n, 11 + h)
    g = torch.Generator().manual_seed(h)
    x = torch.randn(n, h, generator=g, dtype=torch.float64)
    xd = x.float().to(DEV)
    L, P = _lib.lib(), _lib.ptr
    rb, re = 117, n - 5
    # GIN: verbatim CSR
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    col, dst = _edges(csr, n)
    out = torch.full((n, h), float("nan"), device=DEV)
    _run(lambda: _lib.check(L.mignn_sum_aggregate(
        P(csr.row_ptr), P(csr.col), P(xd), h, 1.25, rb, re, h, P(out), h, _lib.stream(xd.device)), "sum"))
    xr = xd.double().cpu()
    ref = torch.zeros((n, h), dtype=torch.float64).index_add_(0, dst, xr[col]) + 1.25 * xr
    mag = torch.zeros((n, h), dtype=torch.float64).index_add_(0, dst, xr[col].abs()) + 1.25 * xr.abs()
    _check(out[rb:re].cpu(), ref[rb:re], mag[rb:re], f"sum h={h}")
    assert torch.isnan(out[:rb]).all() and torch.isnan(out[re:]).all()
    # GCN: one self-loop per node, gcn_norm weights
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    col, dst = _edges(csr, n)
    dinv = csr.dinv.cpu().double()
    out = torch.full((n, h), float("nan"), device=DEV)
    _run(lambda: _lib.check(L.mignn_gcn_aggregate(
        P(csr.row_ptr), P(csr.col), P(csr.dinv), P(xd), h, rb, re, h, P(out), h,
        _lib.stream(xd.device)), "gcn"))
    w = (dinv[col] * dinv[dst])[:, None]
    ref = torch.zeros((n, h), dtype=torch.float64).index_add_(0, dst, w * xr[col])
    mag = torch.zeros((n, h), dtype=torch.float64).index_add_(0, dst, (w * xr[col]).abs())
    _check(out[rb:re].cpu(), ref[rb:re], mag[rb:re], f"gcn h={h}")


@pytest.mark.parametrize("h", [32, 64, 128, 256, 48])
def test_gat_aggregate(h):
    n = 2500
    ei = _graph(n, 23 + h)
    csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
    col, dst = _edges(csr, n)
    g = torch.Generator().manual_seed(h + 1)
    x = torch.randn(n, h, generator=g).to(DEV)
    logits = (torch.randn(n, 2 * HEADS, generator=g) * 3).to(DEV)
    L, P = _lib.lib(), _lib.ptr
    rb, re = 9, n - 100
    out = torch.full((n, HEADS * h), float("nan"), device=DEV)
    _run(lambda: _lib.check(L.mignn_gat_aggregate(
        P(csr.row_ptr), P(csr.col), P(logits), P(x), h, rb, re, h, HEADS, 0.2, P(out), HEADS * h,
        _lib.stream(x.device)), "gat"))
    lg = logits.cpu().double()
    s = lg[col, :HEADS] + lg[dst, HEADS:]
    s = torch.where(s > 0, s, 0.2 * s)
    a = _seg_softmax(s, dst, n)                                   # [E, heads]
    xr = x.cpu().double()
    msg = a[:, :, None] * xr[col][:, None, :]                    # [E, heads, h]
    ref = torch.zeros((n, HEADS, h), dtype=torch.float64).index_add_(0, dst, msg).view(n, -1)
    mag = torch.zeros((n, HEADS, h), dtype=torch.float64).index_add_(0, dst, msg.abs()).view(n, -1)
    deg = (csr.row_ptr[1:] - csr.row_ptr[:-1]).cpu()
    _check(out[rb:re].cpu(), ref[rb:re], mag[rb:re] + 1e-7 * ref[rb:re].abs().amax(), f"gat h={h}",
           deg[rb:re])


@pytest.mark.parametrize("h", [64, 128, 256, 40])
def test_transformer_aggregate(h):
    n = 2500
    ei = _graph(n, 37 + h)
    csr = build_csr(ei, n, _lib.CSR_VERBATIM)
    col, dst = _edges(csr, n)
    g = torch.Generator().manual_seed(h + 2)
    x = torch.randn(n, h, generator=g).to(DEV)
    K1 = HEADS * h + HEADS
    qt = (torch.randn(n, K1, generator=g) * 0.3).to(DEV)
    scale = 1.0 / math.sqrt(h)
    L, P = _lib.lib(), _lib.ptr
    rb, re = 33, n
    out = torch.full((n, K1), float("nan"), device=DEV)
    _run(lambda: _lib.check(L.mignn_transformer_aggregate(
        P(csr.row_ptr), P(csr.col), P(qt), K1, P(x), h, rb, re, h, HEADS, scale, P(out), K1,
        _lib.stream(x.device)), "tf"))
    q = qt.cpu().double()
    xr = x.cpu().double()
    qh = q[:, :HEADS * h].view(n, HEADS, h)
    s = ((qh[dst] * xr[col][:, None, :]).sum(-1) + q[dst, HEADS * h:]) * scale   # [E, heads]
    a = _seg_softmax(s, dst, n)
    msg = a[:, :, None] * xr[col][:, None, :]
    ref = torch.zeros((n, HEADS, h), dtype=torch.float64).index_add_(0, dst, msg).view(n, -1)
    asum = torch.zeros((n, HEADS), dtype=torch.float64).index_add_(0, dst, a)
    ref = torch.cat([ref, asum], 1)
    mag = torch.zeros((n, HEADS, h), dtype=torch.float64).index_add_(0, dst, msg.abs()).view(n, -1)
    mag = torch.cat([mag, asum], 1)
    # score rounding (a dot of h fp32 products) perturbs alpha by ~h * 2^-24 |q||x| relative
    sc = (qh.abs()[dst] * xr.abs()[col][:, None, :]).sum(-1).amax() * scale
    deg = (csr.row_ptr[1:] - csr.row_ptr[:-1]).cpu()
    _check(out[rb:re].cpu(), ref[rb:re], mag[rb:re] * (1.0 + float(sc) * 0.5) + 1e-6,
           f"tf h={h}", deg[rb:re])
    # a row with no entries: zeros (not NaN), alpha sum 0
    rp = csr.row_ptr.cpu()
    empty = ((rp[1:] - rp[:-1]) == 0).nonzero().flatten()
    empty = empty[empty >= rb]
    if empty.numel():
        assert (out[empty.to(DEV)] == 0).all()
