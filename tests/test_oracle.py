"""Pin the CPU oracle (oracle/flowgnn_oracle.py) before trusting it.

1. Against the committed golden vectors produced by running the reference's
   own FlowGNN wrapper (gnn_model.py) on reference-built graphs.
2. Against a second, loop-level restatement of the PyG conv semantics below
   (independent of torch scatter ops) on hand-checkable graphs -- the conv
   arithmetic itself has no reference golden vectors (PyG absent: parity
   unpinned by the reference).
"""

import math

import numpy as np
import pytest
import torch

from helpers import (bfs_graph, model_fixture, model_names, ref_err, surrogate_fixture,
                     surrogate_names, tiny_fixture, tiny_names)
from oracle import flowgnn_oracle as orc

torch.set_num_threads(min(8, torch.get_num_threads()))


@pytest.mark.parametrize("name", model_names())
def test_oracle_matches_reference_wrapper(name):
    cfg, sd, outs, _ = model_fixture(name)
    for gname, (y32, y64) in outs.items():
        x, ei, ea = bfs_graph(gname)
        ea_in = None if cfg["layer_type"] == "Transformer" else ea
        got = orc.flowgnn_forward(sd, cfg, x, ei, ea_in, dtype=torch.float32)
        # same op sequence as the reference wrapper run -> bitwise equal
        assert torch.equal(got, y32), (name, gname, (got - y32).abs().max())
        got64 = orc.flowgnn_forward(sd, cfg, x, ei, ea_in, dtype=torch.float64)
        assert torch.allclose(got64, y64, rtol=0, atol=1e-12)
        # fp32 CPU forward vs fp64: the accuracy floor the GPU is compared with
        # (outputs are O(1)..O(10): fp32 rounding alone gives ~1e-7 relative)
        d = (y32.double() - y64).abs().max().item()
        assert d == pytest.approx(ref_err(name, gname), rel=1e-9)
        assert d < 2e-6 * max(1.0, y64.abs().max().item())
        # the fixtures are not near-constant: outputs span O(1) (the 1e-5 bound bites)
        assert y64.abs().max().item() > 0.3 and y64.std().item() > 0.05


@pytest.mark.parametrize("name", surrogate_names())
def test_oracle_matches_reference_surrogate(name):
    """FlowGNNSurrogate (gnn_model.py:223-291) = decoder(encoder(x) + bc):
    the oracle composition reproduces the reference's own module run."""
    cfg, sd, bc, outs = surrogate_fixture(name)
    x, ei, ea = bfs_graph("train")
    half = dict(cfg, num_layers=cfg["num_layers"] // 2)
    enc = {k[8:]: v for k, v in sd.items() if k.startswith("encoder.")}
    dec = {k[8:]: v for k, v in sd.items() if k.startswith("decoder.")}
    for tag, b in (("nobc", None), ("bc", bc)):
        y32, y64 = outs[tag]
        e = orc.flowgnn_forward(enc, half, x, ei, ea, dtype=torch.float32)
        if b is not None:
            e = e + b
        got = orc.flowgnn_forward(dec, half, e, ei, ea, dtype=torch.float32)
        assert torch.equal(got, y32), (name, tag)
        assert got.shape[1] == 8


def test_transformer_edge_attr_raises_like_reference():
    cfg, sd, _, err = model_fixture("transformer_h64_l2")
    x, ei, ea = bfs_graph("train")
    with pytest.raises(RuntimeError) as exc:
        orc.flowgnn_forward(sd, cfg, x, ei, ea)
    assert str(exc.value).split("\n")[0] == err


@pytest.mark.parametrize("name", tiny_names())
@pytest.mark.parametrize("lt", ["GCN", "GAT", "GIN", "Transformer"])
def test_oracle_tiny_fixtures(name, lt):
    x, ei, sd, y32, y64 = tiny_fixture(name, lt)
    cfg = dict(hidden_dim=8, num_layers=2, layer_type=lt)
    got = orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float64)
    assert torch.allclose(got, y64, rtol=0, atol=1e-12)


# ---------------------------------------------------------------------------
# Loop-level restatement of PyG semantics (float64, plain Python)
# ---------------------------------------------------------------------------

def _rows_in(ei, n, mode):
    """mode 'gcn': drop self-loops, one per node appended; 'raw': verbatim."""
    rows = {i: [] for i in range(n)}
    for s, d in zip(ei[0].tolist(), ei[1].tolist()):
        if mode == "gcn" and s == d:
            continue
        rows[d].append(s)
    if mode == "gcn":
        for i in range(n):
            rows[i].append(i)
    return rows


def loop_gcn(x, ei, W, b):
    n = x.shape[0]
    h = x @ W.T
    rows = _rows_in(ei, n, "gcn")
    deg = [len(rows[i]) for i in range(n)]
    out = np.zeros_like(h)
    for i in range(n):
        for j in rows[i]:
            out[i] += h[j] / math.sqrt(deg[j] * deg[i])
    return out + b


def loop_gat(x, ei, W, asrc, adst, b, heads):
    n = x.shape[0]
    C = W.shape[0] // heads
    h = (x @ W.T).reshape(n, heads, C)
    a_s = (h * asrc.reshape(1, heads, C)).sum(-1)
    a_d = (h * adst.reshape(1, heads, C)).sum(-1)
    rows = _rows_in(ei, n, "gcn")
    out = np.zeros((n, heads, C))
    for i in range(n):
        for hd in range(heads):
            e = [a_s[j, hd] + a_d[i, hd] for j in rows[i]]
            e = [v if v > 0 else 0.2 * v for v in e]
            m = max(e)
            p = [math.exp(v - m) for v in e]
            s = sum(p) + 1e-16
            for j, pj in zip(rows[i], p):
                out[i, hd] += pj / s * h[j, hd]
    return out.mean(1) + b


def loop_gin(x, ei, eps, W1, b1, W2, b2):
    n = x.shape[0]
    agg = np.zeros_like(x)
    for s, d in zip(ei[0].tolist(), ei[1].tolist()):
        agg[d] += x[s]
    z = agg + (1 + eps) * x
    return np.maximum(z @ W1.T + b1, 0) @ W2.T + b2


def loop_transformer(x, ei, Wq, bq, Wk, bk, Wv, bv, Ws, bs, heads):
    n = x.shape[0]
    C = Wq.shape[0] // heads
    q = (x @ Wq.T + bq).reshape(n, heads, C)
    k = (x @ Wk.T + bk).reshape(n, heads, C)
    v = (x @ Wv.T + bv).reshape(n, heads, C)
    rows = _rows_in(ei, n, "raw")
    out = np.zeros((n, heads, C))
    for i in range(n):
        if not rows[i]:
            continue
        for hd in range(heads):
            sc = [float(q[i, hd] @ k[j, hd]) / math.sqrt(C) for j in rows[i]]
            m = max(sc)
            p = [math.exp(s - m) for s in sc]
            tot = sum(p) + 1e-16
            for j, pj in zip(rows[i], p):
                out[i, hd] += pj / tot * v[j, hd]
    return out.mean(1) + x @ Ws.T + bs


GRAPHS = {
    "path": (6, [[0, 1, 1, 2, 2, 3, 3, 4, 4, 5], [1, 0, 2, 1, 3, 2, 4, 3, 5, 4]]),
    "selfloops_dups": (5, [[0, 0, 0, 1, 2, 1, 4, 2, 2], [0, 0, 1, 0, 1, 2, 2, 3, 3]]),
    "isolated": (4, [[0, 1], [1, 0]]),
}


@pytest.mark.parametrize("gname", list(GRAPHS))
def test_conv_semantics_loop_restatement(gname):
    n, e = GRAPHS[gname]
    rng = np.random.default_rng(3)
    H, heads = 6, 4
    x = rng.standard_normal((n, H))
    ei = np.array(e, dtype=np.int64)
    T = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float64))  # noqa: E731
    tei = torch.from_numpy(ei)
    W = rng.standard_normal((H, H)) * 0.3
    b = rng.standard_normal(H) * 0.1
    np.testing.assert_allclose(orc.gcn_conv(T(x), tei, T(W), T(b)).numpy(),
                               loop_gcn(x, ei, W, b), atol=1e-12)
    Wg = rng.standard_normal((heads * H, H)) * 0.3
    asrc, adst = rng.standard_normal((heads, H)), rng.standard_normal((heads, H))
    np.testing.assert_allclose(
        orc.gat_conv(T(x), tei, T(Wg), T(asrc).view(1, heads, H), T(adst).view(1, heads, H),
                     T(b), heads).numpy(),
        loop_gat(x, ei, Wg, asrc, adst, b, heads), atol=1e-12)
    W1, W2 = rng.standard_normal((H, H)) * 0.3, rng.standard_normal((H, H)) * 0.3
    b1, b2 = rng.standard_normal(H) * 0.1, rng.standard_normal(H) * 0.1
    for eps in (0.0, 0.25):
        np.testing.assert_allclose(
            orc.gin_conv(T(x), tei, eps, T(W1), T(b1), T(W2), T(b2)).numpy(),
            loop_gin(x, ei, eps, W1, b1, W2, b2), atol=1e-12)
    Wq, Wk, Wv = (rng.standard_normal((heads * H, H)) * 0.3 for _ in range(3))
    bq, bk, bv = (rng.standard_normal(heads * H) * 0.1 for _ in range(3))
    Ws, bs = rng.standard_normal((H, H)) * 0.3, rng.standard_normal(H) * 0.1
    np.testing.assert_allclose(
        orc.transformer_conv(T(x), tei, T(Wq), T(bq), T(Wk), T(bk), T(Wv), T(bv), T(Ws), T(bs),
                             heads).numpy(),
        loop_transformer(x, ei, Wq, bq, Wk, bk, Wv, bv, Ws, bs, heads), atol=1e-12)
