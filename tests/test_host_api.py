"""Host-side contract of the engine (no GPU needed): C-ABI exports, the
FlowGNN constructor / state_dict layout / error behaviour of the reference
(gnn_model.py:14-220), Data/Batch, and the weight re-association algebra the
GAT / TransformerConv kernels rely on (emulated on the CPU in float64)."""

import ctypes
import math
import os
import re

import pytest
import torch

from helpers import model_fixture, model_names
import mignn
from mignn import _lib
from mignn.data import Batch, Data
from mignn.gnn_model import FlowGNN, HEADS
from oracle import flowgnn_oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "mignn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mignn_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(_lib.LIB_PATH), "build libmignn.so first (__graft_entry__.build())"
    h = ctypes.CDLL(_lib.LIB_PATH)
    funcs = header_functions()
    assert len(funcs) >= 14
    for f in funcs:
        assert hasattr(h, f), f"{f} declared in include/mignn.h but not exported"
    assert set(funcs) == set(_lib.SIGNATURES), "ctypes signature table out of sync with header"
    assert _lib.lib().mignn_abi_version() == 1


def _dynamic_symbols(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True,
                         text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_product_library_has_no_diagnostic_state():
    """libmignn.so (what the product path loads) exports no timing-study entry
    (mignn_diag_*) and exactly the C functions of include/mignn.h: ablation
    switches and traces live only in libmignn_diag.so (built from the same
    sources with -DMIGNN_DIAG), so no call can change a later product launch."""
    syms = {s for s in _dynamic_symbols(_lib.LIB_PATH) if s.startswith("mignn_")}
    assert not {s for s in syms if s.startswith("mignn_diag")}, sorted(syms)
    assert syms == set(header_functions()), sorted(syms ^ set(header_functions()))
    diag = {s for s in _dynamic_symbols(_lib.DIAG_LIB_PATH) if s.startswith("mignn_diag")}
    assert diag == set(_lib.DIAG_SIGNATURES), sorted(diag ^ set(_lib.DIAG_SIGNATURES))


@pytest.mark.parametrize("name", model_names())
def test_state_dict_layout_matches_reference(name):
    cfg, sd, _, _ = model_fixture(name)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    mine = m.state_dict()
    assert list(mine.keys()) == list(sd.keys())
    for k in sd:
        assert tuple(mine[k].shape) == tuple(sd[k].shape), k
    m.load_state_dict(sd, strict=True)


def test_gat_legacy_key_layout_loads():
    cfg, sd, _, _ = model_fixture("gat_h64_l2")
    legacy = {}
    for k, v in sd.items():
        if k.endswith(".lin.weight") and k.startswith("gnn_layers"):
            legacy[k.replace(".lin.weight", ".lin_src.weight")] = v
            legacy[k.replace(".lin.weight", ".lin_dst.weight")] = v
        else:
            legacy[k] = v
    m = FlowGNN(input_dim=3, output_dim=7, **cfg)
    m.load_state_dict(legacy, strict=True)
    assert torch.equal(m.gnn_layers[0].lin.weight, sd["gnn_layers.0.lin.weight"])


def test_errors_mirror_reference():
    with pytest.raises(ValueError, match="Unknown layer type"):
        FlowGNN(layer_type="SAGE")
    m = FlowGNN(hidden_dim=16, num_layers=1).eval()
    with pytest.raises(ValueError, match=r"edge_index must have shape \[2, num_edges\]"):
        m(torch.zeros(4, 3), torch.zeros(3, 5, dtype=torch.long))
    # no CPU path: the product refuses CPU tensors loudly
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        m(torch.zeros(4, 3), torch.zeros(2, 5, dtype=torch.long))
    # model.train(): GCN trains on the device (CPU tensors refused the same
    # every layer type trains on the device
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        m.train()(torch.zeros(4, 3), torch.zeros(2, 5, dtype=torch.long))
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        FlowGNN(hidden_dim=16, num_layers=1, layer_type="Transformer").train()(
            torch.zeros(4, 3), torch.zeros(2, 5, dtype=torch.long))


def test_weighted_mse_loss_host_side():
    from mignn.normalization import WeightedMSELoss
    crit = WeightedMSELoss()
    assert crit.field_weights["p"] == 3.0 and crit.use_fieldwise and crit.pressure_ref_weight == 0.1
    assert crit.weights.tolist() == [1.0, 1.0, 1.0, 3.0, 0.5, 0.5, 0.5]
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        crit(torch.zeros(4, 7), torch.zeros(4, 7))


def test_predict_fields_slices():
    m = FlowGNN(hidden_dim=16, num_layers=1, output_dim=8)
    out = torch.arange(16.0).view(2, 8)
    f = m.predict_fields(out)
    assert f["U"].shape == (2, 3) and f["p"][0, 0] == 3 and f["nut"][1, 0] == 14
    assert "residual" in f and f["residual"][0, 0] == 7
    assert "residual" not in m.predict_fields(out[:, :7])


def test_data_and_batch():
    d1 = Data(x=torch.zeros(3, 3), edge_index=torch.tensor([[0, 1], [1, 2]]),
              edge_attr=torch.zeros(2, 4), num_nodes=3)
    d2 = Data(x=torch.ones(2, 3), edge_index=torch.tensor([[0], [1]]), edge_attr=torch.ones(1, 4),
              y=None, num_nodes=2)
    assert d1.num_nodes == 3 and d1.num_edges == 2
    b = Batch.from_data_list([d1, d2])
    assert b.num_nodes == 5 and b.edge_index.tolist() == [[0, 1, 3], [1, 2, 4]]
    assert b.batch.tolist() == [0, 0, 0, 1, 1] and b.edge_attr.shape == (3, 4)
    assert b.to("cpu").x.shape == (5, 3)


def test_surrogate_structure():
    s = mignn.FlowGNNSurrogate(hidden_dim=16, num_layers=4)
    assert s.encoder.num_layers == 2 and s.decoder.input_dim == 16 and s.decoder.output_dim == 8


# ---------------------------------------------------------------------------
# The re-associated weights reproduce the reference conv math (float64 CPU
# emulation of the kernel dataflow: aggregate on x, then one GEMM).
# ---------------------------------------------------------------------------

def _graph(n=40, e=160, seed=0):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=g)
    x = torch.randn(n, 16, generator=g, dtype=torch.float64)
    return x, ei


def test_gat_reassociation_algebra():
    H = 16
    layer = mignn.gnn_model.GATConv(H, H)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in layer.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    x, ei = _graph()
    ref = orc.gat_conv(x, ei, layer.lin.weight.double(), layer.att_src.double(),
                       layer.att_dst.double(), layer.bias.double(), HEADS)
    wlog, wcat = FlowGNN._gat_weights(layer)
    logits = x @ wlog.double().T                          # [N, 2*heads]
    ei2 = orc.add_self_loops(orc.remove_self_loops(ei), x.shape[0])
    alpha = logits[ei2[0], :HEADS] + logits[ei2[1], HEADS:]
    alpha = orc.segment_softmax(torch.nn.functional.leaky_relu(alpha, 0.2), ei2[1], x.shape[0])
    agg = torch.zeros(x.shape[0], HEADS, H, dtype=torch.float64)
    agg.index_add_(0, ei2[1], alpha.unsqueeze(-1) * x[ei2[0]].unsqueeze(1))
    got = agg.reshape(x.shape[0], -1) @ wcat.double().T + layer.bias.double()
    assert (got - ref).abs().max().item() < 1e-5   # wlog/wcat are rounded to fp32


def test_transformer_reassociation_algebra():
    H = 16
    layer = mignn.gnn_model.TransformerConv(H, H)
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():
        for p in layer.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    x, ei = _graph(seed=3)
    d = lambda t: t.detach().double()  # noqa: E731
    ref = orc.transformer_conv(x, ei, d(layer.lin_query.weight), d(layer.lin_query.bias),
                               d(layer.lin_key.weight), d(layer.lin_key.bias),
                               d(layer.lin_value.weight), d(layer.lin_value.bias),
                               d(layer.lin_skip.weight), d(layer.lin_skip.bias), HEADS)
    wqk, bqk, wout, bout = (t.double() for t in FlowGNN._tf_weights(layer))
    n = x.shape[0]
    qt = x @ wqk.T + bqk                                  # [N, heads*H]
    assert qt.shape[1] == HEADS * H
    src, dst = ei[0], ei[1]
    q = qt.view(n, HEADS, H)
    # no q_i . b_k term: constant over a row's entries, cancelled by the softmax
    s = (q[dst] * x[src].unsqueeze(1)).sum(-1) / math.sqrt(H)
    a = orc.segment_softmax(s, dst, n)
    agg = torch.zeros(n, HEADS, H, dtype=torch.float64).index_add_(0, dst, a.unsqueeze(-1) * x[src].unsqueeze(1))
    sig = torch.zeros(n, HEADS, dtype=torch.float64).index_add_(0, dst, a)
    A = torch.cat([agg.reshape(n, -1), sig, x], 1)
    got = A @ wout.T + bout
    assert (got - ref).abs().max().item() < 1e-5


def test_attention_layer_entry_points_validate_before_launching():
    """mignn_gat_layer / mignn_transformer_layer (csrc/attn_layers.hip) reject
    bad arguments with MIGNN_ERR_ARG and a message before any device work, and
    report their scratch sizes (host-only paths: no GPU needed)."""
    L = _lib.lib()
    buf = (ctypes.c_float * 4096)()
    p = ctypes.addressof(buf)          # never dereferenced: validation fails first
    al = (p + 255) & ~255
    # scratch sizes: [n_x, 2 heads] logits + [rows, heads h] aggregate, 256-B aligned
    assert L.mignn_gat_layer_scratch_bytes(10, 4, 8, 4) == 512 + 512
    assert L.mignn_gat_layer_scratch_bytes(0, 4, 8, 4) == 512
    assert L.mignn_gat_layer_scratch_bytes(-1, 4, 8, 4) == 0
    # q~ and aggregate [rows, heads h + heads] each
    assert L.mignn_transformer_layer_scratch_bytes(4, 8, 4) == 2 * 768
    assert L.mignn_transformer_layer_scratch_bytes(4, 0, 4) == 0

    def gat(flags=0, x=p, rb=0, re=4, scratch=al, nbytes=1024):
        return L.mignn_gat_layer(p, p, x, 8, 10, rb, re, 8, 4, 0.2, p, None, 8, p, None, None,
                                 None, None, flags, scratch, nbytes, p, 8, None)

    assert gat(rb=0, re=0) == 0                     # empty range: nothing to do
    for kw, msg in [({"flags": 1 << 30}, "unknown flags"), ({"x": None}, "null pointer"),
                    ({"rb": 5, "re": 4}, "bad row range"), ({"re": 11}, "bad row range"),
                    ({"nbytes": 1023}, "scratch"), ({"scratch": al + 4}, "scratch")]:
        assert gat(**kw) == 1, kw
        assert msg in _lib.last_error(), (kw, _lib.last_error())

    def tf(flags=0, bqk=p, rb=0, re=4, nbytes=1536):
        return L.mignn_transformer_layer(p, p, p, 8, rb, re, 8, 4, 0.35, p, None, bqk, p, None,
                                         p, None, None, flags, al, nbytes, p, 8, None)

    assert tf(re=0) == 0
    for kw, msg in [({"flags": 1 << 30}, "unknown flags"), ({"bqk": None}, "null pointer"),
                    ({"rb": 3, "re": 2}, "bad row range"), ({"nbytes": 1535}, "scratch")]:
        assert tf(**kw) == 1, kw
        assert msg in _lib.last_error(), (kw, _lib.last_error())
