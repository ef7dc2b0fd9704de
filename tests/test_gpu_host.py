"""Host-layer behaviour on the GPU: graph-cache keying, caches derived from
BatchNorm running statistics, BatchNorm1d(momentum=None), and the training
path's errors."""

import pytest
import torch

from mignn import FlowGNN, _lib
from mignn.synthetic import grid_graph, seeded_state_dict
from oracle import flowgnn_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


def _model(lt="GCN", H=64, L=2, seed=1):
    cfg = dict(hidden_dim=H, num_layers=L, layer_type=lt)
    m = FlowGNN(input_dim=3, output_dim=7, dropout=0.0, **cfg)
    sd = seeded_state_dict(m.state_dict(), seed=seed)
    m.load_state_dict(sd)
    return m.to(DEV).eval(), sd, cfg


@pytest.mark.parametrize("form", ["int32", "transposed_view"])
def test_csr_cache_distinct_same_size_graphs(form):
    """Two different graphs of the same size passed as int32 (converted
    inside) or as an [E, 2].t() view: the cache key is the caller's tensor,
    which the entry keeps alive, so the second graph never gets the first
    graph's CSR even when the allocator would recycle the address."""
    m, sd, cfg = _model()
    x, _ = grid_graph(10, 9, 8, device=DEV)
    n = x.shape[0]
    for it in range(4):
        _, ei = grid_graph(10, 9, 8, device=DEV, permute_seed=it)   # a relabelled mesh
        if form == "int32":
            ein = ei.to(torch.int32)
        else:
            ein = ei.t().contiguous().t()
        del ei
        with torch.no_grad():
            y = m(x, ein)
        ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ein.cpu().long(), None, dtype=torch.float64)
        assert (y.cpu().double() - ref).abs().max().item() <= 1e-5, it
        del ein


def test_eval_train_eval_uses_updated_running_stats():
    """A train-mode forward updates BN running stats in place (raw-pointer
    kernel writes); the next eval forward must fold the NEW statistics."""
    m, _, cfg = _model()
    x, ei = grid_graph(12, 10, 9, device=DEV)
    with torch.no_grad():
        m(x, ei)                        # fills the eval caches
        m.train()
        m(x, ei)                        # no optimizer step: weights unchanged
        m.eval()
        y = m(x, ei)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = orc.flowgnn_forward(sd, cfg, x.cpu(), ei.cpu(), None, dtype=torch.float64)
    assert (y.cpu().double() - ref).abs().max().item() <= 1e-5


def test_bn_momentum_none_cumulative_average():
    """BatchNorm1d(momentum=None): running stats are the cumulative average
    over batches (factor 1 / num_batches_tracked), as torch computes it."""
    h, n = 48, 3000
    g = torch.Generator().manual_seed(0)
    bn_ref = torch.nn.BatchNorm1d(h, momentum=None)
    bn = torch.nn.BatchNorm1d(h, momentum=None).to(DEV)
    from mignn import train_ops as T
    for it in range(3):
        z = torch.randn(n, h, generator=g) * (1 + it) + it
        bn_ref.train()
        bn_ref(z)
        T.bn_relu_dropout(z.to(DEV), bn, 0.0)
    torch.cuda.synchronize()
    assert int(bn.num_batches_tracked) == 3
    assert torch.allclose(bn.running_mean.cpu(), bn_ref.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(bn.running_var.cpu(), bn_ref.running_var, rtol=1e-5, atol=1e-6)


def test_train_single_node_raises_like_torch():
    m, _, _ = _model()
    m.train()
    x = torch.rand(1, 3, device=DEV)
    ei = torch.zeros(2, 1, dtype=torch.int64, device=DEV)
    with pytest.raises(ValueError, match="Expected more than 1 value per channel when training"):
        m(x, ei)


def test_train_width_limits_named():
    m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=264, num_layers=1,
                layer_type="GAT").to(DEV).train()
    x, ei = grid_graph(4, 4, 4, device=DEV)
    with pytest.raises(NotImplementedError, match="hidden_dim <= 256"):
        m(x, ei)


def test_layer_error_reports_filtered_edges():
    """gnn_model.py:175-181: the message carries the post-filter edge count
    and range (invalid indices dropped, :133-141)."""
    m, _, _ = _model(lt="Transformer")
    x, ei = grid_graph(4, 4, 4, device=DEV)
    n = x.shape[0]
    bad = torch.tensor([[n + 5], [0]], device=DEV)
    ei2 = torch.cat([ei, bad], 1)
    ea = torch.zeros(ei2.shape[1], 4, device=DEV)
    with pytest.raises(RuntimeError) as exc:
        with torch.no_grad():
            m(x, ei2, ea)
    msg = str(exc.value)
    assert f"num_edges: {ei.shape[1]}" in msg
    assert f"edge_index range: [0, {n - 1}]" in msg
    assert f"edge_attr shape: torch.Size([{ei.shape[1]}, 4])" in msg
