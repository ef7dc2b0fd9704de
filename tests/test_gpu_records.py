"""GCN layer 1 from layer-0 records (mignn_gcn_layer0_records +
mignn_gcn_layer_f16x3_rec) against the materialised path (layer-0 rows
written by mignn_gcn_layer0_coords, layer 1 by mignn_gcn_layer_f16x3).

The records kernel expands every x row with the layer-0 kernel's own fma
order and sums in the same order, so the two paths must agree BIT FOR BIT --
on the mesh in the locality order (in-tile + out-of-tile register slots), in
a shuffled order (many out-of-tile entries: the beyond-slot loop) and with hub
rows (the row-at-a-time slow path).  Arithmetic against the fp64 oracle is
covered by the model-level parity tests, which take this path by default."""

import pytest
import torch

from mignn import FlowGNN
from mignn.synthetic import grid_graph, seeded_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from mignn import _lib
    _lib.lib()


def _model(H, L, seed=3, bn=True):
    m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=H, num_layers=L, layer_type="GCN",
                use_batch_norm=bn)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=seed))
    return m.to(DEV).eval()


def _both(m, x, ei, monkeypatch):
    with torch.no_grad():
        monkeypatch.setenv("MIGNN_REC", "0")
        y0 = m(x, ei)
        monkeypatch.setenv("MIGNN_REC", "1")
        assert m._records_layer1()
        y1 = m(x, ei)
    return y0, y1


def _hub_graph(n, hubs, fan, seed):
    """A 3-D grid plus `hubs` nodes receiving `fan` random edges each."""
    x, ei = grid_graph(20, 16, n // 320, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(seed)
    N = x.shape[0]
    dst = torch.randint(0, N, (hubs,), device=DEV, generator=g).repeat_interleave(fan)
    src = torch.randint(0, N, (hubs * fan,), device=DEV, generator=g)
    return x, torch.cat([ei, torch.stack([src, dst])], 1)


@pytest.mark.parametrize("H", [64, 128])
@pytest.mark.parametrize("order", ["locality", "shuffled", "natural"])
def test_records_layer1_bitwise(H, order, monkeypatch):
    m = _model(H, 3)
    x, ei = grid_graph(40, 36, 30, device=DEV, permute_seed=7 if order == "shuffled" else None)
    if order == "natural":
        m.reorder = "0"
    y0, y1 = _both(m, x, ei, monkeypatch)
    assert torch.isfinite(y1).all()
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("H", [64, 128])
def test_records_layer1_hub_rows_bitwise(H, monkeypatch):
    """Rows of 100+ entries (the kernel's row-at-a-time slow path) and many
    out-of-tile entries per row."""
    m = _model(H, 2, seed=5)
    x, ei = _hub_graph(320 * 12, hubs=9, fan=150, seed=1)
    y0, y1 = _both(m, x, ei, monkeypatch)
    assert torch.equal(y0, y1)


def test_records_layer1_no_batchnorm_ragged(monkeypatch):
    """No BN (epilogue without the affine), a node count that is not a
    multiple of the 64-row tile."""
    m = _model(128, 4, seed=11, bn=False)
    x, ei = grid_graph(13, 11, 7, device=DEV, permute_seed=3)
    y0, y1 = _both(m, x, ei, monkeypatch)
    assert torch.equal(y0, y1)
