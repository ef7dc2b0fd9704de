"""The receptive-field sampler used by the full-size GPU parity tests
(helpers.khop_subgraph) is exact: an L-layer oracle forward on the subgraph
reproduces the whole-graph forward at the seeds, for every layer type,
including duplicate self-loops, isolated nodes and invalid edges."""

import pytest
import torch

from helpers import khop_subgraph
from mignn.synthetic import seeded_state_dict
from oracle import flowgnn_oracle as orc

torch.set_num_threads(min(8, torch.get_num_threads()))


def _random_mesh(n, seed):
    g = torch.Generator().manual_seed(seed)
    # a 3-D grid-like graph with extra random edges, self-loops, an isolated node
    side = round(n ** (1 / 3))
    ids = torch.arange(side ** 3)
    i, j, k = ids % side, (ids // side) % side, ids // (side * side)
    nb = torch.stack([((i + 1) % side) + j * side + k * side * side,
                      i + ((j + 1) % side) * side + k * side * side,
                      i + j * side + ((k + 1) % side) * side * side], 1)
    src = torch.cat([ids.repeat_interleave(3), nb.reshape(-1)])
    dst = torch.cat([nb.reshape(-1), ids.repeat_interleave(3)])
    extra = torch.randint(0, side ** 3, (2, side ** 3 // 4), generator=g)
    loops = torch.randint(0, side ** 3, (side ** 3 // 10,), generator=g)
    ei = torch.cat([torch.stack([src, dst]), extra, torch.stack([loops, loops]),
                    torch.tensor([[0, side ** 3 + 3], [side ** 3 + 5, 1]])], 1)
    x = torch.rand((side ** 3 + 1, 3), generator=g)       # last node isolated
    return x, ei


@pytest.mark.parametrize("lt", ["GCN", "GAT", "GIN", "Transformer"])
@pytest.mark.parametrize("L", [1, 3])
def test_khop_subgraph_is_exact(lt, L):
    x, ei = _random_mesh(1000, L)
    n = x.shape[0]
    cfg = dict(hidden_dim=16, num_layers=L, layer_type=lt)
    from mignn.gnn_model import FlowGNN
    sd = seeded_state_dict(FlowGNN(input_dim=3, output_dim=7, **cfg).state_dict(), seed=3)
    full = orc.flowgnn_forward(sd, cfg, x, ei, None, dtype=torch.float64)
    seeds = torch.tensor([0, 5, 17, n - 1, 333])
    nodes, sub = khop_subgraph(ei, n, seeds, L)
    assert nodes.numel() < n            # a real restriction, not the whole graph
    part = orc.flowgnn_forward(sd, cfg, x[nodes], sub, None, dtype=torch.float64)
    assert torch.allclose(part[:seeds.numel()], full[seeds], rtol=0, atol=1e-12)
