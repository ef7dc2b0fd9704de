"""
TEST INFRASTRUCTURE ONLY -- CPU oracle for the FlowGNN forward hot path.

This module is the *checker*, never the product.  Only `tests/`,
`__graft_entry__.smoke()` (as the checker of a GPU result) and the
`cpu_baseline` leg of `bench.py` may import it.  The MI355X product path lives
in `gnn-bfs-rans_amd/` and fails loudly when its HIP library is missing.

What it restates
----------------
* The reference wrapper `FlowGNN.forward` (gnn_model.py:104-197): edge
  validation / silent filtering (:125-156), `input_proj` (:159), the layer loop
  `x = relu(BN(x + conv(x)))` (:162-192), `output_proj` (:195).
* The third-party conv arithmetic the wrapper calls.  `torch_geometric` is
  **not vendored** in /root/reference and not installed here; the reference pins
  it only as `torch-geometric>=2.3.0` (requirements.txt:2).  The semantics below
  restate PyG >= 2.3's published algorithms:
    - GCNConv  (gnn_model.py:63, :166): `gcn_norm` = add_remaining_self_loops
      (drop every self-loop, append exactly one per node, weight 1),
      deg = scatter_add(w, dst), w_ji = deg_j^-1/2 * deg_i^-1/2;
      h = x W^T; out_i = sum_j w_ji h_j; + bias.
    - GATConv(heads=4, concat=False) (gnn_model.py:65-68, :168):
      remove_self_loops + add_self_loops; e_ji = LeakyReLU_0.2(a_src[j] + a_dst[i]);
      per-destination softmax (x - max, exp, / (sum + 1e-16)); mean over heads; + bias.
    - GINConv(eps=0, train_eps=False) (gnn_model.py:70-75, :166):
      nn(sum_{j->i} x_j + (1 + eps) x_i) over edge_index *as given*.
    - TransformerConv(heads=4, concat=False, beta=False, edge_dim=None)
      (gnn_model.py:77-80, :170): q,k,v = lin(x); alpha = softmax_dst(q_i.k_j/sqrt(C));
      out = mean_h sum_j alpha v_j + lin_skip(x).  PyG's `message` adds a
      non-None `edge_attr` to `value_j` even without `lin_edge`; with the
      reference's [E,4] edge_attr that is a broadcast error, which the wrapper
      re-raises as "Message passing failed in layer i (Transformer)".
    - BatchNorm (gnn_model.py:87, :188): `BatchNorm1d(eps=1e-5)`, eval mode.

Parity status
-------------
* Wrapper logic and graph construction: pinned by running the reference's own
  `gnn_model.FlowGNN` / `graph_constructor` / `openfoam_loader` code with these
  classes injected as `torch_geometric.nn` (tests/golden/make_golden.py).
* Conv arithmetic: **parity unpinned by the reference** (PyG absent, no
  reference golden vectors exist for it).  Pinned here only
  by hand-checkable small-graph tests (tests/test_oracle.py).
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

SOFTMAX_EPS = 1e-16  # PyG utils.softmax denominator guard


# --------------------------------------------------------------------------
# PyG utility restatements
# --------------------------------------------------------------------------

def remove_self_loops(edge_index: torch.Tensor) -> torch.Tensor:
    """PyG utils.remove_self_loops (edge_attr-free form)."""
    mask = edge_index[0] != edge_index[1]
    return edge_index[:, mask]


def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG utils.add_self_loops: append (i, i) for every node."""
    loop = torch.arange(num_nodes, dtype=edge_index.dtype).unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1)


def add_remaining_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG utils.add_remaining_self_loops with edge_weight=None: every existing
    self-loop is dropped and exactly one (i, i) per node is appended."""
    return add_self_loops(remove_self_loops(edge_index), num_nodes)


def gcn_norm(edge_index: torch.Tensor, num_nodes: int, dtype: torch.dtype):
    """PyG nn.conv.gcn_conv.gcn_norm (add_self_loops=True, improved=False,
    flow='source_to_target')."""
    ei = add_remaining_self_loops(edge_index, num_nodes)
    w = torch.ones(ei.shape[1], dtype=dtype)
    row, col = ei[0], ei[1]
    deg = torch.zeros(num_nodes, dtype=dtype).scatter_add_(0, col, w)
    dinv = deg.pow(-0.5)
    dinv.masked_fill_(dinv == float("inf"), 0.0)
    w = dinv[row] * w * dinv[col]
    return ei, w, dinv


def segment_softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG utils.softmax(src, index): x - max, exp, / (sum + 1e-16), per index."""
    shape = (num_nodes,) + tuple(src.shape[1:])
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    src_max = torch.full(shape, float("-inf"), dtype=src.dtype).scatter_reduce(
        0, idx, src.detach(), reduce="amax", include_self=True)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = torch.zeros(shape, dtype=src.dtype).index_add_(0, index, out) + SOFTMAX_EPS
    return out / out_sum.index_select(0, index)


def scatter_add_rows(msg: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    out = torch.zeros((num_nodes,) + tuple(msg.shape[1:]), dtype=msg.dtype)
    return out.index_add_(0, index, msg)


# --------------------------------------------------------------------------
# Functional conv restatements (all CPU, any float dtype)
# --------------------------------------------------------------------------

def gcn_conv(x, edge_index, weight, bias):
    N = x.shape[0]
    h = x @ weight.t()
    ei, w, _ = gcn_norm(edge_index, N, x.dtype)
    msg = h.index_select(0, ei[0]) * w.view(-1, 1)
    return scatter_add_rows(msg, ei[1], N) + bias


def gat_conv(x, edge_index, weight, att_src, att_dst, bias, heads=4, negative_slope=0.2):
    N = x.shape[0]
    C = weight.shape[0] // heads
    h = (x @ weight.t()).view(N, heads, C)
    a_s = (h * att_src).sum(-1)
    a_d = (h * att_dst).sum(-1)
    ei = add_self_loops(remove_self_loops(edge_index), N)
    alpha = a_s.index_select(0, ei[0]) + a_d.index_select(0, ei[1])
    alpha = F.leaky_relu(alpha, negative_slope)
    alpha = segment_softmax(alpha, ei[1], N)
    msg = h.index_select(0, ei[0]) * alpha.unsqueeze(-1)
    out = scatter_add_rows(msg, ei[1], N)
    return out.mean(dim=1) + bias


def gin_conv(x, edge_index, eps, w1, b1, w2, b2):
    N = x.shape[0]
    out = scatter_add_rows(x.index_select(0, edge_index[0]), edge_index[1], N)
    out = out + (1 + eps) * x
    h = torch.relu(out @ w1.t() + b1)
    return h @ w2.t() + b2


def transformer_conv(x, edge_index, wq, bq, wk, bk, wv, bv, wskip, bskip,
                     heads=4, edge_attr=None):
    N = x.shape[0]
    C = wq.shape[0] // heads
    q = (x @ wq.t() + bq).view(N, heads, C)
    k = (x @ wk.t() + bk).view(N, heads, C)
    v = (x @ wv.t() + bv).view(N, heads, C)
    src, dst = edge_index[0], edge_index[1]
    alpha = (q.index_select(0, dst) * k.index_select(0, src)).sum(-1) / math.sqrt(C)
    alpha = segment_softmax(alpha, dst, N)
    out = v.index_select(0, src)
    if edge_attr is not None:
        # PyG TransformerConv.message: `out = out + edge_attr` whenever edge_attr
        # is not None, even with lin_edge=None -> [E,heads,C] + [E,4] broadcast.
        out = out + edge_attr
    out = out * alpha.view(-1, heads, 1)
    out = scatter_add_rows(out, dst, N).mean(dim=1)
    return out + (x @ wskip.t() + bskip)


def batch_norm_eval(x, weight, bias, running_mean, running_var, eps=1e-5):
    return F.batch_norm(x, running_mean, running_var, weight, bias, False, 0.0, eps)


# --------------------------------------------------------------------------
# PyG-named module classes.  Injected as `torch_geometric.nn` to run the
# reference's own gnn_model.FlowGNN (tests/golden/make_golden.py); their
# parameter names reproduce PyG's state_dict layout.
# --------------------------------------------------------------------------

class GCNConv(nn.Module):
    def __init__(self, in_channels, out_channels, **kw):
        super().__init__()
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def forward(self, x, edge_index, edge_weight=None):
        return gcn_conv(x, edge_index, self.lin.weight, self.bias)


class GATConv(nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, dropout=0.0,
                 negative_slope=0.2, **kw):
        super().__init__()
        assert not concat, "FlowGNN uses concat=False (gnn_model.py:67)"
        self.heads, self.out_channels = heads, out_channels
        self.negative_slope, self.dropout = negative_slope, dropout
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.zeros(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.zeros(1, heads, out_channels))
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def forward(self, x, edge_index, edge_attr=None):
        if self.training and self.dropout > 0:
            raise NotImplementedError("oracle covers eval mode only")
        return gat_conv(x, edge_index, self.lin.weight, self.att_src, self.att_dst,
                        self.bias, self.heads, self.negative_slope)


class GINConv(nn.Module):
    def __init__(self, nn_module, eps=0.0, train_eps=False, **kw):
        super().__init__()
        self.nn = nn_module
        self.register_buffer("eps", torch.tensor([float(eps)]))

    def forward(self, x, edge_index):
        N = x.shape[0]
        out = scatter_add_rows(x.index_select(0, edge_index[0]), edge_index[1], N)
        out = out + (1 + self.eps) * x
        return self.nn(out)


class TransformerConv(nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, beta=False,
                 dropout=0.0, edge_dim=None, bias=True, root_weight=True, **kw):
        super().__init__()
        assert not concat and not beta and edge_dim is None and root_weight
        self.heads, self.out_channels, self.dropout = heads, out_channels, dropout
        self.lin_key = nn.Linear(in_channels, heads * out_channels)
        self.lin_query = nn.Linear(in_channels, heads * out_channels)
        self.lin_value = nn.Linear(in_channels, heads * out_channels)
        self.lin_skip = nn.Linear(in_channels, out_channels, bias=bias)

    def forward(self, x, edge_index, edge_attr=None):
        if self.training and self.dropout > 0:
            raise NotImplementedError("oracle covers eval mode only")
        return transformer_conv(
            x, edge_index, self.lin_query.weight, self.lin_query.bias,
            self.lin_key.weight, self.lin_key.bias, self.lin_value.weight,
            self.lin_value.bias, self.lin_skip.weight, self.lin_skip.bias,
            self.heads, edge_attr)


class BatchNorm(nn.Module):
    """PyG nn.norm.BatchNorm: wraps BatchNorm1d as `.module`."""

    def __init__(self, in_channels, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, **kw):
        super().__init__()
        self.module = nn.BatchNorm1d(in_channels, eps, momentum, affine, track_running_stats)

    def forward(self, x):
        return self.module(x)


class MessagePassing(nn.Module):  # imported (unused) by gnn_model.py:8
    pass


def global_mean_pool(x, batch):  # imported (unused) by gnn_model.py:8
    raise NotImplementedError


# --------------------------------------------------------------------------
# Functional FlowGNN forward (restates gnn_model.py:104-197, eval mode)
# --------------------------------------------------------------------------

def _p(sd: Dict[str, torch.Tensor], key: str, dtype) -> torch.Tensor:
    return sd[key].detach().to("cpu", dtype)


def gat_weight(sd, prefix):
    """Accept PyG 2.5+ (`lin.weight`) and 2.3/2.4 (`lin_src.weight`) layouts."""
    for k in (prefix + "lin.weight", prefix + "lin_src.weight"):
        if k in sd:
            return k
    raise KeyError(prefix + "lin.weight")


def flowgnn_forward(sd: Dict[str, torch.Tensor], cfg: Dict, x, edge_index,
                    edge_attr=None, dtype=torch.float32) -> torch.Tensor:
    """CPU restatement of FlowGNN.forward in eval mode.

    `cfg` = {hidden_dim, num_layers, layer_type, use_batch_norm}.
    """
    layer_type = cfg["layer_type"]
    L = cfg["num_layers"]
    use_bn = cfg.get("use_batch_norm", True)
    x = x.detach().to("cpu", dtype)
    edge_index = edge_index.detach().to("cpu", torch.long)
    if edge_attr is not None:
        edge_attr = edge_attr.detach().to("cpu", dtype)
    N = x.shape[0]
    # gnn_model.py:126-127
    if edge_index.shape[0] != 2:
        raise ValueError(f"edge_index must have shape [2, num_edges], got {edge_index.shape}")
    # gnn_model.py:130-149
    if edge_index.shape[1] > 0:
        if edge_index.min().item() < 0 or edge_index.max().item() >= N:
            valid = ((edge_index[0] >= 0) & (edge_index[0] < N) &
                     (edge_index[1] >= 0) & (edge_index[1] < N))
            edge_index = edge_index[:, valid]
            if edge_attr is not None and edge_attr.shape[0] > 0:
                edge_attr = edge_attr[valid]
        if edge_index.shape[1] == 0:
            edge_index = torch.arange(N, dtype=torch.long).repeat(2, 1)
            if edge_attr is not None:
                edge_attr = torch.zeros((N, edge_attr.shape[1]), dtype=dtype)
    # gnn_model.py:152-156
    if edge_attr is not None and edge_index.shape[1] > 0:
        if edge_attr.shape[0] != edge_index.shape[1]:
            raise ValueError(
                f"edge_attr must have {edge_index.shape[1]} entries, got {edge_attr.shape[0]}")
    P = lambda k: _p(sd, k, dtype)  # noqa: E731
    x = x @ P("input_proj.weight").t() + P("input_proj.bias")
    for i in range(L):
        pre = f"gnn_layers.{i}."
        try:
            if layer_type == "GCN":
                xn = gcn_conv(x, edge_index, P(pre + "lin.weight"), P(pre + "bias"))
            elif layer_type == "GAT":
                xn = gat_conv(x, edge_index, P(gat_weight(sd, pre)), P(pre + "att_src"),
                              P(pre + "att_dst"), P(pre + "bias"))
            elif layer_type == "GIN":
                eps = float(sd[pre + "eps"].reshape(-1)[0]) if pre + "eps" in sd else 0.0
                xn = gin_conv(x, edge_index, eps, P(pre + "nn.0.weight"), P(pre + "nn.0.bias"),
                              P(pre + "nn.2.weight"), P(pre + "nn.2.bias"))
            elif layer_type == "Transformer":
                xn = transformer_conv(
                    x, edge_index, P(pre + "lin_query.weight"), P(pre + "lin_query.bias"),
                    P(pre + "lin_key.weight"), P(pre + "lin_key.bias"),
                    P(pre + "lin_value.weight"), P(pre + "lin_value.bias"),
                    P(pre + "lin_skip.weight"), P(pre + "lin_skip.bias"),
                    heads=4, edge_attr=edge_attr)
            else:
                raise ValueError(f"Unknown layer type: {layer_type}")
        except RuntimeError as e:  # gnn_model.py:173-181
            raise RuntimeError(
                f"Message passing failed in layer {i} ({layer_type}): {str(e)}") from e
        x = x + xn
        if use_bn:
            bp = f"batch_norms.{i}.module."
            x = batch_norm_eval(x, P(bp + "weight"), P(bp + "bias"),
                                P(bp + "running_mean"), P(bp + "running_var"))
        x = torch.relu(x)
    h = torch.relu(x @ P("output_proj.0.weight").t() + P("output_proj.0.bias"))
    h = torch.relu(h @ P("output_proj.3.weight").t() + P("output_proj.3.bias"))
    h = torch.relu(h @ P("output_proj.6.weight").t() + P("output_proj.6.bias"))
    return h @ P("output_proj.8.weight").t() + P("output_proj.8.bias")
