"""Test-side helpers: fixture loading and small independent restatements."""

import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache = {}


def npz(name):
    if name not in _cache:
        _cache[name] = dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
    return _cache[name]


def bfs_graph(which="train"):
    g = npz("bfs_graphs.npz")
    x = torch.from_numpy(g[f"{which}_x"])
    ei = torch.from_numpy(g[f"{which}_ei"].astype(np.int64))
    ea = torch.from_numpy(g[f"{which}_ea"])
    return x, ei, ea


def model_names():
    m = npz("models.npz")
    return sorted({k.split("/")[0] for k in m})


def _fixture_sd(m, name):
    """The fixture's weights, regenerated from the stored seed
    (mignn.synthetic.seeded_state_dict) on the REFERENCE model's stored
    state_dict layout (keys, order, shapes, dtypes) and checked bit for bit
    against the stored digest."""
    from mignn.synthetic import seeded_state_dict_from_layout
    return seeded_state_dict_from_layout(str(m[f"{name}/sd_layout"]), int(m[f"{name}/seed"]),
                                         str(m[f"{name}/sd_sha256"]))


def model_fixture(name):
    m = npz("models.npz")
    cfg = json.loads(str(m[f"{name}/cfg"]))
    sd = _fixture_sd(m, name)
    outs = {}
    for gname in ("train", "infer"):
        if f"{name}/{gname}/y32" in m:
            outs[gname] = (torch.from_numpy(m[f"{name}/{gname}/y32"]),
                           torch.from_numpy(m[f"{name}/{gname}/y64"]))
    err = str(m[f"{name}/edge_attr_error"]) if f"{name}/edge_attr_error" in m else None
    return cfg, sd, outs, err


def ref_err(name, gname, which="models.npz"):
    """The reference fp32 CPU forward's own max-abs error vs fp64 on that
    fixture (the accuracy floor a faithful fp32 implementation sits at)."""
    return float(npz(which)[f"{name}/{gname}/ref_err"])


def parity_tol(name, gname, which="models.npz"):
    """Max-abs bound vs the fp64 oracle: the north star's 1e-5, or twice the
    reference fp32 CPU forward's own error where that alone exceeds half of
    it (deep configs whose outputs reach O(10): fp32 ulp ~1e-6 there)."""
    return max(1e-5, 2.0 * ref_err(name, gname, which))


def surrogate_names():
    return sorted({k.split("/")[0] for k in npz("surrogate.npz")})


def surrogate_fixture(name):
    m = npz("surrogate.npz")
    cfg = json.loads(str(m[f"{name}/cfg"]))
    sd = _fixture_sd(m, name)
    outs = {tag: (torch.from_numpy(m[f"{name}/{tag}/y32"]), torch.from_numpy(m[f"{name}/{tag}/y64"]))
            for tag in ("nobc", "bc")}
    n = outs["bc"][0].shape[0]
    bc = torch.rand((n, cfg["hidden_dim"]),
                    generator=torch.Generator().manual_seed(int(m[f"{name}/bc_seed"]))) * 2 - 1
    return cfg, sd, bc, outs


def tiny_names():
    t = npz("tiny_graphs.npz")
    return sorted({k.split("/")[0] for k in t})


def tiny_fixture(name, layer_type):
    t = npz("tiny_graphs.npz")
    x = torch.from_numpy(t[f"{name}/x"])
    ei = torch.from_numpy(t[f"{name}/ei"].astype(np.int64)).reshape(2, -1)
    pre = f"{name}/{layer_type}/sd/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in t.items() if k.startswith(pre)}
    return x, ei, sd, torch.from_numpy(t[f"{name}/{layer_type}/y32"]), \
        torch.from_numpy(t[f"{name}/{layer_type}/y64"])


def grid_graph_np(nx, ny, nz, z_begin=0, z_count=None):
    """numpy restatement of mignn_grid_graph (csrc/graph_build.hip)."""
    zc = nz if z_count is None else z_count
    k, j, i = np.meshgrid(np.arange(z_begin, z_begin + zc), np.arange(ny), np.arange(nx),
                          indexing="ij")
    i, j, k = i.ravel(), j.ravel(), k.ravel()
    gid = (k * ny + j) * nx + i
    nb = np.stack([
        (k * ny + j) * nx + (i - 1) % nx, (k * ny + j) * nx + (i + 1) % nx,
        (k * ny + (j - 1) % ny) * nx + i, (k * ny + (j + 1) % ny) * nx + i,
        (((k - 1) % nz) * ny + j) * nx + i, (((k + 1) % nz) * ny + j) * nx + i], 1)
    src = nb.reshape(-1)
    dst = np.repeat(gid, 6)
    x = np.stack([(i + 0.5) / nx, (j + 0.5) / ny, (k + 0.5) / nz], 1).astype(np.float32)
    return x, np.stack([src, dst]).astype(np.int64)


def csr_np(ei, n, one_self_loop):
    """Independent restatement of the CSR contract of mignn_csr_build."""
    src, dst = ei[0], ei[1]
    valid = (src >= 0) & (src < n) & (dst >= 0) & (dst < n)
    keep = valid & ~((src == dst) if one_self_loop else np.zeros_like(valid))
    rows = [[] for _ in range(n)]
    for s, d, kp in zip(src, dst, keep):
        if kp:
            rows[d].append(int(s))
    if one_self_loop:
        for i in range(n):
            rows[i].append(i)
    elif ei.shape[1] > 0 and not keep.any():
        rows = [[i] for i in range(n)]
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.array([c for r in rows for c in r], np.int64)
    return row_ptr, col


def khop_subgraph(edge_index, num_nodes, seeds, hops):
    """Receptive field of `seeds` for an L-layer FlowGNN (hops = L): nodes at
    in-distance <= L + 1 and every in-edge of the nodes at distance <= L.
    Any L-layer forward on the subgraph gives the seeds exactly the outputs of
    the forward on the whole graph -- GCN degrees (deg^-1/2 of sources at
    distance L), GAT / Transformer softmax rows and GIN sums are all complete
    there (test infrastructure: checks a GPU forward at full size against the
    CPU oracle on a bounded sample).  Works on any device; returns
    (node ids [M] (seeds first), relabelled edge_index [2, E'] int64)."""
    dev = edge_index.device
    src, dst = edge_index[0], edge_index[1]
    valid = (src >= 0) & (src < num_nodes) & (dst >= 0) & (dst < num_nodes)
    src, dst = src[valid], dst[valid]
    dist = torch.full((num_nodes,), hops + 2, dtype=torch.int32, device=dev)
    dist[seeds] = 0
    for d in range(1, hops + 2):
        frontier = dist[dst] == d - 1
        nb = src[frontier]
        dist[nb] = torch.minimum(dist[nb], torch.full_like(dist[nb], d))
    seeds = seeds.to(dev)
    others = torch.nonzero(dist <= hops + 1).flatten()
    others = others[dist[others] > 0]
    nodes = torch.cat([seeds, others[~torch.isin(others, seeds)]])
    keep = dist[dst] <= hops
    new = torch.full((num_nodes,), -1, dtype=torch.int64, device=dev)
    new[nodes] = torch.arange(nodes.numel(), device=dev)
    sub = torch.stack([new[src[keep]], new[dst[keep]]])
    assert bool((sub >= 0).all())
    return nodes, sub
