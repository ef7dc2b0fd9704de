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


def model_fixture(name):
    m = npz("models.npz")
    cfg = json.loads(str(m[f"{name}/cfg"]))
    pre = f"{name}/sd/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in m.items() if k.startswith(pre)}
    outs = {}
    for gname in ("train", "infer"):
        if f"{name}/{gname}/y32" in m:
            outs[gname] = (torch.from_numpy(m[f"{name}/{gname}/y32"]),
                           torch.from_numpy(m[f"{name}/{gname}/y64"]))
    err = str(m[f"{name}/edge_attr_error"]) if f"{name}/edge_attr_error" in m else None
    return cfg, sd, outs, err


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
