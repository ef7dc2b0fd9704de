"""Synthetic inputs for parity tests and the benchmark.

* `seeded_state_dict` re-draws every FlowGNN parameter from a seeded CPU
  generator, so a given (architecture, seed) pair yields bit-identical weights
  on any machine.
* `grid_graph` builds the 3-D periodic hex grid (6-neighbour, E = 6N, no
  self-loops) directly on the GPU with the native generator
  (`mignn_grid_graph`, csrc/graph_build.hip).  Node order is natural
  lexicographic (i fastest); an optional seeded permutation gives the
  locality stress case.
"""

from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch


def seeded_state_dict(template: Dict[str, torch.Tensor], seed: int = 0,
                      scale: str = "fan_in") -> Dict[str, torch.Tensor]:
    """Return a new state_dict with the same keys/shapes as `template`.

    scale="fan_in" (default): matrix weights ~ U(-a, a) with a = sqrt(6 / fan_in)
    (He-uniform, the scale of a trained ReLU network: activations and outputs
    stay O(1) through the layers, so an absolute error bound bites);
    attention vectors [1, heads, C] ~ U(-a, a) with a = sqrt(3 / C); biases
    ~ U(-0.1, 0.1); GIN's first Linear (`nn.0`, fed a sum over deg + 1 rows,
    not a mean) 1/8 of that, or deep GIN stacks grow without bound.  scale="uniform": every weight, bias and attention vector
    ~ U(-0.1, 0.1) (SURVEY.md §8d's original draw; near-constant outputs).
    Both: BatchNorm weight ~ U(0.5, 1.5), bias ~ U(-0.1, 0.1), running_mean
    ~ N(0, 0.1^2), running_var ~ U(0.5, 1.5); GIN `eps` and
    `num_batches_tracked` are kept.
    """
    if scale not in ("fan_in", "uniform"):
        raise ValueError(f"scale must be 'fan_in' or 'uniform', got {scale!r}")
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, t in template.items():
        shape, dtype = t.shape, t.dtype
        if k.endswith("num_batches_tracked") or k.endswith(".eps"):
            out[k] = t.detach().cpu().clone()
            continue
        if k.endswith("running_mean"):
            v = torch.randn(shape, generator=g) * 0.1
        elif k.endswith("running_var"):
            v = torch.rand(shape, generator=g) + 0.5
        elif ".module.weight" in k and k.startswith("batch_norms"):
            v = torch.rand(shape, generator=g) + 0.5
        else:
            u = torch.rand(shape, generator=g) * 2 - 1
            if scale == "fan_in" and len(shape) == 2:
                v = u * math.sqrt(6.0 / shape[1])
                if k.endswith(".nn.0.weight"):   # GIN: input is a SUM over deg+1 rows
                    v = v / 8.0
            elif scale == "fan_in" and len(shape) == 3:       # GAT att_src / att_dst
                v = u * math.sqrt(3.0 / shape[2])
            else:
                v = u * 0.1
        out[k] = v.to(dtype)
    return out


def state_dict_digest(sd: Dict[str, torch.Tensor]) -> str:
    """sha256 over a state_dict's keys and raw tensor bytes (sorted keys)."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def seeded_state_dict_from_layout(layout_json: str, seed: int, digest: Optional[str] = None,
                                  scale: str = "fan_in") -> Dict[str, torch.Tensor]:
    """seeded_state_dict on a stored state_dict layout ([[key, shape, dtype], ...]
    JSON, e.g. a reference model's), checked against `digest` when given."""
    import json
    template = {k: torch.zeros(shape, dtype=getattr(torch, dt))
                for k, shape, dt in json.loads(layout_json)}
    sd = seeded_state_dict(template, seed=seed, scale=scale)
    if digest is not None and state_dict_digest(sd) != digest:
        raise ValueError("regenerated state_dict does not match the stored digest")
    return sd


def grid_dims(num_nodes: int) -> Tuple[int, int, int]:
    """Named synthetic sizes."""
    named = {
        1_000_000: (100, 100, 100),
        10_000_000: (250, 200, 200),
        100_000_000: (500, 400, 500),
    }
    if num_nodes in named:
        return named[num_nodes]
    n = round(num_nodes ** (1.0 / 3.0))
    return (n, n, n)


def grid_graph(nx: int, ny: int, nz: int, device="cuda", permute_seed: Optional[int] = None,
               z_begin: int = 0, z_count: Optional[int] = None):
    """Periodic nx*ny*nz hex grid on `device` (native generator).

    Returns (x [N,3] f32 in [0,1]^3, edge_index [2, 6N] int64).  With
    `z_begin/z_count` only the k-slab [z_begin, z_begin+z_count) is emitted
    with global node ids (used by the sharded path).  `permute_seed`
    relabels nodes with a seeded random permutation (locality stress case).
    """
    from . import _lib

    nzc = nz if z_count is None else z_count
    n = nx * ny * nzc
    x = torch.empty((n, 3), dtype=torch.float32, device=device)
    ei = torch.empty((2, 6 * n), dtype=torch.int64, device=device)
    _lib.check(_lib.lib().mignn_grid_graph(nx, ny, nz, z_begin, nzc, _lib.ptr(ei), _lib.ptr(x),
                                           _lib.stream()), "mignn_grid_graph")
    if permute_seed is not None:
        assert z_count is None, "permutation is defined on the full grid only"
        g = torch.Generator().manual_seed(permute_seed)
        perm = torch.randperm(n, generator=g).to(device)      # old id -> new id
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(n, device=device)
        x = x[inv]
        ei = perm[ei]
    return x, ei


def hex_polymesh(nx: int, ny: int, nz: int, device="cuda"):
    """OpenFOAM-ordered polyMesh connectivity of a non-periodic nx*ny*nz hex
    block (blockMesh cell order, i fastest): internal faces sorted by owner,
    then neighbour (c+1, c+nx, c+nx*ny), followed by the boundary faces
    (-x, +x, -y, +y, -z, +z patches); cell centres on the unit cube.
    Returns a dict shaped like OpenFOAMLoader.load_mesh() (input synthesis for
    the graph-builder benchmark / tests)."""
    n = nx * ny * nz
    c = torch.arange(n, device=device, dtype=torch.int64)
    i, j, k = c % nx, (c // nx) % ny, c // (nx * ny)
    nb = torch.stack([torch.where(i < nx - 1, c + 1, -1), torch.where(j < ny - 1, c + nx, -1),
                      torch.where(k < nz - 1, c + nx * ny, -1)], 1).reshape(-1)
    own = c.repeat_interleave(3)
    keep = nb >= 0
    owner_int, neigh = own[keep], nb[keep]
    bnd = [c[i == 0], c[i == nx - 1], c[j == 0], c[j == ny - 1], c[k == 0], c[k == nz - 1]]
    names = ["xmin", "xmax", "ymin", "ymax", "zmin", "zmax"]
    starts, o = [], int(owner_int.numel())
    for b in bnd:
        starts.append(o)
        o += int(b.numel())
    owner = torch.cat([owner_int] + bnd)
    cc = torch.stack([(i + 0.5) / nx, (j + 0.5) / ny, (k + 0.5) / nz], 1).double()
    return {"owner": owner, "neighbour": neigh, "cell_centers": cc, "n_cells": n,
            "internal_mask": torch.ones(n, dtype=torch.bool, device=device),
            "boundaries": {nm: {"startFace": st, "nFaces": int(b.numel())}
                           for nm, st, b in zip(names, starts, bnd)}}
