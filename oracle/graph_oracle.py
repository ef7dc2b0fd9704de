"""CPU oracle for the mesh -> graph step.  TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker of the native builder
(mignn.graph / csrc/graph_construct.hip), never by the product path.

A vectorised numpy restatement of the reference's GraphConstructor
(graph_constructor.py), pinned to the reference's own outputs on its OpenFOAM
case (tests/golden/mesh.npz, made by tests/golden/make_mesh_fixture.py):

  build_edge_index          graph_constructor.py:28-56
  compute_edge_attributes   graph_constructor.py:58-90
  build_graph               graph_constructor.py:92-269
  get_boundary_mask         graph_constructor.py:276-296
"""

from __future__ import annotations

import numpy as np


def build_edge_index(owner, neighbour):
    """Internal faces -> (o, n), (n, o) interleaved; boundary faces -> (o, o)."""
    owner = np.asarray(owner, dtype=np.int64)
    neighbour = np.asarray(neighbour, dtype=np.int64)
    ni = len(neighbour)
    pair = np.empty((2, 2 * ni), dtype=np.int64)
    pair[0, 0::2], pair[1, 0::2] = owner[:ni], neighbour
    pair[0, 1::2], pair[1, 1::2] = neighbour, owner[:ni]
    b = owner[ni:]
    return np.concatenate([pair, np.stack([b, b])], 1)


def compute_edge_attributes(edge_index, cell_centers):
    """(unit direction, distance) in float64 -- sum of squares in x, y, z
    order -- rounded to float32; zeros for self-loops and invalid indices."""
    ei = np.asarray(edge_index, dtype=np.int64)
    cc = np.asarray(cell_centers, dtype=np.float64)
    n = len(cc)
    s, d = ei
    ok = (s >= 0) & (s < n) & (d >= 0) & (d < n) & (s != d)
    out = np.zeros((ei.shape[1], 4), dtype=np.float32)
    dv = cc[d[ok]] - cc[s[ok]]
    dist = np.sqrt((dv[:, 0] * dv[:, 0] + dv[:, 1] * dv[:, 1]) + dv[:, 2] * dv[:, 2])
    unit = np.where(dist[:, None] > 0, dv / np.where(dist > 0, dist, 1.0)[:, None], dv)
    out[ok, :3] = unit.astype(np.float32)
    out[ok, 3] = dist.astype(np.float32)
    return out


def build_graph(mesh, field_data=None, node_features=None, filter_internal=False,
                n_internal_cells=None):
    """Returns (x float32, edge_index int64, edge_attr float32, n_nodes)."""
    owner = np.asarray(mesh["owner"], dtype=np.int64)
    neighbour = np.asarray(mesh["neighbour"], dtype=np.int64)
    cc = np.asarray(mesh["cell_centers"], dtype=np.float64)
    n_cells = int(mesh["n_cells"])
    mask = None
    if filter_internal:
        if n_internal_cells is not None:
            mask = np.zeros(n_cells, dtype=bool)
            mask[:n_internal_cells] = True
        elif "internal_mask" in mesh:
            mask = np.asarray(mesh["internal_mask"], dtype=bool)
    if mask is not None:
        keep_idx = np.nonzero(mask)[0]
        n_nodes = len(keep_idx)
        o2n = np.full(n_cells, -1, dtype=np.int64)
        o2n[keep_idx] = np.arange(n_nodes)
        ni = len(neighbour)
        a, b = o2n[owner[:ni]], o2n[neighbour]
        k = (a >= 0) & (b >= 0)
        a, b = a[k], b[k]
        ei = np.empty((2, 2 * len(a)), dtype=np.int64)
        ei[0, 0::2], ei[1, 0::2] = a, b
        ei[0, 1::2], ei[1, 1::2] = b, a
        centers = cc[keep_idx]
    else:
        keep_idx = np.arange(n_cells)
        n_nodes = n_cells
        ei = build_edge_index(owner, neighbour)
        centers = cc
    if ei.shape[1] > 0:
        ei = ei[:, (ei[0] < n_nodes) & (ei[1] < n_nodes)]
    if ei.shape[1] > 0 and n_nodes > 0:
        iso = np.setdiff1d(np.arange(n_nodes), np.unique(ei))
        ei = np.concatenate([ei, np.stack([iso, iso])], 1)
    elif n_nodes > 0:
        ei = np.stack([np.arange(n_nodes), np.arange(n_nodes)])
    ea = compute_edge_attributes(ei, centers)
    feats = cc if node_features is None else np.asarray(node_features, dtype=np.float64)
    x = feats[keep_idx]
    if field_data is not None:
        cols = [x]
        if "U" in field_data:
            cols.append(np.asarray(field_data["U"], dtype=np.float64))
        for name in ("p", "k", "epsilon", "nut"):
            if name in field_data:
                cols.append(np.asarray(field_data[name], dtype=np.float64).reshape(-1, 1))
        x = np.hstack(cols)
    return x.astype(np.float32), ei, ea, n_nodes


def get_boundary_mask(owner, n_cells, start_face, n_faces):
    owner = np.asarray(owner, dtype=np.int64)
    mask = np.zeros(n_cells, dtype=bool)
    f = np.arange(start_face, start_face + n_faces)
    f = f[(f >= 0) & (f < len(owner))]
    mask[owner[f]] = True
    return mask
