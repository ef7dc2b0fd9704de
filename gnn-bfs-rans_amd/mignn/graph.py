"""Mesh -> graph on the device: the reference's
`GraphConstructor` (graph_constructor.py) with the same methods, arguments,
edge order and rules, computed by the native kernels of
csrc/graph_construct.hip instead of per-edge Python loops.

    gc = GraphConstructor(mesh_data)          # OpenFOAMLoader.load_mesh() dict
    data = gc.build_graph(node_features=mesh_data["cell_centers"],
                          filter_internal=True, n_internal_cells=n)

Results equal the reference's bit for bit (edge_index, float32 edge_attr from
float64 arithmetic, float32 x); tests/test_gpu_graph.py checks them against
the reference's own outputs on its OpenFOAM case (tests/golden/mesh.npz).
One host read per graph: the edge count, to size the outputs (the reference
syncs with `.item()` per edge).
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .data import Data

MESH_ALL, MESH_FIRST_N, MESH_MASK = 0, 1, 2


def _dev_tensor(a, dtype, device):
    if torch.is_tensor(a):
        return a.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(a), dtype=dtype, device=device).contiguous()


class GraphConstructor:
    """graph_constructor.py:11-296 on the device."""

    def __init__(self, mesh_data: Dict, device="cuda"):
        self.mesh_data = mesh_data
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("mignn GraphConstructor runs on ROCm devices only (no CPU path)")
        self.owner = _dev_tensor(mesh_data["owner"], torch.int64, self.device)
        self.neighbour = _dev_tensor(mesh_data["neighbour"], torch.int64, self.device)
        self.cell_centers = _dev_tensor(mesh_data["cell_centers"], torch.float64, self.device)
        self.n_cells = int(mesh_data["n_cells"])
        if self.cell_centers.shape != (self.n_cells, 3):
            raise ValueError(f"cell_centers must be [n_cells, 3], got {tuple(self.cell_centers.shape)}")

    # ------------------------------------------------------------------ core
    def _build(self, mode: int, mask=None, n_first: int = 0, isolated: bool = True,
               features: Optional[torch.Tensor] = None):
        L, P = _lib.lib(), _lib.ptr
        st = _lib.stream(self.device)
        n_faces, n_int = self.owner.numel(), self.neighbour.numel()
        nbytes = L.mignn_mesh_graph_scratch_bytes(n_faces, self.n_cells)
        if nbytes == 0:
            raise _lib.MignnError("mesh graph scratch query failed: " + _lib.last_error())
        scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        counts = torch.zeros(4, dtype=torch.int64, device=self.device)
        m = None if mask is None else _dev_tensor(mask, torch.uint8, self.device)
        _lib.check(L.mignn_mesh_graph_count(P(self.owner), n_faces, P(self.neighbour), n_int,
                                            self.n_cells, mode, P(m), n_first, int(isolated),
                                            P(counts), P(scratch), nbytes, st),
                   "mignn_mesh_graph_count")
        n_nodes, _, _, E = (int(v) for v in counts.cpu())   # the one host read: sizes
        ei = torch.empty((2, E), dtype=torch.int64, device=self.device)
        ea = torch.empty((E, 4), dtype=torch.float32, device=self.device)
        x = None
        fd = 0
        if features is not None:
            fd = int(features.shape[1])
            x = torch.empty((n_nodes, fd), dtype=torch.float32, device=self.device)
        _lib.check(L.mignn_mesh_graph_emit(P(self.owner), n_faces, P(self.neighbour), n_int,
                                           self.n_cells, mode, P(self.cell_centers), P(features),
                                           fd, E, P(ei), P(ea), P(x), max(fd, 1), P(scratch),
                                           nbytes, st), "mignn_mesh_graph_emit")
        return ei, ea, x, n_nodes

    # ------------------------------------------------------------------ API
    def build_edge_index(self) -> torch.Tensor:
        """graph_constructor.py:28-56: internal faces both ways, boundary
        faces as self-loops, face order."""
        ei, _, _, _ = self._build(MESH_ALL, isolated=False)
        return ei

    def compute_edge_attributes(self, edge_index: torch.Tensor) -> torch.Tensor:
        """graph_constructor.py:58-90: (unit direction, distance), float64
        arithmetic rounded to float32; zeros for self-loops."""
        ei = _dev_tensor(edge_index, torch.int64, self.device)
        E = int(ei.shape[1])
        ea = torch.empty((E, 4), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().mignn_edge_attributes(_lib.ptr(ei), E, self.n_cells,
                                                    _lib.ptr(self.cell_centers), _lib.ptr(ea),
                                                    _lib.stream(self.device)),
                   "mignn_edge_attributes")
        return ea

    def build_graph(self, field_data: Optional[Dict] = None,
                    node_features: Optional[np.ndarray] = None,
                    filter_internal: bool = False,
                    n_internal_cells: Optional[int] = None) -> Data:
        """graph_constructor.py:92-269 (same branches and fallbacks)."""
        mode, mask, n_first = MESH_ALL, None, 0
        if filter_internal:
            if n_internal_cells is not None:
                mode, n_first = MESH_FIRST_N, int(n_internal_cells)
                if n_first > self.n_cells:
                    raise IndexError(f"n_internal_cells {n_first} > n_cells {self.n_cells}")
            elif "internal_mask" in self.mesh_data:
                mode, mask = MESH_MASK, self.mesh_data["internal_mask"]
        feats = self.cell_centers if node_features is None else \
            _dev_tensor(node_features, torch.float64, self.device)
        if feats.dim() != 2 or feats.shape[0] != self.n_cells:
            raise ValueError("node_features must have one row per mesh cell")
        ei, ea, x, n_nodes = self._build(mode, mask, n_first, True, feats)
        if field_data is not None:      # :241-254, fields appended as given
            cols = [x]
            if "U" in field_data:
                cols.append(_dev_tensor(field_data["U"], torch.float64, self.device).float())
            for name in ("p", "k", "epsilon", "nut"):
                if name in field_data:
                    cols.append(_dev_tensor(field_data[name], torch.float64, self.device)
                                .reshape(-1, 1).float())
            x = torch.cat(cols, 1)
        return Data(x=x, edge_index=ei, edge_attr=ea, num_nodes=n_nodes)

    def get_boundary_mask(self, boundary_name: str) -> torch.Tensor:
        """graph_constructor.py:276-296 (bool [n_cells] on the device)."""
        if boundary_name not in self.mesh_data["boundaries"]:
            raise ValueError(f"Boundary {boundary_name} not found")
        b = self.mesh_data["boundaries"][boundary_name]
        mask = torch.empty(self.n_cells, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib().mignn_boundary_mask(
            _lib.ptr(self.owner), self.owner.numel(), int(b["startFace"]), int(b["nFaces"]),
            self.n_cells, _lib.ptr(mask), _lib.stream(self.device)), "mignn_boundary_mask")
        return mask.bool()
