"""OpenFOAM ASCII case reader: drop-in for the reference's
`openfoam_loader.OpenFOAMLoader` (openfoam_loader.py:12-296).

Same class, method names, return types and error behaviour; the parsing and
the cell-centre computation run in libmignn.so (csrc/foam_reader.hip, host
code -- byte scanning and a per-cell vertex set, nothing for the GPU).

`compat="reference"` (default) reproduces the reference's parse exactly,
including the header-digit quirk of `read_array` (openfoam_loader.py:62-65:
every digit run of the file counts, so owner/neighbour get the header's
numbers prepended and n_cells becomes 49,181 on the bundled case); that is
the graph the reference's models are trained and evaluated on.
`compat="openfoam"` reads owner/neighbour as OpenFOAM defines the list (the
count after the FoamFile header), i.e. the true 12,225-cell mesh.

Faces come back as a `FaceList` (CSR offsets + vertex ids) that indexes like
the reference's object array (`faces[i]` -> that face's vertex ids).
"""

from __future__ import annotations

import ctypes
import re
from pathlib import Path
from typing import Dict, Tuple

import numpy as np

from . import _lib

_COMPAT = {"reference": 0, "openfoam": 1}


def _read_bytes(path: Path) -> bytes:
    # text mode like the reference's open(..., 'r'): universal newlines
    with open(path, "r") as f:
        return f.read().encode()


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _call(name: str, *args):
    _lib.check(getattr(_lib.lib(), name)(*args), name)


class FaceList:
    """Faces as CSR (offsets [n+1], verts); `faces[i]` is face i's vertex ids."""

    def __init__(self, offsets: np.ndarray, verts: np.ndarray):
        self.offsets = offsets
        self.verts = verts

    def __len__(self) -> int:
        return len(self.offsets) - 1

    def __getitem__(self, i):
        return self.verts[self.offsets[i]:self.offsets[i + 1]]

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


def _as_facelist(faces) -> FaceList:
    if isinstance(faces, FaceList):
        return faces
    lens = np.array([len(f) for f in faces], dtype=np.int64)
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    verts = (np.concatenate([np.asarray(f, dtype=np.int64) for f in faces])
             if len(lens) else np.zeros(0, np.int64))
    return FaceList(off, verts)


class OpenFOAMLoader:
    """Loads OpenFOAM mesh and field data (openfoam_loader.py:12-23)."""

    def __init__(self, case_path: str, compat: str = "reference"):
        if compat not in _COMPAT:
            raise ValueError(f"compat must be one of {sorted(_COMPAT)}")
        self.case_path = Path(case_path)
        self.mesh_path = self.case_path / "constant" / "polyMesh"
        self.compat = compat

    # -- mesh files ---------------------------------------------------------
    def read_points(self) -> np.ndarray:
        """openfoam_loader.py:25-46 -> float64 [n_points, 3]."""
        buf = _read_bytes(self.mesh_path / "points")
        out = np.empty((buf.count(b"(") + 1, 3), dtype=np.float64)
        n = ctypes.c_int64(0)
        _call("mignn_foam_parse_points", buf, len(buf), _p(out), out.shape[0], ctypes.byref(n))
        return out[:n.value].copy()

    def read_owner_neighbour(self) -> Tuple[np.ndarray, np.ndarray]:
        """openfoam_loader.py:48-70 -> (owner, neighbour) int32, like the reference."""
        def read_array(path: Path) -> np.ndarray:
            buf = _read_bytes(path)
            out = np.empty(len(buf) // 2 + 1, dtype=np.int64)
            n = ctypes.c_int64(0)
            try:
                _call("mignn_foam_parse_labels", buf, len(buf), _COMPAT[self.compat], _p(out),
                      out.shape[0], ctypes.byref(n))
            except _lib.MignnError as e:
                if "array size" in str(e):
                    raise ValueError(f"Could not find array size in {path}") from None
                raise
            return out[:n.value].astype(np.int32)

        return (read_array(self.mesh_path / "owner"),
                read_array(self.mesh_path / "neighbour"))

    def read_faces(self) -> FaceList:
        """openfoam_loader.py:72-92 -> FaceList (the reference: object array of lists)."""
        buf = _read_bytes(self.mesh_path / "faces")
        cap_f = buf.count(b"(") + 1
        off = np.empty(cap_f + 1, dtype=np.int64)
        verts = np.empty(len(buf) // 2 + 1, dtype=np.int64)
        nf, nv = ctypes.c_int64(0), ctypes.c_int64(0)
        _call("mignn_foam_parse_faces", buf, len(buf), _p(off), cap_f, _p(verts), verts.shape[0],
              ctypes.byref(nf), ctypes.byref(nv))
        return FaceList(off[:nf.value + 1].copy(), verts[:nv.value].copy())

    def read_boundary(self) -> Dict:
        """openfoam_loader.py:94-112: patch name -> {type, nFaces, startFace}.

        A few hundred bytes of dictionary text; parsed with the same pattern
        the reference uses so patch selection is identical."""
        content = (self.mesh_path / "boundary").read_text()
        pattern = r"(\w+)\s*\{[^}]*type\s+(\w+);[^}]*nFaces\s+(\d+);[^}]*startFace\s+(\d+);"
        return {name: {"type": t, "nFaces": int(nf), "startFace": int(sf)}
                for name, t, nf, sf in re.findall(pattern, content, re.DOTALL)}

    # -- fields -------------------------------------------------------------
    def _field_bytes(self, time_dir: str, field_name: str) -> bytes:
        path = self.case_path / time_dir / field_name
        if not path.exists():
            raise FileNotFoundError(f"Field file not found: {path}")
        return _read_bytes(path)

    def read_scalar_field(self, time_dir: str, field_name: str) -> np.ndarray:
        """openfoam_loader.py:114-142 -> float64 [n]."""
        buf = self._field_bytes(time_dir, field_name)
        out = np.empty(len(buf) // 2 + 1, dtype=np.float64)
        n = ctypes.c_int64(0)
        try:
            _call("mignn_foam_parse_scalar_field", buf, len(buf), _p(out), out.shape[0],
                  ctypes.byref(n))
        except _lib.MignnError as e:
            raise ValueError(f"{e} in {field_name}") from None
        return out[:n.value].copy()

    def read_vector_field(self, time_dir: str, field_name: str) -> np.ndarray:
        """openfoam_loader.py:144-189 -> float64 [n, 3]."""
        buf = self._field_bytes(time_dir, field_name)
        out = np.empty((buf.count(b"(") + 1, 3), dtype=np.float64)
        n = ctypes.c_int64(0)
        try:
            _call("mignn_foam_parse_vector_field", buf, len(buf), _p(out), out.shape[0],
                  ctypes.byref(n))
        except _lib.MignnError as e:
            raise ValueError(f"{e} in {field_name}") from None
        return out[:n.value].copy()

    # -- derived mesh data --------------------------------------------------
    def get_cell_centers(self, points: np.ndarray, owner: np.ndarray, neighbour: np.ndarray,
                         faces) -> np.ndarray:
        """openfoam_loader.py:191-227: mean of each cell's unique vertices, float64,
        bit-identical to the reference (its set iteration order is emulated)."""
        pts = np.ascontiguousarray(points, dtype=np.float64)
        own = np.ascontiguousarray(owner, dtype=np.int64)
        nei = np.ascontiguousarray(neighbour, dtype=np.int64)
        fl = _as_facelist(faces)
        off = np.ascontiguousarray(fl.offsets, dtype=np.int64)
        verts = np.ascontiguousarray(fl.verts, dtype=np.int64)
        n_cells = int(max(own.max(), nei.max())) + 1
        centers = np.zeros((n_cells, 3), dtype=np.float64)
        _call("mignn_foam_cell_centers", _p(pts), pts.shape[0], _p(own), own.shape[0], _p(nei),
              nei.shape[0], _p(off), _p(verts), len(fl), n_cells, _p(centers))
        return centers

    def get_internal_cells(self, owner: np.ndarray, neighbour: np.ndarray) -> np.ndarray:
        """openfoam_loader.py:229-248: cells touching an internal face."""
        n_cells = int(max(np.max(owner), np.max(neighbour))) + 1
        mask = np.zeros(n_cells, dtype=bool)
        mask[np.asarray(neighbour)] = True
        mask[np.asarray(owner)[:len(neighbour)]] = True
        return mask

    def load_mesh(self) -> Dict:
        """openfoam_loader.py:250-269 (same keys)."""
        points = self.read_points()
        owner, neighbour = self.read_owner_neighbour()
        faces = self.read_faces()
        boundaries = self.read_boundary()
        cell_centers = self.get_cell_centers(points, owner, neighbour, faces)
        internal_mask = self.get_internal_cells(owner, neighbour)
        return {
            "points": points,
            "owner": owner,
            "neighbour": neighbour,
            "faces": faces,
            "boundaries": boundaries,
            "cell_centers": cell_centers,
            "n_cells": len(cell_centers),
            "internal_mask": internal_mask,
            "n_internal_cells": np.sum(internal_mask),
        }

    def load_fields(self, time_dir: str, fields: list = None) -> Dict:
        """openfoam_loader.py:271-296: missing / unparsable fields are warned and skipped."""
        if fields is None:
            fields = ["U", "p", "k", "epsilon", "nut"]
        field_data = {}
        for field in fields:
            try:
                if field == "U":
                    field_data[field] = self.read_vector_field(time_dir, field)
                else:
                    field_data[field] = self.read_scalar_field(time_dir, field)
            except (FileNotFoundError, ValueError) as e:
                print(f"Warning: Could not load field {field}: {e}")
        return field_data
