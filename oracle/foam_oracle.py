"""CPU oracle for the OpenFOAM ASCII reader.  TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker of the native reader
(mignn.openfoam_loader / csrc/foam_reader.hip), never by the product path.

A plain-Python restatement of the parse rules of the reference's
OpenFOAMLoader, pinned to the reference's own outputs on its OpenFOAM case
(tests/golden/mesh.npz) by tests/test_foam_reader.py.  Every function takes
the file's text (not a path) so synthetic edge cases need no files:

  points         openfoam_loader.py:25-46   every "( numbers )" group
  labels         openfoam_loader.py:53-65   digit runs of the whole file,
                                            2nd .. n+1-th (header quirk)
  faces          openfoam_loader.py:72-92   every "k( ids )" group
  scalar_field   openfoam_loader.py:114-142
  vector_field   openfoam_loader.py:144-189 line based
  cell_centers   openfoam_loader.py:191-227 CPython set per cell -- the
                                            real set, so its iteration order
                                            is the reference's by definition
"""

from __future__ import annotations

import io
import re
from collections import defaultdict

import numpy as np

_COUNT = re.compile(r"(\d+)\s*\(")
_NUMS_IN_PARENS = re.compile(r"\(([-\d.eE+\s]+)\)")


def points(text: str) -> np.ndarray:
    if _COUNT.search(text) is None:
        raise ValueError("Could not find number of points")
    return np.array([[float(t) for t in g.split()] for g in _NUMS_IN_PARENS.findall(text)])


def labels(text: str) -> np.ndarray:
    m = _COUNT.search(text)
    if m is None:
        raise ValueError("Could not find array size")
    n = int(m.group(1))
    runs = re.findall(r"\d+", text)
    return np.array([int(r) for r in runs[1:n + 1]], dtype=np.int32)


def faces(text: str) -> list:
    if _COUNT.search(text) is None:
        raise ValueError("Could not find number of faces")
    return [[int(t) for t in ids.split()]
            for _, ids in re.findall(r"(\d+)\s*\(([\d\s]+)\)", text)]


def scalar_field(text: str) -> np.ndarray:
    m = re.search(r"internalField\s+nonuniform\s+List<scalar>\s*(\d+)", text)
    if m is None:
        raise ValueError("Could not find internal field")
    v = re.search(r"internalField[^(]*\(([^)]+)\)", text, re.DOTALL)
    if v is None:
        raise ValueError("Could not find values")
    toks = re.findall(r"[-\d.eE+]+", v.group(1))[:int(m.group(1))]
    return np.array([float(t) for t in toks])


def vector_field(text: str) -> np.ndarray:
    lines = io.StringIO(text).readlines()   # split on '\n' only, like f.readlines()
    n = start = None
    for i, line in enumerate(lines):
        if "internalField" in line and "nonuniform" in line:
            if i + 1 < len(lines):
                m = re.search(r"\d+", lines[i + 1])
                n = int(m.group(0)) if m else None
            start = next((j + 1 for j in range(i + 1, min(i + 5, len(lines)))
                          if "(" in lines[j]), None)
            break
    if n is None or start is None:
        raise ValueError("Could not find internal field")
    out = []
    for line in lines[start:]:
        if len(out) >= n:
            break
        m = _NUMS_IN_PARENS.search(line.strip())
        if m:
            c = [float(t) for t in m.group(1).split()]
            if len(c) == 3:
                out.append(c)
    if len(out) != n:
        raise ValueError(f"Expected {n} vectors, found {len(out)}")
    return np.array(out)


def cell_centers(pts, owner, neighbour, face_list) -> np.ndarray:
    n_cells = int(max(np.max(owner), np.max(neighbour))) + 1
    verts = defaultdict(set)
    for lst in (owner, neighbour):   # owner faces first, then neighbour faces
        for i, c in enumerate(lst):
            verts[int(c)].update(np.asarray(face_list[i], dtype=np.int32))
    out = np.zeros((n_cells, 3))
    for c in range(n_cells):
        if verts.get(c):
            out[c] = np.mean(pts[np.array(list(verts[c]), dtype=np.int32)], axis=0)
    return out
