"""Generate tests/golden/mesh.npz: the reference's mesh arrays and the outputs
of its GraphConstructor on them (SURVEY.md §8f-1 parity fixtures).

Runs ONLY in the build container, where /root/reference exists: it imports
the reference's openfoam_loader.py / graph_constructor.py and runs them on the
reference's own OpenFOAM case (a plain attribute bag stands in for
torch_geometric.data.Data, as in make_golden.py).  Saved (data only):

  mesh/owner, mesh/neighbour      int64, as read by OpenFOAMLoader
  mesh/cell_centers               float64 [n_cells, 3]
  mesh/internal_mask              bool [n_cells]
  mesh/boundary_names, mesh/boundary_start, mesh/boundary_nfaces
  field282/<U|p|k|epsilon|nut>    float64 fields of time 282
  <case>/x, <case>/ei, <case>/ea  GraphConstructor.build_graph outputs for
      internal_n  filter_internal=True, n_internal_cells = len(p)   (train.py)
      internal_m  filter_internal=True (mesh internal_mask)
      all         no filtering                                       (inference.py)
      fields      internal_n + field_data of time 282 (10 features)
  raw/ei, raw/ea                  build_edge_index() / compute_edge_attributes()
  bmask/<name>                    get_boundary_mask(name)

Usage:  python tests/golden/make_mesh_fixture.py
"""

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


class _Data:  # stand-in for torch_geometric.data.Data (attribute bag)
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


def main():
    pyg = types.ModuleType("torch_geometric")
    data = types.ModuleType("torch_geometric.data")
    data.Data = _Data
    pyg.data = data
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.data"] = data
    sys.path.insert(0, REF)
    from openfoam_loader import OpenFOAMLoader
    from graph_constructor import GraphConstructor

    loader = OpenFOAMLoader(os.path.join(REF, "OpenFOAM-data"))
    mesh = loader.load_mesh()
    f282 = loader.load_fields("282")
    gc = GraphConstructor(mesh)
    out = {
        "mesh/owner": np.asarray(mesh["owner"], dtype=np.int64),
        "mesh/neighbour": np.asarray(mesh["neighbour"], dtype=np.int64),
        "mesh/cell_centers": np.asarray(mesh["cell_centers"], dtype=np.float64),
        "mesh/internal_mask": np.asarray(mesh["internal_mask"], dtype=bool),
    }
    names = sorted(mesh["boundaries"])
    out["mesh/boundary_names"] = np.array(names)
    out["mesh/boundary_start"] = np.array([mesh["boundaries"][b]["startFace"] for b in names],
                                          dtype=np.int64)
    out["mesh/boundary_nfaces"] = np.array([mesh["boundaries"][b]["nFaces"] for b in names],
                                           dtype=np.int64)
    for k, v in f282.items():
        out[f"field282/{k}"] = np.asarray(v, dtype=np.float64)
    n_int = len(f282["p"])
    cases = {
        "internal_n": dict(filter_internal=True, n_internal_cells=n_int),
        "internal_m": dict(filter_internal=True),
        "all": dict(),
        "fields": dict(field_data=f282, filter_internal=True, n_internal_cells=n_int),
    }
    for name, kw in cases.items():
        g = gc.build_graph(**kw)
        out[f"{name}/x"] = g.x.numpy()
        out[f"{name}/ei"] = g.edge_index.numpy().astype(np.int64)
        out[f"{name}/ea"] = g.edge_attr.numpy()
        print(name, g.x.shape, tuple(g.edge_index.shape))
    ei = gc.build_edge_index()
    out["raw/ei"] = ei.numpy().astype(np.int64)
    out["raw/ea"] = gc.compute_edge_attributes(ei).numpy()
    for b in names:
        out[f"bmask/{b}"] = gc.get_boundary_mask(b)
    np.savez_compressed(os.path.join(HERE, "mesh.npz"), **out)
    print("wrote", os.path.join(HERE, "mesh.npz"))


if __name__ == "__main__":
    main()
