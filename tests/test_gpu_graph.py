"""GPU parity of the native mesh -> graph builder (mignn.graph,
csrc/graph_construct.hip): bit-exact against the reference's
own GraphConstructor outputs on its OpenFOAM case (tests/golden/mesh.npz) and
against the oracle (oracle/graph_oracle.py, itself pinned to those outputs)
on synthetic meshes with the edge cases the reference handles: isolated
cells, filtered cells, masks with holes, no internal faces, coincident
centres, extra node features and field columns."""

import os

import numpy as np
import pytest
import torch

from mignn import _lib
from mignn.graph import GraphConstructor
from oracle import graph_oracle as go

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden", "mesh.npz")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


@pytest.fixture(scope="module")
def fx():
    d = np.load(GOLD)
    names = [str(n) for n in d["mesh/boundary_names"]]
    mesh = {"owner": d["mesh/owner"], "neighbour": d["mesh/neighbour"],
            "cell_centers": d["mesh/cell_centers"], "n_cells": len(d["mesh/cell_centers"]),
            "internal_mask": d["mesh/internal_mask"],
            "boundaries": {n: {"startFace": int(s), "nFaces": int(c)} for n, s, c in
                           zip(names, d["mesh/boundary_start"], d["mesh/boundary_nfaces"])}}
    fields = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith("field282/")}
    return d, mesh, fields


CASES = {
    "internal_n": lambda f: dict(filter_internal=True, n_internal_cells=len(f["p"])),
    "internal_m": lambda f: dict(filter_internal=True),
    "all": lambda f: dict(),
    "fields": lambda f: dict(field_data=f, filter_internal=True, n_internal_cells=len(f["p"])),
}


@pytest.mark.parametrize("case", list(CASES))
def test_build_graph_matches_reference(fx, case):
    d, mesh, fields = fx
    g = GraphConstructor(mesh).build_graph(**CASES[case](fields))
    assert np.array_equal(g.edge_index.cpu().numpy(), d[f"{case}/ei"])
    assert np.array_equal(g.edge_attr.cpu().numpy(), d[f"{case}/ea"])
    assert np.array_equal(g.x.cpu().numpy(), d[f"{case}/x"])
    assert g.num_nodes == d[f"{case}/x"].shape[0]


def test_edge_index_attributes_masks_match_reference(fx):
    d, mesh, _ = fx
    gc = GraphConstructor(mesh)
    ei = gc.build_edge_index()
    assert np.array_equal(ei.cpu().numpy(), d["raw/ei"])
    assert np.array_equal(gc.compute_edge_attributes(ei).cpu().numpy(), d["raw/ea"])
    for name in mesh["boundaries"]:
        assert np.array_equal(gc.get_boundary_mask(name).cpu().numpy(), d[f"bmask/{name}"]), name
    with pytest.raises(ValueError):
        gc.get_boundary_mask("no_such_patch")


def _random_mesh(seed, n_cells=300, n_int=500, n_bnd=120, holes=True):
    """A face list like a polyMesh: internal faces (o < n), then boundary
    faces; some cells referenced by no face (isolated), duplicated centres."""
    r = np.random.default_rng(seed)
    used = n_cells - 7 if holes else n_cells
    o = r.integers(0, used - 1, n_int)
    n = o + 1 + r.integers(0, np.maximum(1, used - 1 - o))
    n = np.minimum(n, used - 1)
    ob = r.integers(0, used, n_bnd)
    cc = r.normal(size=(n_cells, 3))
    cc[5] = cc[6]                                  # coincident centres
    mask = r.random(n_cells) < 0.8
    return {"owner": np.concatenate([o, ob]), "neighbour": n, "cell_centers": cc,
            "n_cells": n_cells, "internal_mask": mask,
            "boundaries": {"wall": {"startFace": n_int, "nFaces": n_bnd},
                           "past_end": {"startFace": n_int + n_bnd - 10, "nFaces": 40}}}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_synthetic_meshes_vs_oracle(seed):
    mesh = _random_mesh(seed)
    gc = GraphConstructor(mesh)
    feats = np.random.default_rng(seed + 10).normal(size=(mesh["n_cells"], 5))
    fields = {"U": np.random.default_rng(seed).normal(size=(120, 3)),
              "p": np.random.default_rng(seed + 1).normal(size=120)}
    for kw in (dict(), dict(filter_internal=True), dict(filter_internal=True, n_internal_cells=120),
               dict(filter_internal=True, n_internal_cells=0), dict(node_features=feats),
               dict(field_data=fields, filter_internal=True, n_internal_cells=120),
               dict(filter_internal=True, n_internal_cells=mesh["n_cells"])):
        g = gc.build_graph(**kw)
        x, ei, ea, n = go.build_graph(mesh, **kw)
        assert g.num_nodes == n, kw
        assert np.array_equal(g.edge_index.cpu().numpy(), ei), kw
        assert np.array_equal(g.edge_attr.cpu().numpy(), ea), kw
        assert np.array_equal(g.x.cpu().numpy(), x), kw
    for name, b in mesh["boundaries"].items():
        got = gc.get_boundary_mask(name).cpu().numpy()
        ref = go.get_boundary_mask(mesh["owner"], mesh["n_cells"], b["startFace"], b["nFaces"])
        assert np.array_equal(got, ref), name


def test_no_internal_faces_and_invalid_attribute_ids():
    """Only boundary faces, filtered: no edges -> a self-loop per node (:221-226);
    compute_edge_attributes gives zeros for ids outside the mesh."""
    mesh = {"owner": np.array([0, 1, 2, 2]), "neighbour": np.array([], dtype=np.int64),
            "cell_centers": np.random.default_rng(0).normal(size=(4, 3)), "n_cells": 4,
            "boundaries": {}}
    gc = GraphConstructor(mesh)
    for kw in (dict(filter_internal=True, n_internal_cells=3), dict()):
        g = gc.build_graph(**kw)
        x, ei, ea, n = go.build_graph(mesh, **kw)
        assert np.array_equal(g.edge_index.cpu().numpy(), ei)
        assert np.array_equal(g.edge_attr.cpu().numpy(), ea)
    bad = torch.tensor([[0, 9, -1, 1], [1, 0, 2, 1]], device=DEV)
    ea = gc.compute_edge_attributes(bad).cpu().numpy()
    assert np.array_equal(ea, go.compute_edge_attributes(bad.cpu().numpy(), mesh["cell_centers"]))
    assert (ea[1:] == 0).all()
