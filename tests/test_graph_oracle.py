"""The mesh -> graph oracle (oracle/graph_oracle.py) against the reference's
own GraphConstructor outputs on its OpenFOAM case (tests/golden/mesh.npz):
bit-exact edge_index, float32 edge_attr and x."""

import os

import numpy as np
import pytest

from oracle import graph_oracle as go

GOLD = os.path.join(os.path.dirname(__file__), "golden", "mesh.npz")


@pytest.fixture(scope="module")
def fx():
    d = np.load(GOLD)
    mesh = {"owner": d["mesh/owner"], "neighbour": d["mesh/neighbour"],
            "cell_centers": d["mesh/cell_centers"], "n_cells": len(d["mesh/cell_centers"]),
            "internal_mask": d["mesh/internal_mask"]}
    fields = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith("field282/")}
    return d, mesh, fields


CASES = {
    "internal_n": lambda m, f: dict(filter_internal=True, n_internal_cells=len(f["p"])),
    "internal_m": lambda m, f: dict(filter_internal=True),
    "all": lambda m, f: dict(),
    "fields": lambda m, f: dict(field_data=f, filter_internal=True, n_internal_cells=len(f["p"])),
}


@pytest.mark.parametrize("case", list(CASES))
def test_build_graph_matches_reference(fx, case):
    d, mesh, fields = fx
    x, ei, ea, n = go.build_graph(mesh, **CASES[case](mesh, fields))
    assert np.array_equal(ei, d[f"{case}/ei"])
    assert np.array_equal(ea, d[f"{case}/ea"])
    assert np.array_equal(x, d[f"{case}/x"])
    assert n == d[f"{case}/x"].shape[0]


def test_edge_index_and_attributes_match_reference(fx):
    d, mesh, _ = fx
    ei = go.build_edge_index(mesh["owner"], mesh["neighbour"])
    assert np.array_equal(ei, d["raw/ei"])
    assert np.array_equal(go.compute_edge_attributes(ei, mesh["cell_centers"]), d["raw/ea"])


def test_boundary_masks_match_reference(fx):
    d, mesh, _ = fx
    for name, s, n in zip(d["mesh/boundary_names"], d["mesh/boundary_start"],
                          d["mesh/boundary_nfaces"]):
        got = go.get_boundary_mask(mesh["owner"], mesh["n_cells"], int(s), int(n))
        assert np.array_equal(got, d[f"bmask/{name}"]), name
