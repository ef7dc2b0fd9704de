"""OpenFOAM ASCII reader: the native reader
(mignn.openfoam_loader -> csrc/foam_reader.hip, host code) and the oracle
(oracle/foam_oracle.py), both against the reference loader's outputs on its
own case (tests/golden/mesh.npz; the case's files are in foam_case.npz), and
native vs oracle on synthetic edge cases.  Host-only: no GPU needed."""

import os

import numpy as np
import pytest

from mignn.openfoam_loader import FaceList, OpenFOAMLoader
from oracle import foam_oracle as fo

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def case_dir(tmp_path_factory):
    root = tmp_path_factory.mktemp("foam_case")
    with np.load(os.path.join(GOLD, "foam_case.npz")) as z:
        for rel in z.files:
            p = root / rel
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(z[rel].tobytes())
    return root


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "mesh.npz"))


def _text(case_dir, rel):
    return (case_dir / rel).read_text()


# -- the reference's case ----------------------------------------------------

def test_oracle_matches_reference_outputs(case_dir, gold):
    pm = "constant/polyMesh/"
    own = fo.labels(_text(case_dir, pm + "owner"))
    nei = fo.labels(_text(case_dir, pm + "neighbour"))
    assert np.array_equal(own, gold["mesh/owner"])
    assert np.array_equal(nei, gold["mesh/neighbour"])
    pts = fo.points(_text(case_dir, pm + "points"))
    fl = fo.faces(_text(case_dir, pm + "faces"))
    assert np.array_equal(fo.cell_centers(pts, own, nei, fl), gold["mesh/cell_centers"])
    assert np.array_equal(fo.vector_field(_text(case_dir, "282/U")), gold["field282/U"])
    for f in ("p", "k", "epsilon", "nut"):
        assert np.array_equal(fo.scalar_field(_text(case_dir, "282/" + f)), gold["field282/" + f])


def test_native_load_mesh_bit_exact(case_dir, gold):
    m = OpenFOAMLoader(str(case_dir)).load_mesh()
    assert m["owner"].dtype == np.int32 and m["neighbour"].dtype == np.int32
    assert np.array_equal(m["owner"], gold["mesh/owner"])
    assert np.array_equal(m["neighbour"], gold["mesh/neighbour"])
    assert m["n_cells"] == 49181                        # the header-digit quirk
    assert np.array_equal(m["cell_centers"], gold["mesh/cell_centers"])
    assert np.array_equal(m["internal_mask"], gold["mesh/internal_mask"])
    assert m["n_internal_cells"] == gold["mesh/internal_mask"].sum()
    names = list(gold["mesh/boundary_names"])
    assert sorted(m["boundaries"]) == names
    assert [m["boundaries"][b]["startFace"] for b in names] == list(gold["mesh/boundary_start"])
    assert [m["boundaries"][b]["nFaces"] for b in names] == list(gold["mesh/boundary_nfaces"])


def test_native_faces_and_points_match_oracle(case_dir):
    L = OpenFOAMLoader(str(case_dir))
    fl = L.read_faces()
    ref = fo.faces(_text(case_dir, "constant/polyMesh/faces"))
    assert len(fl) == len(ref) == 49180
    assert np.array_equal(fl.verts, np.concatenate([np.asarray(f) for f in ref]))
    assert list(fl[7]) == ref[7]
    assert np.array_equal(L.read_points(), fo.points(_text(case_dir, "constant/polyMesh/points")))


def test_native_fields_bit_exact(case_dir, gold):
    f = OpenFOAMLoader(str(case_dir)).load_fields("282")
    assert sorted(f) == ["U", "epsilon", "k", "nut", "p"]
    for k, v in f.items():
        assert np.array_equal(v, gold["field282/" + k]), k


def test_openfoam_compat_reads_true_mesh(case_dir, gold):
    m = OpenFOAMLoader(str(case_dir), compat="openfoam").load_mesh()
    assert m["n_cells"] == 12225
    assert len(m["owner"]) == 49180 and len(m["neighbour"]) == 24170
    # the quirk prepends 9 header numbers: the true lists are the shifted ones
    assert np.array_equal(m["owner"][:-9], gold["mesh/owner"][9:])
    assert np.array_equal(m["neighbour"][:-9], gold["mesh/neighbour"][9:])
    assert (m["cell_centers"] != 0).any(axis=1).all()
    with pytest.raises(ValueError):
        OpenFOAMLoader(str(case_dir), compat="bogus")


def test_missing_field_is_skipped(case_dir, capsys):
    f = OpenFOAMLoader(str(case_dir)).load_fields("282", ["p", "omega"])
    assert list(f) == ["p"]
    assert "Could not load field omega" in capsys.readouterr().out


# -- synthetic edge cases: native vs oracle -----------------------------------

HEADER = ("/* banner Version: 2412 */\nFoamFile\n{\n    version     2.0;\n"
          "    note        \"nCells:3\";\n}\n// * * //\n\n")


def _write_case(root, owner, neighbour, faces, points):
    pm = root / "constant" / "polyMesh"
    pm.mkdir(parents=True, exist_ok=True)
    lab = lambda a: HEADER + f"{len(a)}\n(\n" + "\n".join(map(str, a)) + "\n)\n"
    (pm / "owner").write_text(lab(owner))
    (pm / "neighbour").write_text(lab(neighbour))
    (pm / "faces").write_text(HEADER + f"{len(faces)}\n(\n" + "\n".join(
        f"{len(f)}(" + " ".join(map(str, f)) + ")" for f in faces) + "\n)\n")
    (pm / "points").write_text(HEADER + f"{len(points)}\n(\n" + "\n".join(
        "(" + " ".join(repr(float(c)) for c in p) + ")" for p in points) + "\n)\n")
    (pm / "boundary").write_text(HEADER + "1\n(\n    wall\n    {\n        type wall;\n"
                                 "        nFaces 1;\n        startFace 2;\n    }\n)\n")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_polyhedral_mesh_matches_oracle(tmp_path, seed):
    """Random faces of 3-12 vertices with ids up to 5000: sets grow through
    several CPython table resizes and probe collisions, so the emulated
    iteration order (and the float64 sums that depend on it) is exercised."""
    rng = np.random.default_rng(seed)
    n_pts, n_faces, n_cells = 5000, 400, 60
    pts = rng.standard_normal((n_pts, 3)) * 10.0 ** rng.integers(-3, 4, (n_pts, 1))
    faces = [list(rng.integers(0, n_pts, rng.integers(3, 13))) for _ in range(n_faces)]
    owner = list(rng.integers(0, n_cells, n_faces))
    neighbour = list(rng.integers(0, n_cells, 150))
    _write_case(tmp_path, owner, neighbour, faces, pts)
    m = OpenFOAMLoader(str(tmp_path)).load_mesh()
    pm = tmp_path / "constant" / "polyMesh"
    o = fo.labels((pm / "owner").read_text())
    n = fo.labels((pm / "neighbour").read_text())
    assert np.array_equal(m["owner"], o) and np.array_equal(m["neighbour"], n)
    p = fo.points((pm / "points").read_text())
    assert np.array_equal(m["points"], p)
    fl = fo.faces((pm / "faces").read_text())
    assert np.array_equal(m["cell_centers"], fo.cell_centers(p, o, n, fl))
    # the header digits (2412, 2, 0, 3) are prepended, like the reference
    assert list(m["owner"][:4]) == [2, 0, 3, len(owner)]
    # cell centres also accept the reference's list-of-lists faces
    L = OpenFOAMLoader(str(tmp_path))
    assert np.array_equal(L.get_cell_centers(p, o, n, fl), m["cell_centers"])


def test_large_vertex_sets_match_python_set_order(tmp_path):
    """One cell with ~3000 unique vertices (resizes past 50k-style growth
    rules are irrelevant here, but many x4 growths happen) and vertex ids with
    colliding low bits."""
    rng = np.random.default_rng(7)
    ids = np.unique(rng.integers(0, 1 << 16, 4000) * 64)[:3000]
    n_pts = int(ids.max()) + 1
    pts = rng.standard_normal((n_pts, 3))
    faces = [list(ids[i:i + 10]) for i in range(0, len(ids), 10)]
    own = [0] * len(faces)
    nei = [0]
    L = OpenFOAMLoader(str(tmp_path))
    c = L.get_cell_centers(pts, np.array(own), np.array(nei), faces)
    assert np.array_equal(c, fo.cell_centers(pts, np.array(own), np.array(nei), faces))


def _field_case(tmp_path, name, text):
    d = tmp_path / "5"
    d.mkdir(exist_ok=True)
    (d / name).write_text(text)
    return OpenFOAMLoader(str(tmp_path))


SCALAR = (HEADER + "dimensions [0 2 -2 0 0 0 0];\n\ninternalField   nonuniform List<scalar> \n5\n(\n"
          "1.5\n-2e-3\n+7\n.25\n3.E2\n9\n)\n;\nboundaryField { }\n")
VECTOR = (HEADER + "internalField   nonuniform List<vector> \n4\n(\n(1 2 3)\n\n(4 5)\n"
          "  (-1e-3 2.5E+2 .5)  \n(7 8 9) (10 11 12)\n(0 0 0)\n)\n;\n")


def test_scalar_field_edge_cases(tmp_path):
    L = _field_case(tmp_path, "p", SCALAR)
    got = L.read_scalar_field("5", "p")
    assert np.array_equal(got, fo.scalar_field(SCALAR))
    assert len(got) == 5                               # only the first n values
    L = _field_case(tmp_path, "q", HEADER + "internalField uniform 0;\n")
    with pytest.raises(ValueError):
        L.read_scalar_field("5", "q")
    with pytest.raises(FileNotFoundError):
        L.read_scalar_field("5", "nope")


def test_vector_field_edge_cases(tmp_path):
    L = _field_case(tmp_path, "U", VECTOR)
    got = L.read_vector_field("5", "U")
    assert np.array_equal(got, fo.vector_field(VECTOR))
    assert got.shape == (4, 3)                          # 2-tuple skipped, 1st group per line
    short = VECTOR.replace("\n4\n", "\n6\n")
    L = _field_case(tmp_path, "V", short)
    with pytest.raises(ValueError, match="Expected 6 vectors"):
        L.read_vector_field("5", "V")


def test_labels_without_count_raise(tmp_path):
    pm = tmp_path / "constant" / "polyMesh"
    pm.mkdir(parents=True)
    (pm / "owner").write_text("no list here 1 2 3\n")
    (pm / "neighbour").write_text("2(0 1)\n")
    with pytest.raises(ValueError, match="array size"):
        OpenFOAMLoader(str(tmp_path)).read_owner_neighbour()


def test_facelist_container():
    fl = FaceList(np.array([0, 3, 7]), np.arange(7))
    assert len(fl) == 2 and list(fl[1]) == [3, 4, 5, 6]
    assert [list(f) for f in fl] == [[0, 1, 2], [3, 4, 5, 6]]
