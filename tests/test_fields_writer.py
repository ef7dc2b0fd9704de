"""Native OpenFOAM ASCII writer (host code in libmignn.so)
against the files the reference's save_fields_openfoam_format
(inference.py:90-178) wrote for the same fields (tests/golden/fields.npz).
Host-only: runs without a GPU."""

import os

import numpy as np
import pytest

from mignn.normalization import save_fields_openfoam_format

GOLD = os.path.join(os.path.dirname(__file__), "golden", "fields.npz")


def test_writer_byte_identical_to_reference(tmp_path):
    d = np.load(GOLD)
    fields = {k: d[f"pred/{k}"] for k in ("U", "p", "k", "epsilon", "nut")}
    save_fields_openfoam_format(fields, str(tmp_path), "predicted")
    for k in fields:
        got = (tmp_path / "predicted" / k).read_bytes()
        assert got == d[f"of/{k}"].tobytes(), k


@pytest.mark.parametrize("v", [0.0, -0.0, 1e-300, -1e300, 5e-324, 123456.789, float("inf"),
                               float("-inf"), float("nan"), -float("nan"), 9.9999995e-7, 0.5e-5])
def test_value_format_matches_python(tmp_path, v):
    fields = {"U": np.array([[v, -v, 1.0]]), "p": np.array([[v]])}
    save_fields_openfoam_format(fields, str(tmp_path), "t")
    lines = (tmp_path / "t" / "p").read_text().splitlines()
    i = lines.index("(")
    assert lines[i + 1] == f"{v:.6e}"
    lines = (tmp_path / "t" / "U").read_text().splitlines()
    i = lines.index("(")
    assert lines[i + 1] == f"({v:.6e} {-v:.6e} {1.0:.6e})"
