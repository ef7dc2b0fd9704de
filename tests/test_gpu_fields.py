"""GPU parity of the native output side (mignn.normalization, csrc/fields.hip;
SURVEY.md §8f-4) against the reference's FieldNormalizer on its own case
(tests/golden/fields.npz): inverse_transform / transform bit-exact (float64,
numpy operation order), fit to a few ulp (numpy sums pairwise)."""

import os

import numpy as np
import pytest
import torch

from mignn import _lib
from mignn.normalization import FieldNormalizer

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "fields.npz")
MESH = os.path.join(os.path.dirname(__file__), "golden", "mesh.npz")
NAMES = ("U", "p", "k", "epsilon", "nut")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _lib.lib()


@pytest.fixture(scope="module")
def fx():
    d = np.load(GOLD)
    m = np.load(MESH)
    f282 = {k.split("/", 1)[1]: m[k] for k in m.files if k.startswith("field282/")}
    fn = FieldNormalizer()
    fn.scalers = {k: {"mean": d[f"fit282/{k}/mean"][()], "std": d[f"fit282/{k}/std"][()],
                      "per_component": k == "U"} for k in NAMES}
    return d, f282, fn


def _pred_fields(y):
    return {"U": y[:, :3], "p": y[:, 3:4], "k": y[:, 4:5], "epsilon": y[:, 5:6], "nut": y[:, 6:7]}


def test_inverse_transform_bit_exact(fx):
    d, _, fn = fx
    out = fn.inverse_transform(_pred_fields(d["pred/out"]))
    for k in NAMES:
        assert out[k].dtype == np.float64
        assert np.array_equal(out[k], d[f"pred/{k}"]), k
    # device tensors in, device tensors out, same values
    t = torch.from_numpy(d["pred/out"]).cuda()
    out_t = fn.inverse_transform(_pred_fields(t))
    for k in NAMES:
        assert np.array_equal(out_t[k].cpu().numpy(), d[f"pred/{k}"]), k


def test_transform_bit_exact(fx):
    d, f282, fn = fx
    out = fn.transform(f282)
    for k in NAMES:
        assert np.array_equal(out[k], d[f"norm/{k}"]), k


def test_fit_matches_reference(fx):
    d, f282, _ = fx
    fn = FieldNormalizer()
    fn.fit(f282)
    for k in NAMES:
        np.testing.assert_allclose(fn.scalers[k]["mean"], d[f"fit282/{k}/mean"], rtol=1e-12,
                                   atol=1e-300)
        np.testing.assert_allclose(fn.scalers[k]["std"], d[f"fit282/{k}/std"], rtol=1e-12)
    assert fn.scalers["U"]["per_component"] and not fn.scalers["p"]["per_component"]


def test_numpy_legacy_float32_path(fx):
    """numpy < 2: float32 field * float64 scalar stays float32."""
    d, _, fn = fx
    fl = FieldNormalizer(numpy_legacy=True)
    fl.scalers = fn.scalers
    out = fl.inverse_transform(_pred_fields(d["pred/out"]))
    for k in ("p", "k", "epsilon", "nut"):
        sc = fn.scalers[k]
        x = _pred_fields(d["pred/out"])[k]
        ref = x * np.float32(sc["std"]) + np.float32(sc["mean"])
        assert out[k].dtype == np.float32 and np.array_equal(out[k], ref.astype(np.float32)), k
    assert out["U"].dtype == np.float64 and np.array_equal(out["U"], d["pred/U"])
