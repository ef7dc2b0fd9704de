"""Output side of the inference path: the reference's
`FieldNormalizer` (normalization.py:11-133), `predict_fields`
(inference.py:62-87) and `save_fields_openfoam_format` (inference.py:90-178),
on the native kernels / host writer of csrc/fields.hip.

* The scalers keep the reference's layout ({'mean', 'std', 'per_component'}
  per field, numpy float64), so `normalizer.scalers = checkpoint[...]`
  (inference.py:55-57) works unchanged.
* `inverse_transform` / `transform` run on the device in float64 with
  numpy's operation order (multiply, then add; no FMA): bit-identical to the
  reference under NumPy >= 2.  `numpy_legacy=True` reproduces numpy < 2
  value-based casting (scalar scalers keep float32 fields float32).
* The writer produces byte-identical files ("%.6e"), natively.
* `WeightedMSELoss` (normalization.py:136-250), the training criterion of
  train.py:352-363, with its forward and backward on the device
  (mignn_wmse_loss).
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import train_ops as _T

_SCALAR_FIELDS = {
    "p": ("[0 2 -2 0 0 0 0]", "volScalarField"),
    "k": ("[0 2 -2 0 0 0 0]", "volScalarField"),
    "epsilon": ("[0 2 -3 0 0 0 0]", "volScalarField"),
    "nut": ("[0 2 -1 0 0 0 0]", "volScalarField"),
}


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("mignn FieldNormalizer runs on ROCm devices only (no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def _to_dev(a, dev):
    if torch.is_tensor(a):
        return a.to(dev)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


class FieldNormalizer:
    """normalization.py:11-133 on the device."""

    def __init__(self, numpy_legacy: bool = False):
        self.scalers: Dict[str, dict] = {}
        self.field_stats: Dict[str, dict] = {}
        self.numpy_legacy = numpy_legacy

    # ---------------------------------------------------------------- fit
    def fit(self, fields_dict: Dict):
        """normalization.py:18-84 (population std, std <= 1e-10 -> 1.0)."""
        dev = _device()
        for name, data in fields_dict.items():
            x = _to_dev(data, dev)
            x = x if x.dtype in (torch.float32, torch.float64) else x.double()
            per_comp = name == "U" and x.dim() == 2 and x.shape[1] == 3
            cols = x.contiguous() if per_comp else x.reshape(-1, 1).contiguous()
            flat = x.reshape(-1, 1).contiguous()
            mean_c, std_c = self._moments(cols)
            mean_f, std_f = self._moments(flat) if per_comp else (mean_c, std_c)
            mn, mx = float(flat.min()), float(flat.max())
            stats = {"mean": np.float64(mean_f[0]), "std": np.float64(std_f[0]),
                     "min": mn, "max": mx}
            if per_comp:
                stats["per_component_mean"] = mean_c.tolist()
                stats["per_component_std"] = std_c.tolist()
                self.scalers[name] = {"mean": mean_c, "std": np.where(std_c > 1e-10, std_c, 1.0),
                                      "per_component": True}
            else:
                s = np.float64(std_c[0])
                self.scalers[name] = {"mean": np.float64(mean_c[0]),
                                      "std": s if s > 1e-10 else 1.0, "per_component": False}
            self.field_stats[name] = stats

    @staticmethod
    def _moments(cols: torch.Tensor):
        n, c = cols.shape
        mean = torch.empty(c, dtype=torch.float64, device=cols.device)
        std = torch.empty(c, dtype=torch.float64, device=cols.device)
        _lib.check(_lib.lib().mignn_field_moments(
            _lib.ptr(cols), int(cols.dtype == torch.float64), cols.stride(0), n, c,
            _lib.ptr(mean), _lib.ptr(std), _lib.stream(cols.device)), "mignn_field_moments")
        return mean.cpu().numpy(), std.cpu().numpy()

    # ---------------------------------------------------------------- apply
    def _apply(self, fields_dict: Dict, inverse: bool) -> Dict:
        dev = _device()
        out = {}
        for name, data in fields_dict.items():
            if name not in self.scalers:
                out[name] = data
                continue
            sc = self.scalers[name]
            as_numpy = not torch.is_tensor(data)
            x = _to_dev(data, dev)
            if x.dtype not in (torch.float32, torch.float64):
                x = x.double()
            shape = x.shape
            per = name == "U" and sc.get("per_component", False)
            ncol = shape[-1] if (per and x.dim() >= 1) else 1
            x2 = x.reshape(-1, ncol).contiguous()
            mean = np.broadcast_to(np.asarray(sc["mean"], dtype=np.float64), (ncol,))
            std = np.broadcast_to(np.asarray(sc["std"], dtype=np.float64), (ncol,))
            m_d = torch.tensor(np.ascontiguousarray(mean), device=dev)
            s_d = torch.tensor(np.ascontiguousarray(std), device=dev)
            # numpy < 2: a float64 *scalar* scaler leaves a float32 field float32
            legacy = (self.numpy_legacy and x.dtype == torch.float32
                      and np.ndim(sc["mean"]) == 0 and np.ndim(sc["std"]) == 0)
            y = torch.empty(x2.shape, dtype=torch.float32 if legacy else torch.float64, device=dev)
            _lib.check(_lib.lib().mignn_field_affine(
                _lib.ptr(x2), int(x2.dtype == torch.float64), x2.stride(0), x2.shape[0], ncol,
                _lib.ptr(m_d), _lib.ptr(s_d), int(inverse), (1 << ncol) - 1 if legacy else 0,
                None if legacy else _lib.ptr(y), _lib.ptr(y) if legacy else None, y.stride(0),
                _lib.stream(dev)), "mignn_field_affine")
            y = y.reshape(shape)
            out[name] = y.cpu().numpy() if as_numpy else y
        return out

    def transform(self, fields_dict: Dict) -> Dict:
        """normalization.py:86-108: (x - mean) / std."""
        return self._apply(fields_dict, inverse=False)

    def inverse_transform(self, fields_dict: Dict) -> Dict:
        """normalization.py:110-133: x * std + mean."""
        return self._apply(fields_dict, inverse=True)


def predict_fields(model, graph_data, device="cuda", normalizer=None) -> Dict[str, np.ndarray]:
    """inference.py:62-87: forward, split into fields, denormalise (device),
    numpy out."""
    model.eval()
    with torch.no_grad():
        x = graph_data.x.to(device)
        ei = graph_data.edge_index.to(device)
        ea = None if graph_data.edge_attr is None else graph_data.edge_attr.to(device)
        fields = model.predict_fields(model(x, ei, ea))
        if normalizer is not None:
            fields = normalizer.inverse_transform(fields)
        return {k: v.cpu().numpy() for k, v in fields.items()}


def save_fields_openfoam_format(fields: Dict, output_dir: str, time_dir: str = "predicted"):
    """inference.py:90-178, byte-identical files (native writer)."""
    out = Path(output_dir) / time_dir
    out.mkdir(parents=True, exist_ok=True)
    L = _lib.lib()

    def write(name, cls, dims, arr, ncomp):
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float64).reshape(len(arr), -1))
        if a.shape[1] < ncomp:
            raise ValueError(f"{name}: expected {ncomp} components, got {a.shape[1]}")
        _lib.check(L.mignn_write_openfoam_field(
            os.fsencode(str(out / name)), cls.encode(), name.encode(), time_dir.encode(),
            dims.encode(), a.ctypes.data, a.shape[0], ncomp, a.shape[1]),
            "mignn_write_openfoam_field")

    fields["U"]   # the reference reads n_cells from U first (inference.py:101)
    if "U" in fields:
        write("U", "volVectorField", "[0 1 -1 0 0 0 0]", fields["U"], 3)
    for name, (dims, cls) in _SCALAR_FIELDS.items():
        if name in fields:
            write(name, cls, dims, fields[name], 1)


class WeightedMSELoss(nn.Module):
    """normalization.py:136-250: per-field MSE, weighted, plus the pressure
    reference term w_p * prw * (mean(p_pred) - mean(p_target))^2 (fieldwise),
    or the element-weighted mean (use_fieldwise=False).  Device-only."""

    def __init__(self, field_weights: Dict[str, float] = None, use_fieldwise: bool = True,
                 pressure_ref_weight: float = 0.1):
        super().__init__()
        if field_weights is None:
            field_weights = {"U": 1.0, "p": 3.0, "k": 0.5, "epsilon": 0.5, "nut": 0.5}
        self.field_weights = field_weights
        self.use_fieldwise = use_fieldwise
        self.pressure_ref_weight = pressure_ref_weight
        g = field_weights.get
        self.weights = torch.tensor([g("U", 1.0), g("U", 1.0), g("U", 1.0), g("p", 1.0),
                                     g("k", 0.5), g("epsilon", 0.5), g("nut", 0.5)],
                                    dtype=torch.float32)

    def forward(self, pred: torch.Tensor, target: torch.Tensor,
                pressure_ref_weight: float = 0.1) -> torch.Tensor:
        if pred.device.type != "cuda" or target.device.type != "cuda":
            raise RuntimeError("mignn WeightedMSELoss runs on ROCm devices only (no CPU path)")
        if pred.dim() != 2 or target.shape != pred.shape:
            raise RuntimeError(f"pred {tuple(pred.shape)} / target {tuple(target.shape)} mismatch")
        if self.use_fieldwise:   # read at call time, like the reference (:199-231)
            g = self.field_weights.get
            w = [g("U", 1.0)] * 3 + [g("p", 1.0), g("k", 0.5), g("epsilon", 0.5), g("nut", 0.5)]
        else:
            w = self.weights.tolist()
        return _T.weighted_mse(pred, target, w, pressure_ref_weight if self.use_fieldwise else 0.0,
                               self.use_fieldwise)
