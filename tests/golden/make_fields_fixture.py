"""Generate tests/golden/fields.npz: outputs of the reference's output-side
code for the native denormalisation and writers to be
checked against.  Runs ONLY in the build container (imports the reference's
normalization.py and inference.py from /root/reference; PyG stand-ins as
needed).  Saved (data only):

  fit282/<field>/mean|std         FieldNormalizer.fit on the time-282 fields
  pred/out                        a seeded float32 [n, 7] model output
  pred/<field>                    FieldNormalizer.inverse_transform of
                                  FlowGNN.predict_fields(pred/out)
                                  (gnn_model.py:199-220) with the fit282 scalers
  norm/<field>                    FieldNormalizer.transform of the fields
  of/<field>                      the text save_fields_openfoam_format writes
                                  for pred/* (uint8 bytes), time dir 'predicted'

Usage:  python tests/golden/make_fields_fixture.py
"""

import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    pyg = types.ModuleType("torch_geometric")
    data = types.ModuleType("torch_geometric.data")
    data.Data = object
    pyg.data = data
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import flowgnn_oracle as nnm   # PyG-named classes (as make_golden.py)
    pyg.nn = nnm
    sys.modules.update({"torch_geometric": pyg, "torch_geometric.data": data,
                        "torch_geometric.nn": nnm})
    sys.path.insert(0, REF)
    from normalization import FieldNormalizer
    from inference import save_fields_openfoam_format
    mesh = np.load(os.path.join(HERE, "mesh.npz"))
    f282 = {k.split("/", 1)[1]: mesh[k] for k in mesh.files if k.startswith("field282/")}

    fn = FieldNormalizer()
    fn.fit(f282)
    out = {}
    for k, sc in fn.scalers.items():
        out[f"fit282/{k}/mean"] = np.asarray(sc["mean"], dtype=np.float64)
        out[f"fit282/{k}/std"] = np.asarray(sc["std"], dtype=np.float64)
    for k, v in fn.transform(f282).items():
        out[f"norm/{k}"] = np.asarray(v)

    g = np.random.default_rng(7)
    n = 40
    y = g.normal(size=(n, 7)).astype(np.float32)
    y[0] = 0.0
    y[1, 3] = -0.0
    y[2, :3] = [1e-30, -3.5e7, 123456.789]
    out["pred/out"] = y
    t = torch.from_numpy(y)
    fields = {"U": t[:, :3], "p": t[:, 3:4], "k": t[:, 4:5], "epsilon": t[:, 5:6],
              "nut": t[:, 6:7]}
    fields = {k: v.numpy() for k, v in fields.items()}
    den = fn.inverse_transform(fields)
    for k, v in den.items():
        out[f"pred/{k}"] = np.asarray(v)
    with tempfile.TemporaryDirectory() as td:
        save_fields_openfoam_format(den, td, "predicted")
        for k in ("U", "p", "k", "epsilon", "nut"):
            with open(os.path.join(td, "predicted", k), "rb") as fh:
                out[f"of/{k}"] = np.frombuffer(fh.read(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "fields.npz"), **out)
    print({k: (v.shape, v.dtype) for k, v in out.items() if not k.startswith("of/")})


if __name__ == "__main__":
    main()
