"""Generate tests/golden/train.npz: one training step of the reference's own
FlowGNN + WeightedMSELoss (SURVEY.md §8f-3 parity fixtures), GCN, GIN, GAT and Transformer (edge_attr=None).

Runs ONLY in the build container (/root/reference): like make_golden.py it
injects the CPU oracle's PyG-named classes as `torch_geometric.nn` and runs
the reference's gnn_model.FlowGNN in model.train() (batch-statistics BN,
running-stat updates) with dropout = 0 (the mask RNG is not comparable
across implementations; dropout is tested separately), the loss of
train.py:352-363 (normalization.WeightedMSELoss, fieldwise, prw 0.1), and
loss.backward().  Saved per configuration (data only):

  <cfg>/sd/<key>          the state_dict before the step
  <cfg>/target            float32 [N, 7] seeded targets
  <cfg>/out32, out64      forward output (fp32 run / fp64 run of the same model)
  <cfg>/loss32, loss64
  <cfg>/grad32/<param>, grad64/<param>
  <cfg>/bn/<i>/running_mean|running_var|num_batches_tracked   after the step
  <cfg>/elementwise_loss32, <cfg>/elementwise_grad32/<param>  use_fieldwise=False
                          (first configuration only)
fp64 values are stored rounded to float32.

Graph: the reference-built train-path BFS graph (bfs_graphs.npz).

Usage:  python tests/golden/make_train_fixture.py
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gnn-bfs-rans_amd"))
sys.path.insert(0, HERE)

from make_golden import _inject_pyg  # noqa: E402
from mignn.synthetic import seeded_state_dict  # noqa: E402

WEIGHTS = {"U": 1.0, "p": 3.0, "k": 0.5, "epsilon": 0.5, "nut": 0.5}   # train.py:352-360

CONFIGS = {
    "c1_gcn_h64_l2": dict(hidden_dim=64, num_layers=2),
    "c2_gcn_h128_l4": dict(hidden_dim=128, num_layers=4),
    "gcn_h256_l2": dict(hidden_dim=256, num_layers=2),
    "gin_h64_l2": dict(hidden_dim=64, num_layers=2, layer_type="GIN"),
    "gin_h128_l3": dict(hidden_dim=128, num_layers=3, layer_type="GIN"),
    "gat_h64_l2": dict(hidden_dim=64, num_layers=2, layer_type="GAT"),
    "gat_h128_l3": dict(hidden_dim=128, num_layers=3, layer_type="GAT"),
    # TransformerConv: edge_attr=None (with edge_attr the reference raises, §8 a-8)
    "tf_h64_l2": dict(hidden_dim=64, num_layers=2, layer_type="Transformer"),
    "tf_h128_l2": dict(hidden_dim=128, num_layers=2, layer_type="Transformer"),
}


def main():
    _inject_pyg()
    sys.path.insert(0, REF)
    from gnn_model import FlowGNN
    from normalization import WeightedMSELoss

    g = np.load(os.path.join(HERE, "bfs_graphs.npz"))
    x = torch.from_numpy(g["train_x"])
    ei = torch.from_numpy(g["train_ei"].astype(np.int64))
    ea = torch.from_numpy(g["train_ea"])
    out = {}
    for ci, (name, cfg) in enumerate(CONFIGS.items()):
        gen = torch.Generator().manual_seed(500 + ci)
        target = torch.randn((x.shape[0], 7), generator=gen)
        kw = dict(cfg)
        kw.setdefault("layer_type", "GCN")
        model = FlowGNN(input_dim=3, output_dim=7, use_edge_attr=True,
                        dropout=0.0, use_batch_norm=True, **kw)
        sd = seeded_state_dict(model.state_dict(), seed=300 + ci, scale="uniform")
        for k, v in sd.items():
            out[f"{name}/sd/{k}"] = v.numpy().copy()
        out[f"{name}/target"] = target.numpy()
        out[f"{name}/cfg"] = np.array(json.dumps(cfg))
        for dt, tag in ((torch.float32, "32"), (torch.float64, "64")):
            model.load_state_dict(sd)
            model.to(dt).train()
            crit = WeightedMSELoss(field_weights=WEIGHTS, use_fieldwise=True,
                                   pressure_ref_weight=0.1)
            model.zero_grad()
            y = model(x.to(dt), ei, None if kw["layer_type"] == "Transformer" else ea.to(dt))
            loss = crit(y, target.to(dt), pressure_ref_weight=0.1)
            loss.backward()
            # fp64 results stored rounded to float32 (fixture size)
            out[f"{name}/out{tag}"] = y.detach().float().numpy().copy()
            out[f"{name}/loss{tag}"] = np.array(loss.item())
            for pn, p in model.named_parameters():
                out[f"{name}/grad{tag}/{pn}"] = p.grad.float().numpy().copy()
            if tag == "32":
                for i, bn in enumerate(model.batch_norms):
                    m = bn.module
                    # copies: the next load_state_dict writes these buffers in place
                    out[f"{name}/bn/{i}/running_mean"] = m.running_mean.numpy().copy()
                    out[f"{name}/bn/{i}/running_var"] = m.running_var.numpy().copy()
                    out[f"{name}/bn/{i}/num_batches_tracked"] = m.num_batches_tracked.numpy().copy()
            print(f"{name} fp{tag}: loss {loss.item():.8f}")
        if ci != 0:
            continue
        # element-weighted variant (use_fieldwise=False), first configuration
        model.load_state_dict(sd)
        model.float().train()
        model.zero_grad()
        crit = WeightedMSELoss(field_weights=WEIGHTS, use_fieldwise=False)
        loss = crit(model(x, ei, ea), target)
        loss.backward()
        out[f"{name}/elementwise_loss32"] = np.array(loss.item())
        for pn, p in model.named_parameters():
            out[f"{name}/elementwise_grad32/{pn}"] = p.grad.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "train.npz"), **out)
    print("wrote", os.path.join(HERE, "train.npz"))


if __name__ == "__main__":
    main()
