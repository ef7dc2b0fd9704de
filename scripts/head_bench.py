"""Output-head timing at H = 256 (round 3): the fused head256 kernel
(mignn_mlp_head, h = 256) vs the four launches of FlowGNN._output_mlp it
replaces (MIGNN_FUSED256=0 path), on HB_N rows (default configs[4]'s per-GPU
12.6M); HIP events, interleaved rounds; max |fused - launches| / max |ref|."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import FlowGNN  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("HB_N", "12600000"))
H = 256
torch.manual_seed(0)
model = FlowGNN(hidden_dim=H, num_layers=1).to(dev).eval()
assert model.precision == "f16x3"
x = torch.randn(n, H, device=dev)
tmp = torch.empty_like(x)
KINDS = ("fused", "launches")
outs = {k: torch.full((n, model.output_dim), float("nan"), device=dev) for k in KINDS}


def setk(kind):
    model.fused256 = "0" if kind == "launches" else "1"


def run(kind, out):
    setk(kind)
    xin = x.clone() if kind == "launches" else x      # the launch path reuses x as scratch
    model._output_mlp(xin, tmp, out)


with torch.no_grad():
    for k, o in outs.items():
        run(k, o)
    torch.cuda.synchronize()
    ref = outs["launches"]
    res = {"n": n, "h": H, "out_dim": model.output_dim,
           "max_rel_diff": {k: ((outs[k] - ref).abs().max() / ref.abs().max()).item()
                            for k in KINDS}}
    reps = int(os.environ.get("HB_REPS", "5"))
    times = {k: [] for k in outs}
    xs = x.clone()
    for rnd in range(reps + 1):
        for k, o in outs.items():
            setk(k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                model._output_mlp(xs, tmp, o)
            e1.record()
            e1.synchronize()
            if rnd > 0:
                times[k].append(e0.elapsed_time(e1) / 3)
    res["ms"] = {k: round(statistics.median(v), 4) for k, v in times.items()}
    by = n * H * 4 + n * model.output_dim * 4
    res["frac_hbm_fused"] = round(by / (res["ms"]["fused"] * 1e-3) / 8e12, 4)
    res["f16_tflops_fused"] = round(3 * 2 * n * (2 * H * H + H * H // 2) / (res["ms"]["fused"] * 1e-3)
                                    / 1e12, 1)
print(json.dumps(res), flush=True)
