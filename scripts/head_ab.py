"""Same-box A/B of the fused output head (mignn_mlp_head, H = HA_H (128), out 7) on
HA_N rows (default the headline's 10M): the product library against variant
builds of mlp_f16x3.hip (HA_LIBS name=path,...; scripts/build_variant.sh),
one prepared image, one output buffer for the timing, outputs compared
bitwise; HIP events, interleaved rounds, median.  Prints one JSON object."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("HA_N", "10000000"))
H, OUT = int(os.environ.get("HA_H", "128")), 7
g = torch.Generator(device=dev).manual_seed(0)
x = torch.relu(torch.randn(n, H, device=dev, generator=g))
w = [torch.randn(H, H, device=dev, generator=g) * 0.08, torch.randn(H, H, device=dev, generator=g) * 0.08,
     torch.randn(H // 2, H, device=dev, generator=g) * 0.08, torch.randn(OUT, H // 2, device=dev, generator=g) * 0.1]
b = [torch.randn(H, device=dev, generator=g) * 0.05, torch.randn(H, device=dev, generator=g) * 0.05,
     torch.randn(H // 2, device=dev, generator=g) * 0.05, torch.randn(OUT, device=dev, generator=g) * 0.05]
L = _lib.lib()
P = _lib.ptr
st = _lib.stream()
nb = L.mignn_mlp_head_prep_bytes(H)
img = torch.empty(nb, dtype=torch.uint8, device=dev)
_lib.check(L.mignn_mlp_head_prep(P(w[0]), P(b[0]), P(w[1]), P(b[1]), P(w[2]), P(b[2]), P(w[3]), P(b[3]), H,
                                 OUT, P(img), nb, st), "prep")
libs = {"product": L}
for item in [v for v in os.environ.get("HA_LIBS", "").split(",") if v]:
    name, path = item.split("=")
    libs[name] = _lib._load(path, _lib.SIGNATURES)
out = torch.empty(n, OUT, device=dev)


def run(VL, o):
    _lib.check(VL.mignn_mlp_head(P(x), H, n, H, P(img), OUT, P(o), OUT, None, st), "head")


res = {"n": n, "h": H, "bitwise_vs_product": {}}
ref = torch.empty_like(out)
run(L, ref)
torch.cuda.synchronize()
for k, VL in libs.items():
    o = torch.full_like(out, float("nan"))
    run(VL, o)
    torch.cuda.synchronize()
    res["bitwise_vs_product"][k] = bool(torch.equal(o, ref))
reps = int(os.environ.get("HA_REPS", "7"))
times = {k: [] for k in libs}
for rnd in range(reps + 1):
    for k, VL in libs.items():
        run(VL, out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(VL, out)
        e1.record()
        e1.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1) / 3)
res["ms"] = {k: round(statistics.median(v), 4) for k, v in times.items()}
flops = 3 * 2 * n * (2 * H * H + H * H // 2 + H // 2 * 32)
res["f16_mfma_tflops"] = {k: round(flops / (v * 1e-3) / 1e12, 1) for k, v in res["ms"].items()}
print(json.dumps(res))
