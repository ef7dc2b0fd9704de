"""Time the dense node transforms of the H = 256 layers: exact-fp32
mignn_linear vs split-fp16 mignn_linear_f16x3, per shape, with the HBM
roofline (algorithmic bytes = read A (+A2, +residual) + write C)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gnn-bfs-rans_amd"))
from mignn import _lib  # noqa: E402

if os.environ.get("GB_LIB"):                       # an alternative build (experiments)
    _lib.LIB_PATH = os.environ["GB_LIB"]
from mignn.gnn_model import f16x3_image, linear, linear_f16x3  # noqa: E402

L, P = _lib.diag_lib(), _lib.ptr

M = int(os.environ.get("GB_M", 2_000_000))
SHAPES = [  # (name, k1, k2, n, residual)
    ("gin_nn0 256->256", 256, 0, 256, False),
    ("gin_nn2 256->256 +res", 256, 0, 256, True),
    ("tf_qt 256->1024", 256, 0, 1024, False),
    ("tf_qk 256->1028", 256, 0, 1028, False),   # TransformerConv's Q~K with the score constants
    ("tf_qk 256->1040", 256, 0, 1040, False),
    ("tf_out [1028|256]->256 +res", 1028, 256, 256, True),
    ("gat_out 1024->256 +res", 1024, 0, 256, True),
    ("gat_out 512->128 +res", 512, 0, 128, True),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    only = os.environ.get("GB_ONLY", "")
    for name, k1, k2, n, has_res in SHAPES:
        if only and not any(o in name for o in only.split(",")):
            continue
        a = torch.randn(M, k1, device=dev, generator=g)
        a2 = torch.randn(M, k2, device=dev, generator=g) if k2 else None
        w = torch.randn(n, k1 + k2, device=dev, generator=g) / (k1 + k2) ** 0.5
        b = torch.randn(n, device=dev, generator=g)
        res = torch.randn(M, n, device=dev, generator=g) if has_res else None
        out = torch.empty(M, n, device=dev)
        img = f16x3_image(w)
        kw = dict(relu=True, residual=res, a2=a2, out=out)
        if os.environ.get("GB_NO32"):
            t32, c32 = float("nan"), out.clone()
        else:
            t32 = timeit(lambda: linear(a, w, b, **kw))
            c32 = out.clone()
        t16 = timeit(lambda: linear_f16x3(a, img, n, b, **kw))
        d = (out - c32).abs().max().item()
        abl = {}
        for nm, fl in (("no_A", 256), ("no_mfma", 512), ("no_store", 4096), ("no_A_mfma", 768),
                       ("only_loop", 256 | 512 | 4096)):
            flags = 1 | 8 | (2 if has_res else 0) | fl
            abl[nm] = round(timeit(lambda: L.mignn_diag_linear_f16x3(
                P(a), a.stride(0), M, k1, P(a2), a2.stride(0) if k2 else 0, k2, P(img), n, P(b),
                P(res), res.stride(0) if has_res else 0, None, None, flags, P(out), out.stride(0),
                _lib.stream())), 3)
        byts = 4 * M * (k1 + k2 + n + (n if has_res else 0))
        flops = 2 * M * (k1 + k2) * n
        print(f"{name:30s} M={M}: f32 {t32:8.3f} ms ({flops / t32 / 1e9:6.1f} TF)  "
              f"f16x3 {t16:8.3f} ms ({flops / t16 / 1e9:6.1f} TF, {byts / t16 / 1e6:6.0f} GB/s "
              f"= {byts / t16 / 1e6 / 8000:.2f} of 8 TB/s)  max|f16x3-f32| {d:.2e}  ablations {abl}",
              flush=True)
        del a, a2, w, res, out, img, c32
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
