"""Aggregation kernels at the BASELINE leg sizes: batched (default) vs the
entry-at-a-time kernels (mignn_diag_set_agg_legacy), HIP-event timed, with
algorithmic bytes per launch.  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402

if os.environ.get("AGG_LIB"):       # an alternative build of the library (experiments)
    _lib.LIB_PATH = os.path.abspath(os.environ["AGG_LIB"])
from mignn.gnn_model import build_csr, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
L, P = _lib.lib(), _lib.ptr
res = {}


def timeit(fn, reps=int(os.environ.get("AGG_REPS", "5"))):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def ab(name, fn, nbytes):
    out = {}
    for legacy in (1, 0):
        L.mignn_diag_set_agg_legacy(legacy)
        t = timeit(fn)
        out["legacy_ms" if legacy else "batched_ms"] = round(t, 4)
    L.mignn_diag_set_agg_legacy(0)
    out["algorithmic_GB"] = round(nbytes / 1e9, 3)
    out["batched_GBps"] = round(nbytes / out["batched_ms"] / 1e6, 1)
    res[name] = out
    print(name, out, file=sys.stderr, flush=True)


CASES = [("transformer_h256_10M", (250, 200, 200), 256, "tf"),
         ("gin_sum_h256_12.6M", (500, 400, 63), 256, "sum"),
         ("gat_h128_1M", (100, 100, 100), 128, "gat"),
         ("transformer_h128_1M", (100, 100, 100), 128, "tf")]
# AGG_LOCAL=1: the 10M-class cases again in the engine's locality order (the
# order the model runs them in)
if os.environ.get("AGG_LOCAL"):
    CASES = [(n + "_local", d, h, k) for n, d, h, k in CASES[:2]]
for name, dims, h, kind in CASES:
    x0, ei = grid_graph(*dims, device=dev)
    n = x0.shape[0]
    E = ei.shape[1]
    mode = _lib.CSR_ONE_SELF_LOOP if kind == "gat" else _lib.CSR_VERBATIM
    inv = locality_order(x0, ei)[1] if name.endswith("_local") else None
    csr = build_csr(ei, n, mode, relabel=inv)
    del inv
    del ei
    nnz = E + (n if kind == "gat" else 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, h, device=dev, generator=g)
    st = _lib.stream(dev)
    if kind == "sum":
        out = torch.empty(n, h, device=dev)
        fn = lambda: _lib.check(L.mignn_sum_aggregate(P(csr.row_ptr), P(csr.col), P(x), h, 1.0, 0, n, h,  # noqa: E731
                                                      P(out), h, st), "sum")
        nbytes = 4 * (2 * n * h + (n + 1) + nnz)
    elif kind == "gat":
        out = torch.empty(n, 4 * h, device=dev)
        lg = torch.randn(n, 8, device=dev, generator=g)
        fn = lambda: _lib.check(L.mignn_gat_aggregate(P(csr.row_ptr), P(csr.col), P(lg), P(x), h, 0, n, h, 4,  # noqa: E731
                                                      0.2, P(out), 4 * h, st), "gat")
        nbytes = 4 * (n * h + 8 * n + 4 * n * h + (n + 1) + nnz)
    else:
        K1 = 4 * h + 4
        qt = torch.randn(n, K1, device=dev, generator=g) * 0.05
        out = torch.empty(n, K1, device=dev)
        fn = lambda: _lib.check(L.mignn_transformer_aggregate(P(csr.row_ptr), P(csr.col), P(qt), K1, P(x), h, 0,  # noqa: E731
                                                              n, h, 4, h ** -0.5, P(out), K1, st), "tf")
        nbytes = 4 * (n * h + 2 * n * K1 + (n + 1) + nnz)
    ab(name, fn, nbytes)
    del x, out, csr
    torch.cuda.empty_cache()
print(json.dumps(res))
