"""Graph-setup timing on the bench mesh (250x200x200, 10M nodes): the column
order and the CSR build (mignn_csr_build_gcn, relabelled) and the window
plan, HIP events, median of 5; bitwise check of the CSR against a second
build.  CB_LIB: time a variant build instead.  Prints one JSON object."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr, locality_order  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

if os.environ.get("CB_LIB"):   # a variant build of libmignn.so in place of the product
    import ctypes
    _h = ctypes.CDLL(os.environ["CB_LIB"])   # (an older build: the symbols it has)
    _lib._lib = _lib._load(os.environ["CB_LIB"],
                           {k: v for k, v in _lib.SIGNATURES.items() if hasattr(_h, k)})
dev = torch.device("cuda", 0)
pos, ei = grid_graph(250, 200, 200, device=dev)
n = pos.shape[0]


def t(f, reps=5):
    f()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1))
    return round(statistics.median(out), 4)


res = {}
_, inv, info = locality_order(pos, ei, cols=True)
res["order_cols_ms"] = t(lambda: locality_order(pos, ei, cols=True))
res["csr_ms"] = t(lambda: build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv))
a = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
b = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP, relabel=inv)
res["csr_deterministic"] = bool(torch.equal(a.col, b.col) and torch.equal(a.ew, b.ew)
                                and torch.equal(a.row_ptr, b.row_ptr))
import hashlib  # noqa: E402
res["csr_sha1"] = hashlib.sha1(a.row_ptr.cpu().numpy().tobytes() + a.col.cpu().numpy().tobytes()
                               + a.ew.cpu().numpy().tobytes()).hexdigest()
a.order_info = info
L = _lib.lib()
for H in (128, 64):
    nb = L.mignn_gcn_win_plan_bytes(0, n, H)
    plan = torch.empty(nb, dtype=torch.uint8, device=dev)
    res[f"win_plan_ms_{H}"] = t(lambda: _lib.check(L.mignn_gcn_win_plan(
        _lib.ptr(a.row_ptr), _lib.ptr(a.col), _lib.ptr(a.ew), 0, n, H, _lib.ptr(info), _lib.ptr(plan),
        nb, None, _lib.stream()), "plan"))
print(json.dumps(res), flush=True)
