"""LDS-DMA destination bounds of the shipped kernels (round 5):
every global_load_lds_dwordx4 in the diag build checks that its 1 KiB
destination ends inside the issuing kernel's static LDS allocation
(MIGNN_DMA_BOUND, csrc/common.hpp; __builtin_amdgcn_groupstaticsize) and
records a violation in its translation unit's word (mignn_diag_dma_oob_*).
This runs the model forwards that reach every LDS-DMA kernel -- the window
GCN kernels (H = 64: two workgroups per CU; 128, with and without the
row codes of layers 0 / 1), the ring kernel (H = 64: two
per CU), the producer / consumer kernel, the fused GAT kernel (two 4-wave
blocks per CU), the fused GIN and TransformerConv kernels and the split GEMM
-- through the diag build, reads the five words, and compares every output
with the product build's (bitwise: same kernels, same launches).
Prints one JSON object."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import FlowGNN, _lib  # noqa: E402
from mignn.synthetic import grid_graph, seeded_state_dict  # noqa: E402

dev = torch.device("cuda", 0)
UNITS = ("agg", "ring", "win", "pc", "gemm")
CASES = [  # (layer type, hidden, GCN kernel, mesh)
    ("GCN", 64, "win", (64, 48, 40)), ("GCN", 128, "win", (64, 48, 40)),
    ("GCN", 128, "win-rows", (64, 48, 40)),
    ("GCN", 64, "ring", (64, 48, 40)), ("GCN", 128, "pc", (64, 48, 40)),
    ("GAT", 128, "auto", (64, 48, 40)), ("GAT", 64, "auto", (64, 48, 40)),
    ("GIN", 256, "auto", (48, 40, 32)), ("Transformer", 256, "auto", (48, 40, 32)),
]


def words(D, clear=True):
    out = {}
    for u in UNITS:
        w = ctypes.c_uint(0)
        _lib.check(getattr(D, f"mignn_diag_dma_oob_{u}")(ctypes.addressof(w), 1 if clear else 0), u)
        out[u] = int(w.value)
    return out


def forward(lt, H, kern, dims, use_diag):
    _lib._lib = _lib.diag_lib() if use_diag else None
    m = FlowGNN(input_dim=3, output_dim=7, hidden_dim=H, num_layers=3, layer_type=lt, dropout=0.0)
    m.load_state_dict(seeded_state_dict(m.state_dict(), seed=11))
    m = m.to(dev).eval()
    m.reorder = "1"
    m.gcn_kernel = kern.split("-")[0]
    m.gcn_codes = kern != "win-rows"     # win: layers 0 / 1 through the row codes
    x, ei = grid_graph(*dims, device=dev)
    with torch.no_grad():
        y = m(x, ei)
    torch.cuda.synchronize()
    return y


D = _lib.diag_lib()
words(D)
res = {"cases": []}
for lt, H, kern, dims in CASES:
    yd = forward(lt, H, kern, dims, True)
    w = words(D)
    yp = forward(lt, H, kern, dims, False)
    res["cases"].append({"layer": lt, "H": H, "gcn_kernel": kern, "mesh": list(dims),
                         "dma_oob": w, "diag_equals_product": bool(torch.equal(yd, yp))})
    print(json.dumps(res["cases"][-1]), file=sys.stderr, flush=True)
_lib._lib = None
res["all_in_bounds"] = all(not any(c["dma_oob"].values()) for c in res["cases"])
print(json.dumps(res), flush=True)
