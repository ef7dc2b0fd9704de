"""Kernel micro-benchmark on the bench graph: times individual libmignn
entry points (HIP events, one process, interleaved rounds) including the
diagnostic ablations of the fused tile kernel."""
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "gnn-bfs-rans_amd"))
import torch  # noqa: E402

from mignn import _lib  # noqa: E402
from mignn.gnn_model import build_csr  # noqa: E402
from mignn.synthetic import grid_graph  # noqa: E402

dev = torch.device("cuda", 0)
nx, ny, nz = (int(v) for v in os.environ.get("KB_GRID", "250,200,200").split(","))
H = int(os.environ.get("KB_H", "128"))
x0, ei = grid_graph(nx, ny, nz, device=dev, permute_seed=int(os.environ["KB_SHUFFLE"]) if os.environ.get("KB_SHUFFLE") else None)
n = x0.shape[0]
if os.environ.get("KB_PERM"):
    # relabel the mesh into k-pencils of BI x BJ columns (locality experiment)
    bi, bj = (int(v) for v in os.environ["KB_PERM"].split(","))
    assert nx % bi == 0 and ny % bj == 0
    ids = torch.arange(n, device=dev)
    i, j, k = ids % nx, (ids // nx) % ny, ids // (nx * ny)
    npi = nx // bi
    key = ((((j // bj) * npi + (i // bi)) * nz + k) * bj + (j % bj)) * bi + (i % bi)
    pos = torch.empty_like(ids)
    pos[torch.argsort(key)] = ids
    ei = pos[ei]
csr = build_csr(ei, n, _lib.CSR_ONE_SELF_LOOP)
del ei
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(n, H, device=dev, generator=g)
Y = torch.empty_like(X)
W = torch.randn(H, H, device=dev, generator=g) * 0.05
b = torch.randn(H, device=dev, generator=g) * 0.05
sc = torch.rand(H, device=dev, generator=g) + 0.5
sh = torch.randn(H, device=dev, generator=g) * 0.1
L = _lib.lib()
P = _lib.ptr
st = _lib.stream()


def gcn(flags):
    _lib.check(L.mignn_gcn_layer(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H, P(W),
                                 P(b), P(sc), P(sh), flags, P(Y), H, st), "gcn")


def agg(_):
    _lib.check(L.mignn_gcn_aggregate(P(csr.row_ptr), P(csr.col), P(csr.dinv), P(X), H, 0, n, H,
                                     P(Y), H, st), "agg")


def lin(flags):
    _lib.check(L.mignn_linear(P(X), H, n, H, None, 0, 0, P(W), H, P(b), None, 0, None, None,
                              flags, P(Y), H, st), "lin")


def copy(_):
    Y.copy_(X)


def diag(mode_blocks):
    mode, blocks = mode_blocks
    _lib.check(L.mignn_diag_gather(mode, P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), n, nx, ny,
                                   nz, blocks, P(Y), st), "diag")


cases = {
    "gcn_full": (gcn, 15), "gcn_no_mfma": (gcn, 15 | 512), "gcn_no_gather": (gcn, 15 | 256),
    "gcn_xmaj": (gcn, 15 | 1024), "gcn_xmaj_no_mfma": (gcn, 15 | 1024 | 512),
    "gcn_aggregate_only(simple)": (agg, 0), "linear_rows": (lin, 9),
    "linear_no_mfma": (lin, 9 | 512), "linear_no_load": (lin, 9 | 256), "copy(torch)": (copy, 0),
    "diag_csr_gather": (diag, (0, 0)), "diag_csr_gather_g2048": (diag, (0, 2048)),
    "diag_stencil_gather": (diag, (1, 0)), "diag_stencil_gather_g2048": (diag, (1, 2048)),
    "diag_copy": (diag, (2, 0)), "diag_copy_nt": (diag, (2 | 8, 0)),
    "diag_csr_remap": (diag, (0 | 4, 0)), "diag_csr_nt": (diag, (0 | 8, 0)),
    "diag_csr_remap_nt": (diag, (0 | 4 | 8, 0)), "diag_stencil_remap": (diag, (1 | 4, 0)),
    "diag_stencil_nt": (diag, (1 | 8, 0)), "diag_stencil_remap_nt": (diag, (1 | 4 | 8, 0)),
}
if os.environ.get("KB_ONLY"):
    cases = {k: v for k, v in cases.items() if any(t in k for t in os.environ["KB_ONLY"].split(","))}
times = {k: [] for k in cases}
for rnd in range(5):
    for k, (fn, fl) in cases.items():
        fn(fl)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn(fl)
        e1.record()
        e1.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1) / 3)
res = {k: round(statistics.median(v), 4) for k, v in times.items()}
print(json.dumps({"grid": [nx, ny, nz], "H": H, "ms": res}))
