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
    # edge pencils may be narrower (ceil division)
    ids = torch.arange(n, device=dev)
    i, j, k = ids % nx, (ids // nx) % ny, ids // (nx * ny)
    npi = (nx + bi - 1) // bi
    key = ((((j // bj) * npi + (i // bi)) * nz + k) * bj + (j % bj)) * bi + (i % bi)
    pos = torch.empty_like(ids)
    pos[torch.argsort(key)] = ids
    ei = pos[ei]
if os.environ.get("KB_PANEL"):
    # 4x4x4-cell tiles; panels of PxP tile columns swept along k, tiles of a
    # panel's k-level consecutive (locality experiment)
    # KB_PANEL="P" (P x P tile columns) or "PI,PJ"
    pv = [int(v) for v in os.environ["KB_PANEL"].split(",")]
    pi_, pj_ = (pv[0], pv[0]) if len(pv) == 1 else (pv[0], pv[1])
    ids = torch.arange(n, device=dev)
    i, j, k = ids % nx, (ids // nx) % ny, ids // (nx * ny)
    ti, tj, tk = i // 4, j // 4, k // 4
    ntk = (nz + 3) // 4
    npi = ((nx + 3) // 4 + pi_ - 1) // pi_
    key = (((((tj // pj_) * npi + ti // pi_) * ntk + tk) * pj_ + tj % pj_) * pi_ + ti % pi_) * 64 \
        + (k % 4) * 16 + (j % 4) * 4 + i % 4
    pos = torch.empty_like(ids)
    pos[torch.argsort(key, stable=True)] = ids
    ei = pos[ei]
if os.environ.get("KB_MORTON"):
    # relabel nodes in Morton (Z-curve) order of their grid cell (locality experiment)
    ids = torch.arange(n, device=dev)
    c = [ids % nx, (ids // nx) % ny, ids // (nx * ny)]

    def spread(v):
        v = v.to(torch.int64)
        out = torch.zeros_like(v)
        for bit in range(11):
            out |= ((v >> bit) & 1) << (3 * bit)
        return out
    key = spread(c[0]) | (spread(c[1]) << 1) | (spread(c[2]) << 2)
    pos = torch.empty_like(ids)
    pos[torch.argsort(key, stable=True)] = ids
    ei = pos[ei]
if os.environ.get("KB_BLOCK"):
    # relabel: 4x4x4 cell blocks in lexicographic block order, cells of a block consecutive
    bs = int(os.environ["KB_BLOCK"])
    ids = torch.arange(n, device=dev)
    i, j, k = ids % nx, (ids // nx) % ny, ids // (nx * ny)
    nbi, nbj = (nx + bs - 1) // bs, (ny + bs - 1) // bs
    key = (((k // bs) * nbj + j // bs) * nbi + i // bs) * (bs ** 3) + ((k % bs) * bs + j % bs) * bs + i % bs
    pos = torch.empty_like(ids)
    pos[torch.argsort(key, stable=True)] = ids
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
csum0 = [float(t.double().sum()) for t in (X, W, csr.ew, csr.col, csr.row_ptr)]
L = _lib.diag_lib()
P = _lib.ptr
st = _lib.stream()


def gcn(flags):
    _lib.check(L.mignn_diag_gcn_layer(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H, P(W),
                                 P(b), P(sc), P(sh), flags, P(Y), H, st), "gcn")


XFLAGS = int(os.environ.get("KB_XFLAGS", "0"))


def gcn16(flags):
    flags |= XFLAGS
    _lib.check(L.mignn_diag_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                       P(W), P(b), P(sc), P(sh), flags, P(Y), H, st), "gcn16")


def agg(_):
    _lib.check(L.mignn_gcn_aggregate(P(csr.row_ptr), P(csr.col), P(csr.dinv), P(X), H, 0, n, H,
                                     P(Y), H, st), "agg")


def lin(flags):
    _lib.check(L.mignn_diag_linear(P(X), H, n, H, None, 0, 0, P(W), H, P(b), None, 0, None, None,
                              flags, P(Y), H, st), "lin")


HW = [(torch.randn(o, i, device=dev, generator=g) / i ** 0.5) for o, i in
      [(H, H), (H, H), (H // 2, H), (7, H // 2)]]
HB = [torch.randn(w.shape[0], device=dev, generator=g) * 0.1 for w in HW]
HIMG = torch.empty(L.mignn_mlp_head_prep_bytes(H), dtype=torch.uint8, device=dev)
_lib.check(L.mignn_mlp_head_prep(*(P(t) for wb in zip(HW, HB) for t in wb), H, 7, P(HIMG),
                                 HIMG.numel(), st), "prep")
HOUT = torch.empty(n, 7, device=dev)


def head16(_):
    _lib.check(L.mignn_mlp_head(P(X), H, n, H, P(HIMG), 7, P(HOUT), 7, None, st), "head")


def headdiag(mode):
    _lib.check(L.mignn_diag_mlp_head(mode, P(X), n, P(HIMG), P(HOUT), st), "headdiag")


def head32(_):
    from mignn.gnn_model import linear
    h1 = linear(X, HW[0], HB[0], relu=True, out=Y)
    h2 = linear(h1, HW[1], HB[1], relu=True)
    h3 = linear(h2, HW[2], HB[2], relu=True)
    linear(h3, HW[3], HB[3], out=HOUT)


L0COEF = torch.randn(H, 8, device=dev, generator=g) * 0.1
X0 = x0.contiguous()


def layer0(_):
    _lib.check(L.mignn_gcn_layer0_coords(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X0), 3, 3, 0, n,
                                         P(L0COEF), H, P(Y), H, st), "layer0")


def fill(_):
    Y.fill_(1.0)


def readsum(_):
    torch.sum(X, dim=0, out=SUMOUT)


SUMOUT = torch.empty(H, device=dev)


def layer0diag(mode):
    _lib.check(L.mignn_diag_gcn_layer0(mode, P(csr.row_ptr), P(csr.col), P(csr.ew), P(X0), n,
                                       P(L0COEF), P(Y), st), "layer0diag")


def copy(_):
    Y.copy_(X)


def diag(mode_blocks):
    mode, blocks = mode_blocks
    _lib.check(L.mignn_diag_gather(mode, P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), n, nx, ny,
                                   nz, blocks, P(Y), st), "diag")


cases = {
    "gcn_full": (gcn, 15), "gcn16_full": (gcn16, 15), "gcn16_interleaved": (gcn16, 15 | 65536), "gcn16_prio_cons": (gcn16, 15 | 131072), "gcn16_prio_prod": (gcn16, 15 | 262144), "gcn16_dma_late": (gcn16, 15 | 524288),
    "gcn16_no_produce": (gcn16, 15 | 256),
    "gcn16_no_mfma": (gcn16, 15 | 512), "gcn16_no_ext": (gcn16, 15 | 4096),
    "gcn16_no_tables_ext": (gcn16, 15 | 4096 | 16384),
    "gcn16_no_tables_ext_local": (gcn16, 15 | 4096 | 16384 | 8192),
    "gcn16_no_local": (gcn16, 15 | 8192), "gcn16_no_ext_local": (gcn16, 15 | 4096 | 8192),
    "gcn16_only_dma": (gcn16, 15 | 256 | 512), "gcn_no_mfma": (gcn, 15 | 512), "gcn_no_gather": (gcn, 15 | 256),
    "gcn_xmaj": (gcn, 15 | 1024), "gcn_xmaj_no_mfma": (gcn, 15 | 1024 | 512),
    "layer0": (layer0, 0), "layer0_no_gather": (layer0diag, 1), "layer0_no_store": (layer0diag, 2),
    "layer0_neither": (layer0diag, 3), "layer0_onerole": (layer0diag, 4), "head16": (head16, 0), "head16_no_xload": (headdiag, 1), "head16_no_mfma": (headdiag, 2),
    "head16_valu_only": (headdiag, 3), "head16_prio": (headdiag, 4), "head16_w12": (headdiag, 5), "head32(4 launches)": (head32, 0),
    "gcn_aggregate_only(simple)": (agg, 0), "linear_rows": (lin, 9),
    "linear_no_mfma": (lin, 9 | 512), "linear_no_load": (lin, 9 | 256), "copy(torch)": (copy, 0), "fill(torch)": (fill, 0), "colsum_read(torch)": (readsum, 0),
    "diag_csr_gather": (diag, (0, 0)), "diag_csr_gather_g2048": (diag, (0, 2048)),
    "diag_stencil_gather": (diag, (1, 0)), "diag_stencil_gather_g2048": (diag, (1, 2048)),
    "diag_copy": (diag, (2, 0)), "diag_copy_nt": (diag, (2 | 8, 0)),
    "diag_tilecopy": (diag, (3, 0)), "diag_tilecopy_nt": (diag, (3 | 8, 0)),
    "diag_csr_remap": (diag, (0 | 4, 0)), "diag_csr_nt": (diag, (0 | 8, 0)),
    "diag_csr_remap_nt": (diag, (0 | 4 | 8, 0)), "diag_stencil_remap": (diag, (1 | 4, 0)),
    "diag_stencil_nt": (diag, (1 | 8, 0)), "diag_stencil_remap_nt": (diag, (1 | 4 | 8, 0)),
}
if os.environ.get("KB_ONLY"):
    cases = {k: v for k, v in cases.items() if any(t in k for t in os.environ["KB_ONLY"].split(","))}
def clock_mhz(blocks=1024, iters=200000):
    buf = torch.zeros(2 * blocks, dtype=torch.int64, device=dev)
    _lib.check(L.mignn_diag_clock(blocks, iters, P(buf), st), "clock")
    torch.cuda.synchronize()
    b = buf.view(blocks, 2).double().cpu()
    return round(float((b[:, 0] / b[:, 1]).median() * 100.0), 1)


clock_before = clock_mhz()
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
res["clock_mhz_before_after"] = [clock_before, clock_mhz()]
if os.environ.get("KB_TRACE"):
    buf = torch.zeros(8 * 64 * 8, dtype=torch.int64, device=dev)
    _lib.check(L.mignn_diag_set_trace_f16x3(P(buf)), "trace")
    gcn16(15 | 2048 | int(os.environ.get("KB_TRACE_FLAGS", "0")))
    torch.cuda.synchronize()
    _lib.check(L.mignn_diag_set_trace_f16x3(None), "trace")
    t = buf.view(8, 64, 8).cpu().double()
    d = {"p_tables_ext_issue": t[:, 1:60, 1] - t[:, 1:60, 0],
         "p_quad0": t[:, 1:60, 2] - t[:, 1:60, 1],
         "p_quad1": t[:, 1:60, 3] - t[:, 1:60, 2],
         "p_barrier_wait": t[:, 2:61, 0] - t[:, 1:60, 3],
         "c_start_to_spin_done": t[:, 1:60, 4] - t[:, 0:59, 7],
         "c_dma_issue": t[:, 1:60, 5] - t[:, 1:60, 4],
         "c_mfma": t[:, 1:60, 6] - t[:, 1:60, 5],
         "c_epilogue": t[:, 1:60, 7] - t[:, 1:60, 6],
         "step": t[:, 2:61, 0] - t[:, 1:60, 0]}
    res["trace_cycles_median"] = {k: float(v.median()) for k, v in d.items()}
if os.environ.get("KB_CHECK_HEAD"):
    headdiag(int(os.environ.get("KB_CHECK_HEAD_MODE", "0"))) if os.environ.get("KB_CHECK_HEAD_MODE") else head16(0)
    torch.cuda.synchronize()
    rows = torch.randint(0, n, (8192,), generator=torch.Generator().manual_seed(5)).to(dev)
    h = X[rows].double()
    for i, (w, bb) in enumerate(zip(HW, HB)):
        h = h @ w.double().t() + bb.double()
        h = h.clamp_min(0) if i < 3 else h
    res["check_head"] = {"max_err": (HOUT[rows].double() - h).abs().max().item(),
                         "max_ref": h.abs().max().item()}
if os.environ.get("KB_CHECK"):
    # fresh outputs: the fp32 kernel into zeros, the f16x3 kernel into NaNs; fp64
    # reference on 4096 sampled rows (CSR on the CPU)
    Y32 = torch.zeros_like(X)
    _lib.check(L.mignn_diag_gcn_layer(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H, P(W),
                                 P(b), P(sc), P(sh), 15, P(Y32), H, st), "gcn")
    Y16 = torch.full_like(X, float("nan"))
    _lib.check(L.mignn_diag_gcn_layer_f16x3(P(csr.row_ptr), P(csr.col), P(csr.ew), P(X), H, 0, n, H,
                                       P(W), P(b), P(sc), P(sh),
                                       15 | int(os.environ.get("KB_CHECK_FLAGS", "0")), P(Y16), H, st),
               "gcn16")
    torch.cuda.synchronize()
    rows = torch.randint(0, n, (4096,), generator=torch.Generator().manual_seed(5))
    rp = csr.row_ptr.cpu().long()
    colc = csr.col.cpu().long()
    ewc = csr.ew.cpu().double()
    Xd = X.double()
    ref = []
    for r in rows.tolist():
        e = slice(int(rp[r]), int(rp[r + 1]))
        a = (ewc[e].to(dev)[:, None] * Xd[colc[e].to(dev)]).sum(0)
        ref.append(a)
    A = torch.stack(ref)
    rr = rows.to(dev)
    Yr = ((Xd[rr] + b.double() + A @ W.double().t()) * sc.double() + sh.double()).clamp_min(0)
    csum1 = [float(t.double().sum()) for t in (X, W, csr.ew, csr.col, csr.row_ptr)]
    bad = (Y32.abs() > 100).any(1).nonzero().flatten()[:8].tolist()
    res["check_inputs_unchanged"] = csum0 == csum1
    res["check_bad_rows"] = bad
    if bad:
        r = bad[0]
        e = slice(int(csr.row_ptr[r]), int(csr.row_ptr[r + 1]))
        res["check_bad_row0"] = {"cols": csr.col[e].tolist(), "ew": csr.ew[e].tolist(),
                                 "y32": Y32[r, :4].tolist()}
    res["check"] = {"f32_vs_ref_max": (Y32[rr].double() - Yr).abs().max().item(),
                    "f16x3_vs_ref_max": (Y16[rr].double() - Yr).abs().max().item(),
                    "f16x3_vs_f32_max": (Y16 - Y32).abs().max().item(),
                    "f16x3_nan_rows": int(torch.isnan(Y16).any(1).sum().item()),
                    "f32_max": Y32.abs().max().item(), "X_max": X.abs().max().item()}
print(json.dumps({"grid": [nx, ny, nz], "H": H, "ms": res}))
