"""Autograd ops of the training path over libmignn.so.

Each op is a `torch.autograd.Function` whose forward and backward are HIP
kernels (csrc/train.hip, csrc/aggregate.hip, csrc/linear.hip); PyTorch only
records the graph and owns the memory.  They compose `FlowGNN`'s
model.train() forward (gnn_model.py:159-195) so that train.py's
`loss.backward()` (train.py:177) produces every parameter gradient:

  linear            nn.Linear (input_proj :55, output_proj :90-100), optional
                    fused ReLU
  dropout           nn.Dropout / F.dropout (counter-hash mask, regenerated in
                    the backward)
  gcn_residual      x + GCNConv(x)  (:166, :184) -- aggregation first, then
                    the transform, bias and residual in one MFMA epilogue;
                    backward through the reversed-edge CSR
  gin_residual      x + GINConv(x) = x + nn((1+eps) x + sum_j x_j)  (:70-75,
                    :166, :184) -- verbatim sum aggregation, two MFMA Linears
                    (ReLU fused into the first, residual into the second);
                    backward through the reversed verbatim CSR
  gat_residual      x + GATConv(x) (:65-68, :168) -- logits GEMM, softmax
                    aggregation with attention dropout, head-mean GEMM with
                    bias + residual; backward: rows kernel (softmax state,
                    dst-logit grads) + reversed-CSR kernel (dx, src-logit grads)
  transformer_residual  x + TransformerConv(x) (:77-80, :170; edge_attr None) --
                    one [Wq;Wk;Wv] MFMA, softmax aggregation of V with
                    attention dropout (+ residual), lin_skip MFMA epilogue;
                    backward: rows kernel (dQ) + reversed-CSR kernel (dK, dV)
  bn_relu_dropout   BatchNorm (batch statistics, running-stat update) + ReLU +
                    dropout (:188-191) in one elementwise pass
  WeightedMSELoss   normalization.py:136-250 (forward and backward on device)
"""

from __future__ import annotations

import ctypes
from typing import Optional

import torch
from torch.autograd import Function

from . import _lib

P = _lib.ptr


def _st(t: torch.Tensor) -> int:
    return _lib.stream(t.device)


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if (t.is_contiguous() and t.dtype == torch.float32) else t.float().contiguous()


def _red_scratch(n: int, h: int, dev) -> torch.Tensor:
    nb = _lib.lib().mignn_train_scratch_bytes(n, h)
    return torch.empty(nb, dtype=torch.uint8, device=dev)


def gemm(a, sai, sak, b, sbk, sbj, m, n, k, out, ldc=None, residual=None, split=False):
    """out[i, j] = sum_k A(i, k) B(k, j) (+ residual) on the f32 MFMA (mignn_gemm)."""
    ldc = out.stride(0) if ldc is None else ldc
    scratch, nbytes = None, 0
    if split:   # room for mignn_gemm's split partials (<= ~1024 tiles in flight)
        tiles = -(-m // 64) * -(-n // 64)
        nbytes = (1024 // tiles + 1) * m * n * 4
        scratch = torch.empty(nbytes, dtype=torch.uint8, device=out.device)
    _lib.check(_lib.lib().mignn_gemm(
        P(a), sai, sak, P(b), sbk, sbj, m, n, k, P(residual),
        0 if residual is None else residual.stride(0), P(out), ldc, P(scratch), nbytes,
        _st(out)), "mignn_gemm")
    return out


def weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW[o, i] = sum_m dy[m, o] x[m, i]  (nn.Linear weight gradient)."""
    n, o = dy.shape
    i = x.shape[1]
    dw = torch.empty((o, i), dtype=torch.float32, device=dy.device)
    return gemm(dy, 1, dy.stride(0), x, x.stride(0), 1, o, i, n, dw, split=True)


def data_grad(dy: torch.Tensor, w: torch.Tensor, residual=None) -> torch.Tensor:
    """dx[m, i] = sum_o dy[m, o] w[o, i] (+ residual)  (nn.Linear input gradient)."""
    n, o = dy.shape
    i = w.shape[1]
    dx = torch.empty((n, i), dtype=torch.float32, device=dy.device)
    return gemm(dy, dy.stride(0), 1, w, w.stride(0), 1, n, i, o, dx, residual=residual)


_COL_CHUNK = 512   # mignn_col_sums' widest reduction (64 lanes x RED_CC columns)


def col_sums(x: torch.Tensor) -> torch.Tensor:
    n, h = x.shape
    out = torch.empty(h, dtype=torch.float32, device=x.device)
    s = _red_scratch(n, min(h, _COL_CHUNK), x.device)
    for c0 in range(0, h, _COL_CHUNK):   # wide inputs ([Q|K|V] grads): column panels
        xc = x[:, c0:c0 + _COL_CHUNK]
        _lib.check(_lib.lib().mignn_col_sums(P(xc), x.stride(0), n, xc.shape[1], P(out[c0:]),
                                             P(s), s.numel(), _st(x)), "mignn_col_sums")
    return out


def draw_seed() -> int:
    """A dropout seed from torch's (CPU) default generator, so torch.manual_seed
    makes training runs repeatable."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# ---------------------------------------------------------------------------

class _Linear(Function):
    @staticmethod
    def forward(ctx, x, w, b, relu: bool):
        from .gnn_model import linear as _mfma_linear
        x = _c(x)
        n, k = x.shape
        if k % 4 == 0 and x.stride(0) % 4 == 0:
            y = _mfma_linear(x, w, b, relu=relu)
        else:   # thin inputs (input_proj, 3 coordinates): the VALU projection
            if relu:
                raise NotImplementedError("fused ReLU on a thin Linear")
            y = torch.empty((n, w.shape[0]), dtype=torch.float32, device=x.device)
            _lib.check(_lib.lib().mignn_input_proj(
                P(x), n, k, P(w), P(b), w.shape[0], P(y), y.stride(0), _st(x)),
                "mignn_input_proj")
        ctx.relu = relu
        ctx.has_bias = b is not None
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        g = _c(gy)
        if ctx.relu:   # through the fused ReLU: g * (y > 0)
            g = _act_backward(g, y, relu=True, p=0.0, seed=0)
        dx = data_grad(g, w) if ctx.needs_input_grad[0] else None
        dw = weight_grad(g, x) if ctx.needs_input_grad[1] else None
        db = col_sums(g) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None


def _act_backward(dout, y, relu: bool, p: float, seed: int) -> torch.Tensor:
    """d/dy of drop_p(relu?(y)) given the forward's y (no BN)."""
    n, h = dout.shape
    dz = torch.empty_like(dout)
    _lib.check(_lib.lib().mignn_bn_act_backward(
        P(dout), dout.stride(0), P(y), y.stride(0), n, h, None, None, None, None, int(relu),
        float(p), seed, P(dz), dz.stride(0), None, None, None, 0, _st(dout)),
        "mignn_bn_act_backward")
    return dz


class _Dropout(Function):
    @staticmethod
    def forward(ctx, x, p: float, seed: int):
        x = _c(x)
        n, h = x.shape
        y = torch.empty_like(x)
        _lib.check(_lib.lib().mignn_bn_act_forward(
            P(x), x.stride(0), n, h, None, None, None, None, 0, float(p), seed, P(y),
            y.stride(0), _st(x)), "mignn_bn_act_forward")
        ctx.p, ctx.seed = p, seed
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return _act_backward(_c(gy), x, relu=False, p=ctx.p, seed=ctx.seed), None, None


class _GCNResidual(Function):
    """z = x + GCNConv(x) = x + (A x) W^T + b, A = PyG gcn_norm adjacency."""

    @staticmethod
    def forward(ctx, x, w, b, csr, csr_t):
        from .gnn_model import linear as _mfma_linear
        x = _c(x)
        n, h = x.shape
        agg = torch.empty_like(x)
        _lib.check(_lib.lib().mignn_gcn_aggregate(
            P(csr.row_ptr), P(csr.col), P(csr.dinv), P(x), x.stride(0), 0, n, h, P(agg),
            agg.stride(0), _st(x)), "mignn_gcn_aggregate")
        z = _mfma_linear(agg, w, b, residual=x)
        ctx.csr, ctx.csr_t = csr, csr_t
        ctx.save_for_backward(agg, w)
        return z

    @staticmethod
    def backward(ctx, gz):
        agg, w = ctx.saved_tensors
        g = _c(gz)
        n, h = g.shape
        db = col_sums(g)
        dw = weight_grad(g, agg)
        # dx = g + (A^T g) W: A^T = the aggregation over the reversed edges
        # with the same symmetric weights dinv_i * dinv_j
        t = torch.empty_like(g)
        csr, csr_t = ctx.csr, ctx.csr_t
        _lib.check(_lib.lib().mignn_gcn_aggregate(
            P(csr_t.row_ptr), P(csr_t.col), P(csr.dinv), P(g), g.stride(0), 0, n, h, P(t),
            t.stride(0), _st(g)), "mignn_gcn_aggregate(transpose)")
        dx = data_grad(t, w, residual=g)
        return dx, dw, db, None, None


class _GINResidual(Function):
    """z = x + GINConv(x) = x + W2 relu(W1 agg + b1) + b2,
    agg = (1 + eps) x + sum_{j -> i} x_j over edge_index as given (PyG GINConv,
    gnn_model.py:70-75; every self-loop entry adds another x_i)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, self_scale: float, csr, csr_t):
        from .gnn_model import linear as _mfma_linear
        x = _c(x)
        n, h = x.shape
        agg = torch.empty_like(x)
        _lib.check(_lib.lib().mignn_sum_aggregate(
            P(csr.row_ptr), P(csr.col), P(x), x.stride(0), float(self_scale), 0, n, h, P(agg),
            agg.stride(0), _st(x)), "mignn_sum_aggregate")
        h1 = _mfma_linear(agg, w1, b1, relu=True)
        z = _mfma_linear(h1, w2, b2, residual=x)
        ctx.self_scale, ctx.csr_t = self_scale, csr_t
        ctx.save_for_backward(agg, h1, w1, w2)
        return z

    @staticmethod
    def backward(ctx, gz):
        agg, h1, w1, w2 = ctx.saved_tensors
        g = _c(gz)
        n, h = g.shape
        db2 = col_sums(g)
        dw2 = weight_grad(g, h1)
        dh1 = _act_backward(data_grad(g, w2), h1, relu=True, p=0.0, seed=0)
        db1 = col_sums(dh1)
        dw1 = weight_grad(dh1, agg)
        # dx = g + ((1 + eps) dh1 + A^T dh1) W1   (A^T: the reversed verbatim edges;
        # the aggregation commutes with the right-multiplication by W1)
        u = torch.empty_like(dh1)
        csr_t = ctx.csr_t
        _lib.check(_lib.lib().mignn_sum_aggregate(
            P(csr_t.row_ptr), P(csr_t.col), P(dh1), dh1.stride(0), float(ctx.self_scale), 0, n,
            dh1.shape[1], P(u), u.stride(0), _st(g)), "mignn_sum_aggregate(transpose)")
        dx = data_grad(u, w1, residual=g)
        return dx, dw1, db1, dw2, db2, None, None, None


class _GATResidual(Function):
    """z = x + GATConv(x), re-associated: logits = x wlog^T ([N, 2*heads]),
    Y = softmax-aggregate(x) ([N, heads*H]), z = Y wcat^T + b + x.  wlog / wcat
    are the per-step weight images (autograd tensors built from lin.weight,
    att_src, att_dst by FlowGNN); their gradients flow back through them."""

    @staticmethod
    def forward(ctx, x, wlog, wcat, b, csr, csr_t, heads: int, slope: float, p: float,
                seed: int):
        from .gnn_model import linear as _mfma_linear
        x = _c(x)
        wlog, wcat = _c(wlog), _c(wcat)
        n, h = x.shape
        logits = _mfma_linear(x, wlog)
        y = torch.empty((n, heads * h), dtype=torch.float32, device=x.device)
        stats = torch.empty((n, 3 * heads), dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib().mignn_gat_train_forward(
            P(csr.row_ptr), P(csr.col), P(logits), P(x), x.stride(0), n, h, heads, float(slope),
            float(p), seed, P(y), y.stride(0), P(stats), _st(x)), "mignn_gat_train_forward")
        z = _mfma_linear(y, wcat, b, residual=x)
        ctx.csr, ctx.csr_t, ctx.meta = csr, csr_t, (heads, slope, p, seed)
        ctx.save_for_backward(x, logits, y, wlog, wcat, stats)
        return z

    @staticmethod
    def backward(ctx, gz):
        x, logits, y, wlog, wcat, stats = ctx.saved_tensors
        heads, slope, p, seed = ctx.meta
        g = _c(gz)
        n, h = g.shape
        db = col_sums(g)
        dwcat = weight_grad(g, y)                 # [H, heads*H]
        dy = data_grad(g, wcat)                   # [N, heads*H]
        dlog = torch.empty((n, 2 * heads), dtype=torch.float32, device=g.device)
        dxa = torch.empty_like(g)
        csr, csr_t = ctx.csr, ctx.csr_t
        _lib.check(_lib.lib().mignn_gat_train_backward(
            P(csr.row_ptr), P(csr.col), P(csr_t.row_ptr), P(csr_t.col), P(logits), P(x),
            x.stride(0), P(dy), dy.stride(0), P(y), y.stride(0), P(g), g.stride(0), n, h, heads,
            float(slope),
            float(p), seed, P(stats), P(dlog), P(dxa), dxa.stride(0), _st(g)),
            "mignn_gat_train_backward")
        dwlog = weight_grad(dlog, x)              # [2*heads, H]
        dx = data_grad(dlog, wlog, residual=dxa)  # + dlogits . wlog
        return dx, dwlog, dwcat, db, None, None, None, None, None, None


class _TransformerResidual(Function):
    """z = x + TransformerConv(x) = x + O + x ws^T + bs,
    O_i = mean_k sum_j drop(softmax_j(<Q_i,K_j>/sqrt(H))) V_j, [Q|K|V] = x wqkv^T + bqkv."""

    @staticmethod
    def forward(ctx, x, wqkv, bqkv, ws, bs, csr, csr_t, heads: int, p: float, seed: int):
        from .gnn_model import linear as _mfma_linear
        x = _c(x)
        wqkv, bqkv = _c(wqkv), _c(bqkv)
        n, h = x.shape
        qkv = _mfma_linear(x, wqkv, bqkv)                # [N, 3*heads*H]
        o = torch.empty_like(x)
        yh = torch.empty((n, heads * h), dtype=torch.float32, device=x.device)
        stats = torch.empty((n, 3 * heads), dtype=torch.float32, device=x.device)
        scale = 1.0 / float(h) ** 0.5
        _lib.check(_lib.lib().mignn_transformer_train_forward(
            P(csr.row_ptr), P(csr.col), P(qkv), qkv.stride(0), P(x), x.stride(0), n, h, heads,
            scale, float(p), seed, P(o), o.stride(0), P(yh), yh.stride(0), P(stats), _st(x)),
            "mignn_transformer_train_forward")
        z = _mfma_linear(x, ws, bs, residual=o)
        ctx.csr, ctx.csr_t, ctx.meta = csr, csr_t, (heads, scale, p, seed)
        ctx.save_for_backward(x, qkv, wqkv, ws, yh, stats)
        return z

    @staticmethod
    def backward(ctx, gz):
        x, qkv, wqkv, ws, yh, stats = ctx.saved_tensors
        heads, scale, p, seed = ctx.meta
        g = _c(gz)
        n, h = g.shape
        dbs = col_sums(g)
        dws = weight_grad(g, x)
        dqkv = torch.empty_like(qkv)
        csr, csr_t = ctx.csr, ctx.csr_t
        _lib.check(_lib.lib().mignn_transformer_train_backward(
            P(csr.row_ptr), P(csr.col), P(csr_t.row_ptr), P(csr_t.col), P(qkv), qkv.stride(0),
            P(g), g.stride(0), P(yh), yh.stride(0), n, h, heads, float(scale), float(p), seed,
            P(stats), P(dqkv),
            dqkv.stride(0), _st(g)), "mignn_transformer_train_backward")
        dbqkv = col_sums(dqkv)
        dwqkv = weight_grad(dqkv, x)
        dx = data_grad(dqkv, wqkv, residual=data_grad(g, ws, residual=g))
        return dx, dwqkv, dbqkv, dws, dbs, None, None, None, None, None


class _BNReluDropout(Function):
    """dropout(relu(BatchNorm_train(z))); bn_mod = the BatchNorm1d (running
    stats updated in place, as torch does in train mode); bn_mod None: no BN."""

    @staticmethod
    def forward(ctx, z, gamma, beta, bn_mod, p: float, seed: int):
        z = _c(z)
        n, h = z.shape
        dev = z.device
        mean = invstd = None
        if bn_mod is not None:
            if n <= 1:   # torch.nn.functional.batch_norm's training-mode check
                raise ValueError("Expected more than 1 value per channel when training, "
                                 f"got input size {torch.Size([n, h])}")
            mean = torch.empty(h, dtype=torch.float32, device=dev)
            invstd = torch.empty_like(mean)
            s = _red_scratch(n, h, dev)
            track = bn_mod.track_running_stats and bn_mod.running_mean is not None
            # momentum=None (cumulative average, e.g. swa_utils.update_bn): -1
            mom = bn_mod.momentum if bn_mod.momentum is not None else -1.0
            _lib.check(_lib.lib().mignn_bn_train_stats(
                P(z), z.stride(0), n, h, float(bn_mod.eps), float(mom), P(mean), P(invstd),
                P(bn_mod.running_mean) if track else None,
                P(bn_mod.running_var) if track else None,
                P(bn_mod.num_batches_tracked) if track else None, P(s), s.numel(), _st(z)),
                "mignn_bn_train_stats")
        y = torch.empty_like(z)
        _lib.check(_lib.lib().mignn_bn_act_forward(
            P(z), z.stride(0), n, h, P(mean), P(invstd), P(gamma), P(beta), 1, float(p), seed,
            P(y), y.stride(0), _st(z)), "mignn_bn_act_forward")
        ctx.p, ctx.seed, ctx.bn = p, seed, bn_mod is not None
        ctx.save_for_backward(z, mean, invstd, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, gy):
        z, mean, invstd, gamma, beta = ctx.saved_tensors
        g = _c(gy)
        n, h = g.shape
        dz = torch.empty_like(g)
        dgamma = dbeta = s = None
        nbytes = 0
        if ctx.bn:
            dgamma = torch.empty(h, dtype=torch.float32, device=g.device)
            dbeta = torch.empty_like(dgamma)
            s = _red_scratch(n, h, g.device)
            nbytes = s.numel()
        _lib.check(_lib.lib().mignn_bn_act_backward(
            P(g), g.stride(0), P(z), z.stride(0), n, h, P(mean), P(invstd), P(gamma), P(beta),
            1, float(ctx.p), ctx.seed, P(dz), dz.stride(0), P(dgamma), P(dbeta), P(s), nbytes,
            _st(g)), "mignn_bn_act_backward")
        return dz, dgamma, dbeta, None, None, None


class _WMSE(Function):
    @staticmethod
    def forward(ctx, pred, target, weights, prw: float, fieldwise: bool):
        pred, target = _c(pred), _c(target)
        n, ncol = pred.shape
        dev = pred.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        stats = torch.empty(1, dtype=torch.float64, device=dev)
        s = _red_scratch(n, ncol, dev)
        w = _host_floats(weights)
        _lib.check(_lib.lib().mignn_wmse_loss(
            P(pred), pred.stride(0), P(target), target.stride(0), n, ncol, w, float(prw),
            int(fieldwise), P(loss), P(stats), P(s), s.numel(), _st(pred)), "mignn_wmse_loss")
        ctx.weights, ctx.prw, ctx.fieldwise = weights, prw, fieldwise
        ctx.save_for_backward(pred, target, stats)
        return loss

    @staticmethod
    def backward(ctx, gl):
        pred, target, stats = ctx.saved_tensors
        n, ncol = pred.shape
        gl = _c(gl.reshape(()))
        dpred = torch.empty_like(pred)
        _lib.check(_lib.lib().mignn_wmse_loss_backward(
            P(pred), pred.stride(0), P(target), target.stride(0), n, ncol,
            _host_floats(ctx.weights), float(ctx.prw), int(ctx.fieldwise), P(stats), P(gl),
            P(dpred), dpred.stride(0), _st(pred)), "mignn_wmse_loss_backward")
        return dpred, None, None, None, None


def _host_floats(vals):
    """A host float[7] (ctypes arrays pass as pointers; alive for the call)."""
    return (ctypes.c_float * 7)(*[float(v) for v in vals])


# ---------------------------------------------------------------------------
# public functional surface

def linear(x, w, b=None, relu: bool = False):
    return _Linear.apply(x, w, b, relu)


def dropout(x, p: float, training: bool = True, seed: Optional[int] = None):
    if not training or p <= 0.0:
        return x
    return _Dropout.apply(x, float(p), draw_seed() if seed is None else seed)


def gcn_residual(x, w, b, csr, csr_t):
    return _GCNResidual.apply(x, w, b, csr, csr_t)


def gin_residual(x, w1, b1, w2, b2, eps: float, csr, csr_t):
    return _GINResidual.apply(x, w1, b1, w2, b2, 1.0 + float(eps), csr, csr_t)


def gat_residual(x, wlog, wcat, b, csr, csr_t, heads: int, slope: float, p: float,
                 seed: Optional[int] = None):
    seed = draw_seed() if (seed is None and p > 0.0) else (seed or 0)
    return _GATResidual.apply(x, wlog, wcat, b, csr, csr_t, int(heads), float(slope), float(p),
                              seed)


def transformer_residual(x, wqkv, bqkv, ws, bs, csr, csr_t, heads: int, p: float,
                         seed: Optional[int] = None):
    seed = draw_seed() if (seed is None and p > 0.0) else (seed or 0)
    return _TransformerResidual.apply(x, wqkv, bqkv, ws, bs, csr, csr_t, int(heads), float(p),
                                      seed)


def bn_relu_dropout(z, bn_mod, p: float, seed: Optional[int] = None):
    seed = draw_seed() if (seed is None and p > 0.0) else (seed or 0)
    if bn_mod is None:
        return _BNReluDropout.apply(z, None, None, None, float(p), seed)
    return _BNReluDropout.apply(z, bn_mod.weight, bn_mod.bias, bn_mod, float(p), seed)


def weighted_mse(pred, target, weights, pressure_ref_weight: float, fieldwise: bool):
    return _WMSE.apply(pred, target, tuple(float(w) for w in weights),
                       float(pressure_ref_weight), bool(fieldwise))
