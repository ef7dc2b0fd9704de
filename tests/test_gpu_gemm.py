"""Split-fp16 GEMM (mignn_linear_f16x3) against a float64 torch reference.

The bound is the arithmetic's own: every product carries ~2^-22 relative
error of |a||w| (hi/lo fp16 splits of power-of-two-scaled operands, fp32
accumulation), so |C - C64| <= 2e-6 * (|A| @ |W|^T) + fp32 rounding of the
result; the exact-fp32 mignn_linear is held to the same bound for reference."""

import pytest
import torch

from mignn.gnn_model import f16x3_image, linear, linear_f16x3

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from mignn import _lib
    _lib.lib()


def _ref(a, w, a2=None, bias=None, residual=None, scale=None, shift=None, relu=False):
    A = a.double() if a2 is None else torch.cat([a, a2], 1).double()
    W = w.double()
    c = A @ W.T
    mag = A.abs() @ W.abs().T
    if bias is not None:
        c = c + bias.double()
    if residual is not None:
        c = residual.double() + c
        mag = mag + residual.double().abs()
    if scale is not None:
        c = c * scale.double() + shift.double()
        mag = mag * scale.double().abs() + shift.double().abs()
    if relu:
        c = c.clamp_min(0)
    return c, mag


def _check(c, ref, mag):
    err = (c.double() - ref).abs()
    bound = 2e-6 * mag + 2 * torch.finfo(torch.float32).eps * ref.abs() + 1e-30
    worst = (err / bound).max().item()
    assert worst <= 1.0, f"err/bound {worst:.3f}, max err {err.max().item():.3e}"
    return err.max().item()


@pytest.mark.parametrize("m,k,n", [(1, 256, 256), (127, 256, 256), (1000, 256, 128),
                                   (4099, 1028, 256), (777, 256, 1028), (300, 64, 80),
                                   (2048, 512, 512), (129, 4, 64)])
def test_plain_shapes(m, k, n):
    g = torch.Generator(device=DEV).manual_seed(m * 7 + k + n)
    a = torch.randn(m, k, device=DEV, generator=g)
    w = torch.randn(n, k, device=DEV, generator=g) / k ** 0.5
    c = linear_f16x3(a, f16x3_image(w), n)
    ref, mag = _ref(a, w)
    _check(c, ref, mag)
    _check(linear(a, w), ref, mag)


@pytest.mark.parametrize("k1,k2", [(1028, 256), (256, 256), (36, 4)])
def test_two_segments_and_epilogue(k1, k2):
    """[A | A2] straddling a 32-wide chunk (TransformerConv's output GEMM
    [agg | x], k1 = 4H + 4), bias + residual + BN affine + ReLU."""
    m, n = 2500, 256
    g = torch.Generator(device=DEV).manual_seed(k1 + k2)
    a = torch.randn(m, k1, device=DEV, generator=g)
    a2 = torch.randn(m, k2, device=DEV, generator=g)
    w = torch.randn(n, k1 + k2, device=DEV, generator=g) / (k1 + k2) ** 0.5
    bias, scale, shift = (torch.randn(n, device=DEV, generator=g) for _ in range(3))
    res = torch.randn(m, n, device=DEV, generator=g)
    c = linear_f16x3(a, f16x3_image(w), n, bias, a2=a2, residual=res, scale=scale, shift=shift,
                     relu=True)
    ref, mag = _ref(a, w, a2, bias, res, scale, shift, relu=True)
    _check(c, ref, mag)


def test_row_dynamic_range_and_zeros():
    """Online per-row exponent: rows whose magnitude grows by 2^40 along k
    (the accumulator is rescaled as the row max rises), rows that are zero
    until the last chunk, all-zero rows, tiny rows (2^-60)."""
    m, k, n = 512, 512, 256
    g = torch.Generator(device=DEV).manual_seed(9)
    a = torch.randn(m, k, device=DEV, generator=g)
    ramp = torch.pow(2.0, torch.linspace(-20, 20, k, device=DEV))
    a[0:128] *= ramp
    a[128:256] *= torch.flip(ramp, [0])
    a[256:320, : k - 32] = 0
    a[320:384] = 0
    a[384:448] *= 2.0 ** -60
    w = torch.randn(n, k, device=DEV, generator=g)
    w[:, ::7] *= 1e4                                     # per-column W exponent: wide columns
    w[5] *= 1e-20
    c = linear_f16x3(a, f16x3_image(w), n)
    ref, mag = _ref(a, w)
    _check(c, ref, mag)
    assert torch.equal(c[320:384], torch.zeros_like(c[320:384]))


def test_strided_output_and_inputs():
    """Row strides != width (views into wider buffers), output into a slice."""
    m, k, n = 900, 256, 256
    g = torch.Generator(device=DEV).manual_seed(3)
    big = torch.randn(m, k + 64, device=DEV, generator=g)
    a = big[:, 32:32 + k]
    w = torch.randn(n, k, device=DEV, generator=g) / 16
    out = torch.full((m, n + 8), 7.0, device=DEV)
    linear_f16x3(a, f16x3_image(w), n, out=out[:, 4:4 + n])
    ref, mag = _ref(a, w)
    _check(out[:, 4:4 + n], ref, mag)
    assert (out[:, :4] == 7).all() and (out[:, 4 + n:] == 7).all()


def test_rejects_bad_arguments():
    from mignn import _lib
    a = torch.randn(8, 6, device=DEV)                     # k = 6: not a multiple of 4
    w = torch.randn(64, 6, device=DEV)
    img = torch.empty(_lib.lib().mignn_linear_f16x3_prep_bytes(64, 6), dtype=torch.uint8,
                      device=DEV)
    with pytest.raises(RuntimeError):
        linear_f16x3(a, img, 64)
