"""v_pk_fma_f32 in the row-code expansion (DESIGN.md
§3.16): the explicit packed-f32 form must equal layer 0's scalar fma chain
bitwise, and the failure mode that dropped it in round 5 is reproduced.

The expansion computes per feature pair (f, f+1) t = coef[.,7] + sum_k
coef[.,k] v[k] as one v_pk_fma_f32 per input k.  The input v[k] is the SAME
for both halves, so the instruction must broadcast it: with src1 a register
pair holding {v[k], v[k+1]} (the inputs as loaded, 8 B at a time) the high
result has to take src1's LOW half, i.e. op_sel_hi:[1,0,1].  Written without
the modifier (VOP3P's default op_sel_hi:[1,1,1]) the high half multiplies
coef[f+1][k] by v[k+1]: every odd feature of every row wrong, the even ones
exact -- "wrong rows on the box".  The diag kernel (csrc/diag.hip,
mignn_diag_pk_fma) runs the scalar chain (form 0), the packed form with the
broadcast (1), without it (2), and the compiler's own packing (3)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from mignn import _lib
    return _lib.diag_lib()


def _run(L, form, codes, coef):
    from mignn import _lib
    n, h = codes.shape[0], coef.shape[0]
    out = torch.full((n, h), float("nan"), device=codes.device)
    _lib.check(L.mignn_diag_pk_fma(form, _lib.ptr(codes), n, _lib.ptr(coef), h, _lib.ptr(out),
                                   _lib.stream()), "mignn_diag_pk_fma")
    torch.cuda.synchronize()
    return out


def test_pk_fma_expansion_forms(L):
    g = torch.Generator().manual_seed(5)
    n, h = 40000, 128
    codes = torch.randn(n, 8, generator=g) * torch.tensor([1, 1, 1, 3, 3, 3, 0.5, 0.0])
    coef = torch.randn(h, 8, generator=g)
    codes, coef = codes.cuda(), coef.cuda()
    ref = _run(L, 0, codes, coef)
    # the scalar chain is the restatement's fp32 chain (same order, fused)
    c64, v64 = coef.double().cpu(), codes.double().cpu()
    r64 = (v64[:, :7] @ c64[:, :7].T + c64[:, 7]).clamp_min(0)
    assert (ref.cpu().double() - r64).abs().max().item() <= 1e-5 * max(1.0, r64.abs().max().item())
    pk = _run(L, 1, codes, coef)
    assert torch.equal(pk.view(torch.int32), ref.view(torch.int32)), "op_sel_hi:[1,0,1] form not bitwise"
    comp = _run(L, 3, codes, coef)
    assert torch.equal(comp.view(torch.int32), ref.view(torch.int32)), "compiler-packed form not bitwise"
    bad = _run(L, 2, codes, coef)
    # without the broadcast: even features exact, odd features wrong
    assert torch.equal(bad[:, 0::2].view(torch.int32), ref[:, 0::2].view(torch.int32))
    wrong_rows = (bad[:, 1::2] != ref[:, 1::2]).any(1).float().mean().item()
    print(f"pk_fma without op_sel_hi: {wrong_rows:.3f} of the rows wrong (odd features)")
    assert wrong_rows > 0.99
