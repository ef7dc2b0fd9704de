"""ctypes binding of libmignn.so (the C ABI declared in include/mignn.h).

The library is loaded lazily on first use and the product path fails loudly
when it is missing: there is no CPU or eager-PyTorch fallback.  `torch` is
imported first on purpose -- it brings in its HIP runtime
(libamdhip64.so.7), which the dynamic loader then shares with libmignn.so, so
torch's streams and device pointers are valid inside the library.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_size_t, c_void_p

import torch  # noqa: F401  (must precede loading libmignn.so)

LIB_NAME = "libmignn.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# A/B timing scripts (scripts/gpu_ab.sh, gpu_legab.sh) point this at a variant
# build of the same sources; lib() then loads it with a warning on stderr and
# the same ABI-version check.  The product path never sets it.
VARIANT_ENV = "MIGNN_LIB_VARIANT"

EPI_BIAS, EPI_RESIDUAL, EPI_AFFINE, EPI_RELU = 1, 2, 4, 8
CSR_VERBATIM, CSR_ONE_SELF_LOOP, CSR_TRANSPOSE = 0, 1, 4

_P = c_void_p
# name -> (restype, argtypes); mirrors include/mignn.h
SIGNATURES = {
    "mignn_abi_version": (c_int, []),
    "mignn_last_error": (ctypes.c_char_p, []),
    "mignn_device_errors": (c_int, [_P, c_int]),
    "mignn_csr_scratch_bytes": (c_size_t, [c_int64, c_int64]),
    "mignn_csr_build": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, c_size_t, _P]),
    "mignn_linear": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, c_int, _P, c_int, _P, _P,
                             c_int64, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_linear_f16x3_prep_bytes": (c_size_t, [c_int, c_int]),
    "mignn_linear_f16x3_prep": (c_int, [_P, c_int, c_int, _P, c_size_t, _P]),
    "mignn_linear_f16x3": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, c_int, _P, c_int, _P,
                                   _P, c_int64, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_input_proj": (c_int, [_P, c_int64, c_int, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_bn_fold": (c_int, [_P, _P, _P, _P, c_float, c_int, _P, _P, _P]),
    "mignn_gcn_aggregate": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P,
                                    c_int64, _P]),
    "mignn_sum_aggregate": (c_int, [_P, _P, _P, c_int64, c_float, c_int64, c_int64, c_int, _P,
                                    c_int64, _P]),
    "mignn_gat_aggregate": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, c_int,
                                    c_float, _P, c_int64, _P]),
    "mignn_gat_layer_scratch_bytes": (c_size_t, [c_int64, c_int64, c_int, c_int]),
    "mignn_gat_layer": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int64, c_int, c_int,
                                c_float, _P, _P, c_int64, _P, _P, _P, _P, _P, c_int, _P,
                                c_size_t, _P, c_int64, _P]),
    "mignn_gat_layer_next": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int64, c_int, c_int,
                                     c_float, _P, _P, c_int64, _P, _P, _P, _P, _P, c_int, _P,
                                     c_size_t, _P, c_int64, _P, _P, _P]),
    "mignn_transformer_layer_scratch_bytes": (c_size_t, [c_int64, c_int, c_int]),
    "mignn_transformer_layer": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int, c_int,
                                        c_float, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P,
                                        c_size_t, _P, c_int64, _P]),
    "mignn_transformer_fused_prep_bytes": (c_size_t, [c_int, c_int]),
    "mignn_transformer_fused_prep": (c_int, [_P, c_int, c_int, _P, c_size_t, _P]),
    "mignn_transformer_layer_fused": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int, c_int,
                                              c_float, _P, _P, _P, _P, _P, _P, c_int, _P, c_size_t,
                                              _P, c_int64, _P]),
    "mignn_transformer_aggregate": (c_int, [_P, _P, _P, c_int64, _P, c_int64, c_int64, c_int64,
                                            c_int, c_int, c_float, _P, c_int64, _P]),
    "mignn_gcn_layer": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P, _P, _P,
                                c_int, _P, c_int64, _P]),
    "mignn_gcn_layer_f16x3": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P,
                                      _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_ring_plan_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "mignn_gcn_ring_plan": (c_int, [_P, _P, _P, c_int64, c_int64, c_int, _P, c_size_t, _P, _P]),
    "mignn_gcn_layer_ring": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P,
                                     _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_aggregate_ring": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int,
                                         _P, c_int64, _P]),
    "mignn_gcn_win_plan_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "mignn_gcn_win_plan": (c_int, [_P, _P, _P, c_int64, c_int64, c_int, _P, _P, c_size_t, _P, _P]),
    "mignn_gcn_layer_win": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P,
                                    _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_layer_win_codes": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int,
                                          _P, _P, _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_aggregate_win": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int,
                                        _P, c_int64, _P]),
    "mignn_mlp_head_prep_bytes": (c_size_t, [c_int]),
    "mignn_mlp_head_prep": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, c_int, c_int, _P, c_size_t,
                                    _P]),
    "mignn_mlp_head": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int, _P, c_int64, _P, _P]),
    "mignn_csr_build_gcn": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P, _P,
                                    c_size_t, _P]),
    "mignn_csr_build_relabeled": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P,
                                          c_size_t, _P]),
    "mignn_locality_order_scratch_bytes": (c_size_t, [c_int64]),
    "mignn_locality_order": (c_int, [_P, c_int64, c_int64, _P, c_int64, _P, _P, _P, c_size_t,
                                     _P]),
    "mignn_locality_order_cols": (c_int, [_P, c_int64, c_int64, _P, c_int64, _P, _P, _P, _P,
                                          c_size_t, _P]),
    "mignn_gcn_layer0_coords": (c_int, [_P, _P, _P, _P, c_int64, c_int, c_int64, c_int64, _P,
                                        c_int, _P, c_int64, _P]),
    "mignn_range_mark": (c_int, [_P, c_int64, c_int64, c_int64, c_int64, _P, _P, _P, _P]),
    "mignn_range_relabel": (c_int, [_P, c_int64, c_int64, c_int64, _P, _P, c_int64, _P, _P]),
    "mignn_range_partition": (c_int, [_P, _P, _P, c_int64, c_int64, _P, _P, _P]),
    "mignn_csr_build_range": (c_int, [_P, c_int64, c_int64, c_int64, c_int64, _P, _P, c_int64, c_int,
                                      _P, _P, _P, _P, _P, _P, c_size_t, _P]),
    "mignn_gcn_layer0_codes": (c_int, [_P, _P, _P, _P, c_int64, c_int, c_int64, c_int64, _P,
                                       c_int64, _P]),
    "mignn_mesh_graph_scratch_bytes": (c_size_t, [c_int64, c_int64]),
    "mignn_mesh_graph_count": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, _P, c_int64, c_int,
                                       _P, _P, c_size_t, _P]),
    "mignn_mesh_graph_emit": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, _P, _P, c_int,
                                      c_int64, _P, _P, _P, c_int64, _P, c_size_t, _P]),
    "mignn_edge_attributes": (c_int, [_P, c_int64, c_int64, _P, _P, _P]),
    "mignn_boundary_mask": (c_int, [_P, c_int64, c_int64, c_int64, c_int64, _P, _P]),
    "mignn_field_affine": (c_int, [_P, c_int, c_int64, c_int64, c_int, _P, _P, c_int, c_int, _P, _P,
                                   c_int64, _P]),
    "mignn_field_moments": (c_int, [_P, c_int, c_int64, c_int64, c_int, _P, _P, _P]),
    "mignn_write_openfoam_field": (c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.c_char_p, ctypes.c_char_p, _P, c_int64, c_int,
                                           c_int64]),
    "mignn_foam_parse_labels": (c_int, [_P, c_int64, c_int, _P, c_int64, _P]),
    "mignn_foam_parse_points": (c_int, [_P, c_int64, _P, c_int64, _P]),
    "mignn_foam_parse_faces": (c_int, [_P, c_int64, _P, c_int64, _P, c_int64, _P, _P]),
    "mignn_foam_parse_scalar_field": (c_int, [_P, c_int64, _P, c_int64, _P]),
    "mignn_foam_parse_vector_field": (c_int, [_P, c_int64, _P, c_int64, _P]),
    "mignn_foam_cell_centers": (c_int, [_P, c_int64, _P, c_int64, _P, c_int64, _P, _P, c_int64,
                                        c_int64, _P]),
    "mignn_train_scratch_bytes": (c_size_t, [c_int64, c_int]),
    "mignn_gemm": (c_int, [_P, c_int64, c_int64, _P, c_int64, c_int64, c_int64, c_int64, c_int64,
                           _P, c_int64, _P, c_int64, _P, c_size_t, _P]),
    "mignn_col_sums": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, c_size_t, _P]),
    "mignn_bn_train_stats": (c_int, [_P, c_int64, c_int64, c_int, c_float, c_float, _P, _P, _P,
                                     _P, _P, _P, c_size_t, _P]),
    "mignn_bn_act_forward": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, c_int, c_float,
                                     ctypes.c_uint64, _P, c_int64, _P]),
    "mignn_bn_act_backward": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, _P, _P, _P, _P,
                                      c_int, c_float, ctypes.c_uint64, _P, c_int64, _P, _P, _P,
                                      c_size_t, _P]),
    "mignn_wmse_loss": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, _P, c_float, c_int, _P,
                                _P, _P, c_size_t, _P]),
    "mignn_wmse_loss_backward": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, _P, c_float,
                                         c_int, _P, _P, _P, c_int64, _P]),
    "mignn_dropout_mask": (c_int, [c_int64, c_int, c_float, ctypes.c_uint64, _P, _P]),
    "mignn_gat_train_forward": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int, c_int, c_float,
                                        c_float, ctypes.c_uint64, _P, c_int64, _P, _P]),
    "mignn_transformer_train_forward": (c_int, [_P, _P, _P, c_int64, _P, c_int64, c_int64, c_int,
                                                c_int, c_float, c_float, ctypes.c_uint64, _P,
                                                c_int64, _P, c_int64, _P, _P]),
    "mignn_transformer_train_backward": (c_int, [_P, _P, _P, _P, _P, c_int64, _P, c_int64,
                                                 _P, c_int64, c_int64, c_int, c_int, c_float, c_float,
                                                 ctypes.c_uint64, _P, _P, c_int64, _P]),
    "mignn_gat_train_backward": (c_int, [_P, _P, _P, _P, _P, _P, c_int64, _P, c_int64, _P,
                                         c_int64, _P, c_int64, c_int64, c_int, c_int, c_float, c_float,
                                         ctypes.c_uint64, _P, _P, _P, c_int64, _P]),
    "mignn_input_proj_rows": (c_int, [_P, c_int64, c_int, _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gin_layer": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int, c_float, _P, _P, _P,
                                _P, _P, _P, c_int, _P, c_int64, _P, c_int64, _P]),
    "mignn_gin_fused_prep_bytes": (c_size_t, [c_int]),
    "mignn_gin_fused_prep": (c_int, [_P, c_int, _P, c_size_t, _P]),
    "mignn_gin_layer_fused": (c_int, [_P, _P, _P, c_int64, c_int64, c_int64, c_int, c_float, _P,
                                      _P, _P, _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_transformer_layer0_coords": (c_int, [_P, _P, _P, c_int64, c_int, c_int64, c_int64, c_int,
                                                c_int, c_float, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gat_layer0_coords": (c_int, [_P, _P, _P, c_int64, c_int, c_int64, c_int64, c_int, c_int,
                                        c_float, _P, _P, c_int, _P, c_int64, _P, _P, _P]),
    "mignn_gat_layer0_fused": (c_int, [_P, _P, _P, c_int64, c_int, c_int64, c_int64, c_int, c_float,
                                       _P, _P, _P, _P, _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gin_layer0_fused": (c_int, [_P, _P, _P, c_int64, c_int, c_int64, c_int64, c_int, c_float,
                                       _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_layer_fused": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P,
                                      _P, _P, c_int, _P, c_int64, _P]),
    "mignn_gcn_norm": (c_int, [_P, _P, _P, c_int64, c_int64, _P, _P]),
    "mignn_rows_gather": (c_int, [_P, c_int64, _P, c_int64, c_int, _P, c_int64, _P]),
    "mignn_grid_graph": (c_int, [c_int, c_int, c_int, c_int, c_int, _P, _P, _P]),
}

# diagnostic entry points (include/mignn_diag.h; timing studies only)
DIAG_SIGNATURES = {
    "mignn_diag_linear_f16x3": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, c_int, _P,
                                        c_int, _P, _P, c_int64, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_diag_gather": (c_int, [c_int, _P, _P, _P, _P, c_int64, c_int, c_int, c_int, c_int, _P,
                                  _P]),
    "mignn_diag_set_trace": (c_int, [_P]),
    "mignn_diag_set_trace_f16x3": (c_int, [_P]),
    "mignn_diag_clock": (c_int, [c_int, c_int, _P, _P]),
    "mignn_diag_pk_fma": (c_int, [c_int, _P, c_int64, _P, c_int, _P, _P]),
    "mignn_diag_mlp_head": (c_int, [c_int, _P, c_int64, _P, _P, _P]),
    "mignn_diag_gcn_layer": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P, _P, _P,
                                     _P, c_int, _P, c_int64, _P]),
    "mignn_diag_gcn_layer_f16x3": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P,
                                           _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_diag_ring_trace": (c_int, [_P]),
    "mignn_diag_ring": (c_int, [c_int, _P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P,
                                _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_diag_win_trace": (c_int, [_P]),
    "mignn_diag_win": (c_int, [c_int, _P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int, _P,
                               _P, _P, _P, c_int, _P, c_int64, _P]),
    "mignn_diag_dma_oob_agg": (c_int, [_P, c_int]),
    "mignn_diag_dma_oob_ring": (c_int, [_P, c_int]),
    "mignn_diag_dma_oob_win": (c_int, [_P, c_int]),
    "mignn_diag_dma_oob_pc": (c_int, [_P, c_int]),
    "mignn_diag_dma_oob_gemm": (c_int, [_P, c_int]),
    "mignn_diag_set_gat_fused": (c_int, [c_int]),
    "mignn_diag_set_fused_flags": (c_int, [c_int]),
    "mignn_diag_linear": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, c_int, _P, c_int, _P,
                                  _P, c_int64, _P, _P, c_int, _P, c_int64, _P]),
}

_lib = None
_diag = None
DIAG_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmignn_diag.so")


class MignnError(RuntimeError):
    pass


def _load(path, sigs):
    if not os.path.exists(path):
        raise MignnError(
            f"{os.path.basename(path)} not found at {path}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
            "There is no CPU fallback.")
    h = ctypes.CDLL(path)
    for name, (res, args) in sigs.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    if h.mignn_abi_version() != 1:
        raise MignnError("libmignn ABI mismatch")
    return h


def lib():
    """Load (once) and return the ctypes handle of the product library
    (libmignn.so: the C ABI of include/mignn.h, nothing else); raise if the
    .so is missing."""
    global _lib
    if _lib is None:
        path = os.environ.get(VARIANT_ENV) or LIB_PATH
        if path != LIB_PATH:
            import sys
            print(f"mignn: {VARIANT_ENV} set -- loading the variant library {path} "
                  f"instead of {LIB_PATH} (A/B timing only)", file=sys.stderr)
        _lib = _load(path, SIGNATURES)
    return _lib


def diag_lib():
    """The diagnostic build (libmignn_diag.so: the product entry points plus
    the timing-study entries of include/mignn_diag.h).  Used by scripts/ only;
    the product path and the tests never load it."""
    global _diag
    if _diag is None:
        _diag = _load(DIAG_LIB_PATH, {**SIGNATURES, **DIAG_SIGNATURES})
    return _diag


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def last_error() -> str:
    msg = lib().mignn_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str):
    if rc != 0:
        raise MignnError(f"{what} failed (status {rc}): {last_error()}")


DEVERR_SPIN = 1
DEVERR_PLAN = 2
_DEVERR_NAMES = {DEVERR_SPIN: "a bounded in-kernel wait (LDS hand-off) ran out",
                 DEVERR_PLAN: "a window-kernel launch did not match its plan header"}


def device_errors(clear: bool = True) -> int:
    """The current device's sticky in-kernel error bits (mignn_device_errors;
    synchronises the device).  Nonzero means some launch since the last
    clear produced wrong output."""
    word = ctypes.c_uint(0)
    check(lib().mignn_device_errors(ctypes.addressof(word), 1 if clear else 0), "mignn_device_errors")
    return int(word.value)


def check_device_errors(what: str = "mignn kernels"):
    """Raise if any launch since the last check recorded an in-kernel error."""
    bits = device_errors(clear=True)
    if bits:
        names = [v for k, v in _DEVERR_NAMES.items() if bits & k] or [hex(bits)]
        raise MignnError(f"{what}: device error {bits:#x}: " + "; ".join(names))
