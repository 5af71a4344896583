"""ctypes binding of libonebit_hip.so, the C ABI declared in include/onebit_hip.h.

The library is built in-tree (``make -C cmu-11785-idl-1.58bit-asr_amd/csrc`` or
``__graft_entry__.build()``). There is deliberately no fallback: if the library is
missing or a call fails, every caller raises. The reference's eager-torch quantizer
(onebit_asr/quant.py:38-127) is re-stated only under ``oracle/`` as a test checker.

``torch`` is imported before the library is opened so that the ``libamdhip64.so.7``
torch already loaded (same SONAME) is the HIP runtime the kernels run on, and a
``torch.cuda`` stream handle is a valid ``hipStream_t`` for every entry point.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL: shares torch's HIP runtime)

LIB_NAME = "libonebit_hip.so"
LIB_PATH = Path(os.environ.get("ONEBIT_HIP_LIB") or Path(__file__).with_name(LIB_NAME))

OB_OK = 0
OB_ERR_SHAPE = -2
OB_ERR_BITWIDTH = -3

_c_f = ctypes.c_void_p  # device pointers are passed as raw addresses
_i64 = ctypes.c_int64
_int = ctypes.c_int
_sz = ctypes.c_size_t
_f32 = ctypes.c_float
_f64 = ctypes.c_double

# name -> (restype, argtypes); mirrors include/onebit_hip.h one-to-one.
SIGNATURES = {
    "ob_abi_version": (_int, []),
    "ob_source_digest": (ctypes.c_char_p, []),
    "ob_status_string": (ctypes.c_char_p, [_int]),
    "ob_quant_pack": (_int, [_c_f, _c_f, _int, _int, _i64, _i64, _c_f, _c_f, _c_f]),
    "ob_quant_pack_item_blocks": (_i64, [_i64, _i64]),
    "ob_quant_pack_group": (_int, [_c_f, _int, _i64, _c_f]),
    "ob_weight_bf16_item_blocks": (_i64, [_i64, _i64]),
    "ob_bitlinear_fwd_swish_drop": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _i64, _f32, _c_f, _i64,
               _c_f, _c_f, _c_f]),
    "ob_bitlinear_fwd_residual": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _i64, _c_f, _f32, _f32,
               _c_f, _i64, _c_f, _i64, _c_f, _c_f]),
    "ob_bitlinear_bwd_dx_swish_drop": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _i64, _c_f, _f32, _c_f, _i64,
               _c_f, _c_f]),
    "ob_drop_scale_bwd": (_int, [_c_f, _i64, _i64, _f32, _f32, _c_f, _i64, _c_f, _i64, _c_f, _c_f]),
    "ob_residual_drop_fwd": (
        _int, [_c_f, _c_f, _i64, _i64, _f32, _f32, _c_f, _i64, _c_f, _i64, _c_f, _c_f]),
    "ob_convmod_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "ob_convmod_fwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _f32, _c_f, _c_f, _c_f,
               _c_f, _c_f, _sz, _c_f]),
    "ob_convmod_bwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _c_f,
               _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_convmod_bwd_defer": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _c_f,
               _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f, _i64, _c_f, _c_f]),
    "ob_decattn_supported": (_int, [_i64, _i64, _i64]),
    "ob_decattn_fwd": (_int, [_c_f, _i64, _c_f, _i64, _c_f, _i64, _c_f, _i64, _i64, _i64, _i64,
                              _i64, _i64, _f32, _c_f, _i64, _c_f, _c_f, _c_f]),
    "ob_decattn_bwd": (_int, [_c_f, _c_f, _c_f, _i64, _c_f, _i64, _c_f, _i64, _i64, _i64, _i64, _i64,
                              _i64, _f32, _c_f, _c_f, _i64, _c_f, _i64, _c_f, _i64, _c_f]),
    "ob_cm_wgrad_entry_bytes": (_sz, []),
    "ob_cm_wgrad_table": (_int, [_c_f, _i64, _i64, _c_f]),
    "ob_bias_relu_fwd": (_int, [_c_f, _c_f, _i64, _i64, _i64, _c_f]),
    "ob_relu_bias_bwd_workspace": (_sz, [_i64, _i64]),
    "ob_relu_bias_bwd": (_int, [_c_f, _c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_colsum_workspace": (_sz, [_i64]),
    "ob_colsum": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _sz, _c_f]),
    "ob_dense_supported": (_int, [_i64, _i64]),
    "ob_silu_fast_monotone_check": (_int, [ctypes.c_uint32, ctypes.c_uint32, _c_f, _c_f]),
    "ob_dense_gemm_residual_drop": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _i64, _c_f, _f32, _c_f,
                                            _i64, _c_f, _c_f]),
    "ob_dense_gemm": (_int, [_c_f, _i64, _i64, _c_f, _int, _c_f, _i64, _c_f, _c_f]),
    "ob_dense_dw_workspace": (_sz, [_i64, _i64, _i64]),
    "ob_dense_dw": (_int, [_c_f, _c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_subsample_image_bytes": (_sz, [_i64]),
    "ob_subsample_pack": (_int, [_c_f, _i64, _c_f, _c_f]),
    "ob_subsample_fwd": (_int, [_c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _c_f,
                                _c_f, _c_f]),
    "ob_subsample_bwd_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "ob_subsample_bwd": (_int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _c_f,
                                _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_ctc_loss_fwd_groups": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _sz, _c_f]),
    "ob_ctc_loss_bwd_groups": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _c_f, _sz,
               _c_f]),
    "ob_ctc_logits_workspace": (_sz, [_i64, _i64, _i64]),
    "ob_ctc_loss_logits_fwd_groups": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _sz, _c_f]),
    "ob_ctc_loss_logits_bwd_groups": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _c_f, _sz,
               _c_f]),
    "ob_att_kl_workspace": (_sz, [_i64, _i64]),
    "ob_att_kl_loss_fwd": (
        _int, [_c_f, _c_f, _c_f, _i64, _i64, _i64, _int, _f32, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_bitlinear_bwd_dx_passes_sum": (
        _int, [_i64, _c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _i64, _c_f, _c_f]),
    "ob_bitlinear_fwd_residual_ln": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _i64, _c_f, _f32, _f32,
               _c_f, _i64, _c_f, _i64, _c_f, _int, _c_f, _c_f, _f32, _c_f, _c_f, _c_f, _c_f, _c_f,
               _f32, _c_f, _c_f, _c_f, _c_f]),
    "ob_loss_combine_fwd": (_int, [_c_f, _c_f, _c_f, _f32, _f32, _f32, _c_f, _c_f, _c_f]),
    "ob_loss_combine_bwd": (_int, [_c_f, _f32, _f32, _f32, _c_f, _c_f, _c_f, _c_f]),
    "ob_att_kl_loss_bwd": (
        _int, [_c_f, _c_f, _c_f, _i64, _i64, _i64, _f32, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_quant_dequant": (_int, [_c_f, _c_f, _int, _int, _i64, _c_f, _c_f]),
    "ob_quant_ste_bwd_workspace": (_sz, [_i64]),
    "ob_quant_ste_bwd": (_int, [_c_f, _c_f, _c_f, _int, _int, _i64, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_bitlinear_fwd": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _int, _c_f, _i64, _c_f, _c_f]),
    "ob_bitlinear_fwd_signacc": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _int, _c_f, _i64, _c_f, _c_f]),
    "ob_bitlinear_bwd_dx": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _int, _i64, _c_f, _c_f]),
    "ob_bitlinear_bwd_dw_workspace": (_sz, [_i64, _i64, _i64]),
    "ob_bitlinear_bwd_dw": (
        _int,
        [_c_f, _c_f, _i64, _i64, _i64, _c_f, _c_f, _int, _int, _c_f, _c_f, _c_f, _c_f, _sz, _c_f],
    ),
    "ob_quant_pack_dyn": (_int, [_c_f, _c_f, _int, _c_f, _i64, _i64, _c_f, _c_f, _c_f]),
    "ob_bitlinear_bwd_dw_dyn": (
        _int,
        [_c_f, _c_f, _i64, _i64, _i64, _c_f, _c_f, _int, _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f],
    ),
    "ob_dwconv1d_fwd": (_int, [_c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f]),
    "ob_dwconv1d_bwd_workspace": (_sz, [_i64, _i64, _i64]),
    "ob_dwconv1d_bwd": (
        _int, [_c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_ctc_loss_workspace": (_sz, [_i64, _i64, _i64]),
    "ob_ctc_loss_fwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _sz, _c_f]),
    "ob_ctc_loss_bwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _int, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_bitlinear_fwd_passes": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _i64, _c_f, _c_f]),
    "ob_ctc_greedy_decode": (_int, [_c_f, _c_f, _i64, _i64, _i64, _int, _c_f, _c_f, _c_f, _c_f]),
    "ob_layernorm_fwd": (_int, [_c_f, _c_f, _c_f, _i64, _i64, _f32, _c_f, _c_f, _c_f, _c_f]),
    "ob_layernorm_fwd_pair": (_int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _f32, _f32, _c_f,
                                     _c_f, _c_f, _c_f, _c_f, _c_f, _c_f]),
    "ob_layernorm_fwd_amax_workspace": (_sz, [_i64]),
    "ob_layernorm_fwd_amax": (_int, [_c_f, _c_f, _c_f, _i64, _i64, _f32, _c_f, _c_f, _c_f, _i64,
                                     _c_f, _c_f, _sz, _c_f]),
    "ob_layernorm_fwd_i8": (_int, [_c_f, _c_f, _c_f, _i64, _i64, _f32, _i64, _c_f, _c_f, _c_f,
                                   _sz, _c_f]),
    "ob_layernorm_bwd_defer": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f,
               _f32, _f32, _c_f, _i64, _c_f, _i64, _c_f, _i64, _c_f]),
    "ob_layernorm_bwd_pair_workspace": (_sz, [_i64, _i64]),
    "ob_layernorm_bwd_pair": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _c_f, _c_f,
               _c_f, _c_f, _c_f, _c_f, _sz, _c_f, _f32, _f32, _c_f, _i64, _c_f, _i64, _c_f, _i64,
               _i64, _c_f]),
    "ob_ln_param_entry_bytes": (_sz, []),
    "ob_ln_param_table": (_int, [_c_f, _i64, _i64, _c_f]),
    "ob_dw_finish_entry_bytes": (_sz, []),
    "ob_bitlinear_bwd_dw_passes_defer": (
        _int, [_c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _int, _c_f, _c_f, _c_f, _c_f, _c_f,
               _sz, _c_f, _i64, _i64, _c_f, _c_f]),
    "ob_bitlinear_bwd_dw_passes_group_defer": (
        _int, [_i64, _c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _int, _c_f, _c_f, _c_f, _c_f,
               _c_f, _sz, _c_f, _i64, _i64, _c_f, _c_f]),
    "ob_dw_finish_table": (_int, [_c_f, _i64, _i64, _c_f]),
    "ob_dw_grouped_supported": (_int, [_i64, _i64]),
    "ob_dw_grouped_workspace": (_sz, [_c_f, _i64]),
    "ob_dw_grouped_tickets": (_sz, [_c_f, _i64]),
    "ob_dw_grouped": (_int, [_c_f, _i64, _c_f, _sz, _c_f, _sz, _c_f]),
    "ob_dense_dw_defer": (_int, [_c_f, _c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _sz, _c_f, _i64,
                                 _i64, _c_f, _c_f]),
    "ob_layernorm_bwd_workspace": (_sz, [_i64, _i64]),
    "ob_layernorm_bwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_layernorm_bwd_res": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_layernorm_bwd_ex": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f,
               _f32, _f32, _c_f, _i64, _c_f, _i64, _c_f]),
    "ob_act_absmax_workspace": (_sz, [_i64]),
    "ob_act_absmax": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _sz, _c_f]),
    "ob_act_dequant_i8": (_int, [_c_f, _i64, _i64, _c_f, _c_f, _c_f]),
    "ob_bitlinear_fwd_i8": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _c_f, _i64, _c_f, _c_f]),
    "ob_bitlinear_fwd_i8_epi": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _c_f, _i64, _int, _c_f,
               _f32, _c_f, _i64, _c_f, _c_f, _c_f]),
    "ob_bitlinear_fwd_passes_group": (
        _int, [_i64, _c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _i64, _c_f, _c_f]),
    "ob_bitlinear_fwd_i8q": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _c_f, _c_f, _i64, _int, _c_f,
               _f32, _c_f, _i64, _c_f, _c_f, _c_f]),
    "ob_bitlinear_bwd_dx_passes": (
        _int, [_c_f, _i64, _i64, _i64, _c_f, _c_f, _c_f, _c_f, _int, _i64, _c_f, _c_f]),
    "ob_bitlinear_bwd_dw_passes_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "ob_bitlinear_bwd_dw_passes": (
        _int, [_c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _int, _c_f, _c_f, _c_f, _c_f, _c_f,
               _sz, _c_f]),
    "ob_bitlinear_bwd_dw_passes_group_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "ob_bitlinear_bwd_dw_passes_group": (  # pointer arrays: host addresses (ptr_array)
        _int, [_i64, _c_f, _c_f, _i64, _i64, _i64, _i64, _c_f, _c_f, _int, _c_f, _c_f, _c_f, _c_f,
               _c_f, _sz, _c_f]),
    "ob_relattn_fwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64, _f32, _c_f,
               _i64, _c_f, _c_f, _c_f, _c_f]),
    "ob_relattn_saved_elems": (_i64, [_i64, _i64, _i64, _i64]),
    "ob_relattn_probs_elems": (_i64, [_i64, _i64, _i64]),
    "ob_relattn_bwd_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "ob_relattn_bwd": (
        _int, [_c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _i64, _i64, _i64, _i64, _i64,
               _f32, _c_f, _i64, _c_f, _i64, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f, _sz, _c_f]),
    "ob_relattn_set_bwd_mode": (_int, [_int]),
    "ob_relattn_dropout_mask": (_int, [_i64, _i64, _f32, _c_f, _i64, _c_f, _c_f]),
    "ob_embedding_bwd": (_int, [_c_f, _i64, _c_f, _i64, _i64, _i64, _c_f, _c_f]),
    "ob_adamw_plan": (_i64, [_c_f, _i64, _c_f]),
    "ob_adamw_workspace": (_sz, [_i64]),
    "ob_adamw_clip_step": (
        _int, [_c_f, _i64, _c_f, _i64, _c_f, _c_f, _f32, _f64, _f64, _f64, _f64, _f64, _c_f, _c_f,
               _sz, _c_f]),
}

ABI_VERSION = 4  # 4 (round 6): ob_decattn_bwd consumes probs (dS' written there)

_lib = None


class OneBitHipError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Open the library once; raise if it is absent or its ABI does not match."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.is_file():
        raise OneBitHipError(
            f"{LIB_PATH} is missing: build it with `make -C cmu-11785-idl-1.58bit-asr_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback for the BitLinear path"
        )
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ob_abi_version() != ABI_VERSION:
        raise OneBitHipError(f"ABI mismatch: library {lib.ob_abi_version()} != {ABI_VERSION}")
    check_digest(lib)
    _lib = lib
    return lib


def check_digest(lib, expected: str | None = None) -> None:
    """Refuse a stale build: the library's compiled-in source digest must equal the digest of
    the sources next to it. Skipped for an explicitly chosen library (ONEBIT_HIP_LIB, e.g. an
    A/B baseline built from another tree) unless ``expected`` is given."""
    if expected is None:
        if os.environ.get("ONEBIT_HIP_LIB"):
            return
        if not _sources_present():
            # a packaged library without its sources: nothing to compare against
            import warnings

            warnings.warn(f"{LIB_PATH.name}: no csrc/ sources beside it; build digest not checked")
            return
        expected = source_digest()
    got = lib.ob_source_digest().decode()
    if got != expected:
        raise OneBitHipError(
            f"{LIB_PATH.name} was built from other sources (digest {got[:12]} != {expected[:12]} "
            "of csrc/ and include/): rebuild with `make -C cmu-11785-idl-1.58bit-asr_amd/csrc`")


def _sources_present() -> bool:
    csrc = Path(__file__).resolve().parents[1] / "csrc"
    return csrc.is_dir() and any(csrc.glob("*.hip"))


def ptr_array(ptrs):
    """A host array of device addresses for the C ABI's ``T* const*`` arguments; keep the
    returned object alive across the call and pass ``ctypes.addressof`` of it."""
    return (ctypes.c_void_p * len(ptrs))(*[p or None for p in ptrs])


def check(status: int, what: str) -> None:
    if status == OB_OK:
        return
    msg = load().ob_status_string(status).decode()
    if status == OB_ERR_BITWIDTH:
        raise ValueError("bitwidth must be one of {1,2,32}")
    raise OneBitHipError(f"{what}: {msg} (status {status})")


def ptr(t: "torch.Tensor | None") -> int | None:
    return None if t is None else t.data_ptr()


def source_digest() -> str:
    """sha256 over the library's sources (csrc/*.hip, csrc/*.h, include/*.h, file names
    included): identifies the kernel revision a build or a measurement (e.g. PMC traffic)
    belongs to; the library carries the value it was built from (ob_source_digest)."""
    from ._digest import source_digest as _sd

    return _sd()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream
