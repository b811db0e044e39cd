"""ctypes binding of libica_hip.so — the C-ABI boundary (include/ica_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950) and
travels with the repo.  There is NO fallback: if the library is missing or a
call returns non-zero, this raises.  torch must be imported first so that the
HIP runtime torch bundles (soname libamdhip64.so.7) is the one the library
binds to (single runtime, shared streams).
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ICA_HIP_LIB", os.path.join(_HERE, "libica_hip.so"))

_p = C.c_void_p
_i = C.c_int
_l = C.c_long
_f = C.c_float
_sz = C.c_size_t

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "ica_conv_it": [_i],
    "ica_pack_conv_weight_size": [_i, _i, _i, _i, _i],
    "ica_pack_conv_weight": [_p, _p, _i, _i, _i, _l, _l, _i, _i, _i, _i, _p],
    "ica_pack_conv_weight_bf16": [_p, _p, _i, _i, _i, _l, _l, _i, _i, _i, _p],
    "ica_pack_conv_weight_bf16_size": [_i, _i, _i, _i],
    "ica_pack_conv_weight_x6": [_p, _p, _i, _i, _i, _l, _l, _i, _i, _p],
    "ica_pack_conv_weight_x6_size": [_i, _i, _i, _i],
    "ica_pack_gdn_x6": [_p, _p, _i, _p],
    "ica_pack_gdn_x6_size": [_i],
    "ica_pack_up3_bf16": [_p, _p, _i, _p],
    "ica_pack_up3_x6": [_p, _p, _i, _p],
    "ica_pack_up3k3_x6_size": [_i],
    "ica_pack_up3k3_x6": [_p, _p, _p, _i, _p],
    "ica_conv_up3k3_x6": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p],
    "ica_conv_up3_x6": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "ica_conv_up3_bf16": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "ica_conv_ex": [_p, _p],
    "ica_last_launch": [_p, _i, _p],
    "ica_pack_gdn": [_p, _p, _p, _p, _i, _i, _f, _p],
    "ica_pack_gdn_bf16": [_p, _p, _p, _p, _i, _i, _f, _p],
    "ica_pack_up3_size": [_i],
    "ica_pack_up3": [_p, _p, _i, _p],
    "ica_conv_up3": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "ica_conv_down": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p],
    "ica_conv_up": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p],
    "ica_elem_blocks_per_image": [],
    "ica_nchw_to_nc4": [_p, _p, _i, _i, _i, _i, _p],
    "ica_nc4_to_nchw": [_p, _p, _i, _i, _i, _i, _p],
    "ica_reduce_rows": [_p, _p, _i, _i, _f, _p],
    "ica_attack_prologue": [_p, _p, _p, _p, _i, _i, _i, _f, _p],
    "ica_attack_prologue_ex": [_p, _p, _p, _p, _i, _i, _i, _f, _i, _p],
    "ica_attack_loss": [_p, _p, _p, _p, _i, _i, _i, _f, _i, _i, _p],
    "ica_attack_adam": [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _f, _f, _f, _p, _p, _p, _p],
    "ica_attack_adam_ex": [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _f, _f, _f, _p, _p, _p, _i, _p],
    "ica_branch_select": [_p, _f, _i, _p, _p, _p],
    "ica_gather_images": [_p, _p, _p, _i, _l, _p],
    "ica_roi_prologue": [_p, _p, _p, _p, _i, _i, _i, _f, _i, _i, _i, _i, _f, _f, _p],
    "ica_roi_loss": [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _f, _f, _i, _p],
    "ica_roi_adam": [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _f, _f, _p, _i, _i, _i, _i, _f, _f, _p, _p, _p],
    "ica_ifgsm_step": [_p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _i, _p],
    "ica_l1_partial": [_p, _p, _i, _i, _i, _p],
    "ica_gc_likelihood": [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "ica_eb_likelihood": [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "ica_pack_eb": [_p, _p, _p, _i, _p],
    "ica_abs": [_p, _p, _l, _p],
    "ica_cast_f32_bf16": [_p, _p, _l, _p],
    "ica_cast_bf16_f32": [_p, _p, _l, _p],
    # eval-time defences (ica_defend.hip)
    "ica_flip_rot": [_p, _p, _l, _i, _i, _i, _p],
    "ica_bitdepth": [_p, _p, _l, _f, _p],
    "ica_resample_axis": [_p, _p, _l, _i, _i, _i, _i, _p, _p, _p, _i, _p],
    "ica_bitdepth_noise": [_p, _p, _p, _l, _f, _p],
    "ica_bitdepth_noise_bwd": [_p, _p, _l, _f, _p],
    "ica_add": [_p, _p, _p, _l, _p],
    "ica_ensemble_grad": [_p, _p, _p, _l, _f, _p],
    "ica_gc_symbols": [_p, _p, _p, _p, _i, _f, _p, _p, _i, _i, _i, _i, _p],
    "ica_eb_symbols": [_p, _p, _p, _p, _i, _i, _i, _i, _p],
    "ica_dequantize": [_p, _p, _p, _p, _i, _i, _i, _i, _p],
    "ica_pmf_to_quantized_cdf": [_p, _i, _i, _p],
    "ica_rans_encode": [_p, _p, _l, _p, _i, _p, _p, _i, _p, _l, _p],
    "ica_rans_decode": [_p, _l, _p, _l, _p, _i, _p, _p, _i, _p],
    "ica_rans_dec_open": [_p, _l, _p],
    "ica_rans_dec_step": [_p, _i, _p, _l, _p, _i, _p, _p, _i, _p, _p],
    "ica_rans_dec_close": [_p],
    # autoregressive coding of the context models (ica_ar.hip)
    "ica_ar_lds_bytes": [_i, _i, _i],
    "ica_ar_step": [_p, _i, _i, _i, _p],
    "ica_round": [_p, _p, _l, _p],
    "ica_clamp01": [_p, _p, _l, _p],
    "ica_sqdiff_partial": [_p, _p, _p, _i, _l, _i, _p],
    "ica_nc4_bound_to_nchw": [_p, _p, _i, _i, _i, _i, _p],
    "ica_bound_bwd_nc4": [_p, _p, _p, _i, _i, _i, _i, _p],
    "ica_msssim_blocks": [_i, _i, _i, _i],
    "ica_msssim_level": [_p, _p, _i, _i, _i, _p, _i, _i, _f, _f, _p, _p, _p, _p, _p],
    "ica_msssim_level_bwd": [_p, _p, _p, _i, _i, _i, _p, _i, _i, _p, _p, _p],
    "ica_msssim_combine": [_p, _i, _i, _i, _p, _p, _p, _p, _p],
    "ica_avgpool2": [_p, _p, _i, _i, _i, _i, _i, _p],
    "ica_avgpool2_bwd": [_p, _p, _i, _i, _i, _i, _i, _p],
    "ica_scale": [_p, _l, _f, _p],
    # training side (ica_train.hip)
    "ica_wgrad_ws_size": [_i, _i, _i, _i],
    "ica_wgrad_nsplit": [_i, _i, _l],
    "ica_wgrad": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p],
    "ica_channel_sum": [_p, _p, _i, _i, _i, _i, _i, _p],
    "ica_relu_bwd": [_p, _p, _l, _p],
    "ica_abs_bwd": [_p, _p, _l, _p],
    "ica_gdn_xsq": [_p, _p, _p, _l, _p],
    "ica_lrelu_bwd": [_p, _p, _p, _l, _p],
    "ica_gdn_t": [_p, _p, _p, _p, _l, _i, _p],
    "ica_reparam_bwd": [_p, _p, _p, _l, _f, _i, _p],
    "ica_bpp_grad": [_p, _p, _l, _f, _p],
    "ica_gc_bwd": [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p],
    "ica_eb_bwd": [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p],
    "ica_eb_param_scatter": [_p, _p, _p, _i, _p],
    "ica_mse_grad": [_p, _p, _p, _i, _i, _i, _f, _p],
}
_RESTYPES = {"ica_pack_conv_weight_size": _sz, "ica_pack_conv_weight_bf16_size": _sz,
             "ica_pack_conv_weight_x6_size": _sz, "ica_pack_gdn_x6_size": _sz, "ica_pack_up3k3_x6_size": _sz, "ica_pack_up3_size": _sz, "ica_wgrad_ws_size": _sz,
             "ica_rans_encode": _l, "ica_ar_lds_bytes": _sz}



class ConvArgs(C.Structure):
    """include/ica_hip.h ica_conv_args."""
    _fields_ = ([(n, C.c_void_p) for n in ("x", "y", "wp", "bias", "gp", "beta", "save_x", "save_s", "in_x", "in_s",
                                            "save_t", "res", "mask")]
                + [(n, C.c_int) for n in ("N", "Cin", "Hin", "Win", "Cout", "Hout", "Wout", "kind", "KS", "S", "epi",
                                           "it", "fill_mode", "ps", "prec", "layout")])


class ArArgs(C.Structure):
    """include/ica_hip.h ica_ar_args."""
    _fields_ = ([(n, C.c_void_p) for n in ("y", "params", "yhat", "sym", "idx", "sym_in", "means", "wc", "bc", "w1",
                                            "b1", "w2", "b2", "w3", "b3", "table")]
                + [("T", C.c_int), ("bound", C.c_float)]
                + [(n, C.c_int) for n in ("B", "M", "H", "W", "E1", "E2")])


_lib = None


def lib():
    """Load (once) and return the ctypes library; raises if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libica_hip.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
                "There is no CPU/PyTorch fallback for the hot path.")
        L = C.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, _i)
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)
