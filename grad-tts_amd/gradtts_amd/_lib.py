"""ctypes binding of the C ABI in include/gradtts.h (libgradtts.so, gfx950).

This is the binding a maintainer of the reference would add. There is no CPU
fallback: if the library is missing the import fails loudly, and every compute entry point needs
HIP device pointers.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRADTTS_LIB", os.path.join(_HERE, "libgradtts.so"))

GT_OK, GT_ERR_ARG, GT_ERR_HIP, GT_ERR_PARAM, GT_ERR_UNSUPPORTED, GT_ERR_WORKSPACE = range(6)
GT_F32, GT_BF16, GT_BF16_W8, GT_FP8 = 0, 1, 2, 3

# (name, restype, argtypes) for every symbol declared in include/gradtts.h
_c = ctypes
SIGNATURES = [
    ("gt_version", _c.c_char_p, []),
    ("gt_last_error", _c.c_char_p, []),
    ("gt_decoder_create", _c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_float, _c.c_float, _c.c_float,
                                     _c.POINTER(_c.c_void_p)]),
    ("gt_decoder_destroy", None, [_c.c_void_p]),
    ("gt_decoder_set_betas", _c.c_int, [_c.c_void_p, _c.c_float, _c.c_float]),
    ("gt_decoder_pack_count", _c.c_int64, [_c.c_void_p]),
    ("gt_decoder_set_params_device", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_void_p]),
    ("gt_decoder_num_params", _c.c_int, [_c.c_void_p]),
    ("gt_decoder_param_name", _c.c_char_p, [_c.c_void_p, _c.c_int]),
    ("gt_decoder_param_numel", _c.c_int64, [_c.c_void_p, _c.c_int]),
    ("gt_decoder_set_param", _c.c_int, [_c.c_void_p, _c.c_char_p, _c.c_void_p, _c.c_int64]),
    ("gt_decoder_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int, _c.c_int64, _c.c_int64, _c.c_int32]),
    ("gt_estimator_forward", _c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                        _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                        _c.c_void_p]),
    ("gt_reverse_diffusion", _c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                        _c.c_int64, _c.c_int64, _c.c_int32, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                        _c.c_void_p]),
    ("gt_estimator_probe", _c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                      _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_char_p, _c.c_void_p, _c.c_void_p,
                                      _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_decoder_set_graphs", _c.c_int, [_c.c_void_p, _c.c_int]),
    ("gt_decoder_graph_captures", _c.c_int64, [_c.c_void_p]),
    ("gt_decoder_set_small_batch", _c.c_int, [_c.c_void_p, _c.c_int64]),
    ("gt_decoder_set_wide_conv", _c.c_int, [_c.c_void_p, _c.c_int]),
    ("gt_decoder_profile_enable", _c.c_int, [_c.c_void_p, _c.c_int]),
    ("gt_decoder_profile_read", _c.c_int, [_c.c_void_p, _c.c_char_p, _c.c_size_t]),
    ("gt_decoder_profile_filter", _c.c_int, [_c.c_void_p, _c.c_char_p]),
    ("gt_f32_to_e4m3", _c.c_uint8, [_c.c_float]),
    ("gt_quantize_e4m3", _c.c_int, [_c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_void_p,
                                    _c.c_void_p]),
    ("gt_forward_diffusion", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                        _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    ("gt_diffusion_loss_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int, _c.c_int64, _c.c_int64]),
    ("gt_diffusion_loss_t", _c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                       _c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p,
                                       _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_train_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_decoder_grad_numel", _c.c_int64, [_c.c_void_p]),
    ("gt_diffusion_loss_grad", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 6 + [_c.c_int64, _c.c_int64] +
     [_c.c_void_p] * 5 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_estimator_vjp_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_estimator_vjp", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 6 + [_c.c_int64, _c.c_int64] +
     [_c.c_void_p] * 2 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_likelihood_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_likelihood_drift_div", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 6 + [_c.c_int64, _c.c_int64] +
     [_c.c_void_p] * 2 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_likelihood_euler", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 5 + [_c.c_int64, _c.c_int64, _c.c_int32] +
     [_c.c_void_p] * 2 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_text_encoder_create", _c.c_int, [_c.c_int] * 9 + [_c.c_void_p]),
    ("gt_text_encoder_destroy", None, [_c.c_void_p]),
    ("gt_text_encoder_num_params", _c.c_int, [_c.c_void_p]),
    ("gt_text_encoder_param_name", _c.c_char_p, [_c.c_void_p, _c.c_int]),
    ("gt_text_encoder_param_numel", _c.c_int64, [_c.c_void_p, _c.c_int]),
    ("gt_text_encoder_set_param", _c.c_int, [_c.c_void_p, _c.c_char_p, _c.c_void_p, _c.c_int64]),
    ("gt_text_encoder_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_text_encoder_forward", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 2 + [_c.c_int64, _c.c_int64] +
     [_c.c_void_p] * 3 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_durations", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_float] + [_c.c_void_p] * 4),
    ("gt_expand", _c.c_int, [_c.c_void_p] * 4 + [_c.c_int64] * 3 + [_c.c_int32] + [_c.c_void_p] * 4),
    ("gt_path_gather", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int32,
                                  _c.c_void_p, _c.c_void_p]),
    ("gt_text_encoder_set_params_device", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_void_p]),
    ("gt_text_encoder_train_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_text_encoder_grad_numel", _c.c_int64, [_c.c_void_p]),
    ("gt_text_encoder_forward_train", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 2 + [_c.c_int64, _c.c_int64] +
     [_c.c_float, _c.c_float, _c.c_uint64] + [_c.c_void_p] * 3 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_text_encoder_backward", _c.c_int, [_c.c_void_p] + [_c.c_void_p] * 2 + [_c.c_int64, _c.c_int64] +
     [_c.c_float, _c.c_float, _c.c_uint64] + [_c.c_void_p] + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_path_scatter", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int32,
                                   _c.c_void_p, _c.c_void_p]),
    ("gt_tts_aux_losses_workspace_bytes", _c.c_size_t, [_c.c_int64, _c.c_int64]),
    ("gt_tts_aux_losses", _c.c_int, [_c.c_void_p] * 4 + [_c.c_int64] * 3 + [_c.c_void_p] * 3 +
     [_c.c_int64, _c.c_int32] + [_c.c_void_p] * 3 + [_c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_vocoder_create", _c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p,
                                     _c.c_void_p, _c.c_void_p]),
    ("gt_vocoder_create2", _c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p,
                                      _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p]),
    ("gt_vocoder_destroy", None, [_c.c_void_p]),
    ("gt_vocoder_num_params", _c.c_int, [_c.c_void_p]),
    ("gt_vocoder_param_name", _c.c_char_p, [_c.c_void_p, _c.c_int]),
    ("gt_vocoder_param_numel", _c.c_int64, [_c.c_void_p, _c.c_int]),
    ("gt_vocoder_set_param", _c.c_int, [_c.c_void_p, _c.c_char_p, _c.c_void_p, _c.c_int64]),
    ("gt_vocoder_hop", _c.c_int64, [_c.c_void_p]),
    ("gt_vocoder_set_compute_dtype", _c.c_int, [_c.c_void_p, _c.c_int]),
    ("gt_vocoder_workspace_bytes", _c.c_size_t, [_c.c_void_p, _c.c_int64, _c.c_int64]),
    ("gt_vocoder_forward", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p,
                                      _c.c_size_t, _c.c_void_p]),
    ("gt_alignment_workspace_bytes", _c.c_size_t, [_c.c_int64, _c.c_int64, _c.c_int64]),
    ("gt_log_prior_maximum_path", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int64,
                                             _c.c_int64, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p,
                                             _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    ("gt_maximum_path_workspace_bytes", _c.c_size_t, [_c.c_int64, _c.c_int64, _c.c_int64]),
    ("gt_maximum_path", _c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64,
                                   _c.c_int64, _c.c_float, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
]

_lib = None


def lib():
    """Load libgradtts.so once (raises if it has not been built: `python grad-tts_amd/build.py`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `python grad-tts_amd/build.py` "
                              "(no CPU fallback exists for the decoder or MAS)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


OPS_PATH = os.path.join(_HERE, "libgradtts_ops.so")
_ops = None


def ops():
    """torch.ops.gradtts (TORCH_LIBRARY(gradtts) in libgradtts_ops.so, bound to this process's libgradtts.so).
    Raises if the op library has not been built (no fallback path)."""
    global _ops
    if _ops is None:
        import torch
        if not os.path.exists(OPS_PATH):
            raise ImportError(f"{OPS_PATH} not found: build it with `python grad-tts_amd/build.py`")
        lib()                                   # the C ABI first: the op library binds to the same file
        torch.ops.load_library(OPS_PATH)
        torch.ops.gradtts.bind(LIB_PATH)
        _ops = torch.ops.gradtts
    return _ops


class GradTTSError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != GT_OK:
        msg = lib().gt_last_error()
        raise GradTTSError(f"{what} failed (code {rc}): {msg.decode() if msg else ''}")
