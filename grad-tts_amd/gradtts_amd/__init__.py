"""gradtts_amd -- MI355X-native (gfx950) Grad-TTS reverse-diffusion decoder and monotonic alignment.

Drop-in for the reference hot path:
    from gradtts_amd.diffusion import Diffusion, GradLogPEstimator2d     # model/diffusion.py
    from gradtts_amd.monotonic_align import maximum_path                 # model/monotonic_align
The compute lives in libgradtts.so (C ABI: include/gradtts.h); see DESIGN.md.
"""
from .params import estimator_param_shapes, synthetic_state_dict, fix_len_compatibility  # noqa: F401

__all__ = ["estimator_param_shapes", "synthetic_state_dict", "fix_len_compatibility"]
