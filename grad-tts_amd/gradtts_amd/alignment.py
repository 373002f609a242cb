"""The alignment step of ``GradTTS.compute_loss`` (``model/tts.py:141-152``) on the gfx950 path.

``mas_alignment(mu_x, y, x_mask, y_mask)`` computes the log-prior of the encoder means ``mu_x [B, n_feats, Tx]``
against the mel-spectrogram ``y [B, n_feats, Ty]`` (the three fp32 contractions plus constant of tts.py:143-149),
masks it with ``x_mask (x) y_mask`` (tts.py:141) and runs ``maximum_path`` on device (tts.py:151) -- one C-ABI call
(``gt_log_prior_maximum_path``), no host round trip (the reference copies to numpy, monotonic_align/__init__.py:16).
Returns ``attn [B, Tx, Ty]`` (0/1, mu_x.dtype) and, on request, the masked log-prior. Masks are ``[B, 1, Tx]`` /
``[B, 1, Ty]`` (sequence_mask(...).unsqueeze(1), tts.py:139-140) or ``[B, Tx]`` / ``[B, Ty]``.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib


@torch.no_grad()
def mas_alignment(mu_x, y, x_mask, y_mask, return_log_prior=False):
    if not torch.cuda.is_available():
        raise RuntimeError("gradtts_amd.alignment needs a HIP (MI355X) device; there is no CPU path")
    device = mu_x.device if mu_x.is_cuda else torch.device("cuda", torch.cuda.current_device())
    B, F, Tx = mu_x.shape
    Ty = y.shape[-1]
    if y.shape != (B, F, Ty):
        raise ValueError(f"y must be [B, {F}, Ty], got {tuple(y.shape)}")
    mu32 = mu_x.to(device, torch.float32).contiguous()
    y32 = y.to(device, torch.float32).contiguous()
    xm = x_mask.reshape(B, Tx).to(device, torch.float32).contiguous()
    ym = y_mask.reshape(B, Ty).to(device, torch.float32).contiguous()
    paths = torch.empty((B, Tx, Ty), dtype=torch.int32, device=device)
    lp = torch.empty((B, Tx, Ty), dtype=torch.float32, device=device) if return_log_prior else None
    with torch.cuda.device(device):
        ws = torch.empty(lib().gt_alignment_workspace_bytes(B, Tx, Ty), dtype=torch.uint8, device=device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        check(lib().gt_log_prior_maximum_path(mu32.data_ptr(), y32.data_ptr(), xm.data_ptr(), ym.data_ptr(), B, F, Tx,
                                              Ty, paths.data_ptr(), lp.data_ptr() if lp is not None else None,
                                              ws.data_ptr(), ws.numel(), stream), "gt_log_prior_maximum_path")
    attn = paths.to(device=mu_x.device, dtype=mu_x.dtype)
    return (attn, lp) if return_log_prior else attn
