"""ORACLE (test infrastructure only) -- CPU restatement of ``GradTTS.compute_loss`` (model/tts.py:110-194),
differentiated by torch.autograd. Only ``tests/`` import it, as the checker. Pinned to
``tests/golden/tts_loss_*.npz``, which ``tests/golden/make_golden_tts_loss.py`` produced by running the reference.

compute_loss(...) follows tts.py line by line with the reference's random draws handed in (the crop offsets
``random.choice`` gives at :161-165, ``t`` of diffusion.py:284 and ``z`` of :249) and the MAS of :151 as a callable
(the C restatement oracle/mas.c in the tests):
  * encoder                 oracle.text_encoder.text_encoder (optionally with the library's dropout masks)
  * log-prior, MAS          :141-152  (oracle.decoder.log_prior; MAS on the masked fp32 log-prior, as
                                      monotonic_align/__init__.py:13-22 does)
  * dur_loss                :155-156 with utils.py:42-44
  * crop                    :159-181
  * mu_y                    :184-185
  * diff_loss               Diffusion.compute_loss -> loss_t (diffusion.py:274-287, t clamped to [1e-5, 1 - 1e-5])
  * prior_loss              :191-192
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import decoder as odec
from . import text_encoder as ote


def sequence_mask(length, max_length=None):
    """utils.py:6-10."""
    if max_length is None:
        max_length = length.max()
    x = torch.arange(int(max_length), dtype=length.dtype, device=length.device)
    return x.unsqueeze(0) < length.unsqueeze(1)


def compute_loss(enc_p, dec_p, tokens, x_lengths, y, y_lengths, offsets, out_size, t, z, mas, drop=None,
                 dtype=torch.float64):
    """enc_p / dec_p: {state_dict key: tensor} (leaf tensors; gradients accumulate on them). Returns
    (dur_loss, prior_loss, diff_loss, attn [B, Tx, Ty] before the crop)."""
    dev = enc_p["emb.weight"].device
    tokens = torch.as_tensor(tokens).to(dev)
    x_lengths = torch.as_tensor(x_lengths).to(dev)
    y_lengths = torch.as_tensor(y_lengths).to(dev)
    y = torch.as_tensor(y).to(dev, dtype)
    mu_x, logw, x_mask = ote.text_encoder(enc_p, tokens, x_lengths, drop=drop)
    y_max_length = y.shape[-1]
    y_mask = sequence_mask(y_lengths, y_max_length).unsqueeze(1).to(x_mask)
    attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
    with torch.no_grad():
        am = attn_mask.squeeze(1).cpu()
        lp = odec.log_prior(mu_x.detach().cpu(), y.cpu()) * am   # MAS on the host, as the reference's
        tx = am.sum(1)[:, 0].numpy().astype(np.int32)
        ty = am.sum(2)[:, 0].numpy().astype(np.int32)
        paths, _ = mas(lp.numpy().astype(np.float32), tx, ty)
        attn = torch.from_numpy(paths).to(dev, dtype)
    logw_ = torch.log(1e-8 + torch.sum(attn.unsqueeze(1), -1)) * x_mask
    dur_loss = torch.sum((logw - logw_) ** 2) / torch.sum(x_lengths)
    if out_size is not None:
        B = y.shape[0]
        attn_cut = torch.zeros(B, attn.shape[1], out_size, dtype=dtype, device=dev)
        y_cut = torch.zeros(B, y.shape[1], out_size, dtype=dtype, device=dev)
        y_cut_lengths = []
        for i in range(B):
            yl = int(y_lengths[i])
            ycl = out_size + min(yl - out_size, 0)
            y_cut_lengths.append(ycl)
            lo = int(offsets[i])
            y_cut[i, :, :ycl] = y[i, :, lo:lo + ycl]
            attn_cut[i, :, :ycl] = attn[i, :, lo:lo + ycl]
        y_mask = sequence_mask(torch.LongTensor(y_cut_lengths).to(dev)).unsqueeze(1).to(y_mask)
        attn_use, y = attn_cut, y_cut
    else:
        attn_use = attn
    mu_y = torch.matmul(attn_use.transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
    tt = torch.clamp(torch.as_tensor(t).to(dev, dtype), 1e-5, 1.0 - 1e-5)
    zz = torch.as_tensor(z).to(dev, dtype)
    xt, zm = odec.forward_diffusion(y, y_mask, mu_y, tt, zz)
    cum = odec.get_noise(tt[:, None, None], 0.05, 20.0, cumulative=True)
    ne = odec.estimator(dec_p, xt, y_mask, mu_y, tt) * torch.sqrt(1.0 - torch.exp(-cum))
    diff_loss = torch.sum((ne + zm) ** 2) / (torch.sum(y_mask) * 80)
    prior_loss = torch.sum(0.5 * ((y - mu_y) ** 2 + math.log(2 * math.pi)) * y_mask)
    prior_loss = prior_loss / (torch.sum(y_mask) * 80)
    return dur_loss, prior_loss, diff_loss, attn


def params(sd, dtype=torch.float64, device="cpu"):
    return {k: torch.as_tensor(v).to(device, dtype).requires_grad_() for k, v in sd.items()}
