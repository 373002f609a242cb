"""CPU restatement of the reference's text encoder and GradTTS.forward front-end -- TEST
INFRASTRUCTURE ONLY: imported by tests/ (never by the product). Pinned to tests/golden/te_*.npz, which
tests/golden/make_golden_tts.py produced by running the reference itself.

* layer_norm            model/text_encoder.py:11-29 (over channels, eps 1e-4)
* conv_relu_norm        :32-64   (prenet: 3 x [conv k5 (x*mask) -> LayerNorm -> ReLU], x + proj(x), *mask)
* duration_predictor    :67-93
* attention             :135-211 (relative keys/values within +-window_size, masked_fill -1e4)
* ffn, encoder          :220-282
* text_encoder          :321-335
* front_end             model/tts.py:86-101 with utils.py:6-39 (durations, y_lengths, generate_path, mu_y)
* dropout_keep          the library's training-dropout generator (csrc/textenc.h Drop): NOT a reference algorithm
                        (torch's dropout draws cannot be reproduced), restated so the training pass with dropout
                        can be checked mask for mask; ``text_encoder(..., drop=...)`` applies the reference's
                        dropouts (text_encoder.py:48, 166, 234-239, 258-280, 74-91) with these masks
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


M64 = (1 << 64) - 1


def dropout_keep(seed, site, idx, p):
    """Scale factor (1 / (1 - p) kept, 0 dropped) of the library's dropout for element indices `idx` (uint64 array):
    u = top 24 bits of splitmix64's finaliser over seed + site 0x9E37..15 + idx 0xD1B5..03 (mod 2^64), kept iff
    u >= round(p 2^24). p = 0: all ones."""
    idx = np.asarray(idx, dtype=np.uint64)
    if p <= 0:
        return np.ones(idx.shape)
    thr = max(1, int(p * 16777216.0 + 0.5))
    with np.errstate(over="ignore"):
        x = (np.uint64((seed + site * 0x9E3779B97F4A7C15) & M64) + idx * np.uint64(0xD1B54A32D192ED03))
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    u = (x >> np.uint64(40)).astype(np.int64)
    return np.where(u >= thr, 1.0 / (1.0 - p), 0.0)


class Dropouts:
    """The masks of one training pass: seed, p (encoder / duration predictor) and p_prenet, as the library uses
    them (sites: prenet 1-3, duration predictor 8-9, layer l: 16 + 8 l + {0 p_attn, 1 attention output, 2 FFN
    hidden, 3 FFN output}); element index = (b T + t) C + c for [B, C, T] activations, ((b H + h) T + i) T + j
    for p_attn."""

    def __init__(self, seed, p, p_prenet):
        self.seed, self.p, self.pp = seed, p, p_prenet

    def chan(self, site, x, p):   # x [B, C, T]
        B, C, T = x.shape
        idx = (np.arange(B)[:, None, None] * T + np.arange(T)[None, None, :]) * C + np.arange(C)[None, :, None]
        return x * torch.as_tensor(dropout_keep(self.seed, site, idx, p), dtype=x.dtype)

    def attn(self, site, pa):     # pa [B, H, T, T]
        idx = np.arange(pa.numel()).reshape(pa.shape)
        return pa * torch.as_tensor(dropout_keep(self.seed, site, idx, self.p), dtype=pa.dtype)


def layer_norm(x, g, b, eps=1e-4):
    mean = torch.mean(x, 1, keepdim=True)
    var = torch.mean((x - mean) ** 2, 1, keepdim=True)
    x = (x - mean) * torch.rsqrt(var + eps)
    return x * g.view(1, -1, 1) + b.view(1, -1, 1)


def conv(p, key, x, pad=None):
    w = p[key + ".weight"]
    return F.conv1d(x, w, p[key + ".bias"], padding=w.shape[-1] // 2 if pad is None else pad)


def ln(p, key, x):
    return layer_norm(x, p[key + ".gamma"], p[key + ".beta"])


def attention(p, key, x, attn_mask, n_heads=2, window=4, drop=None, site=0):
    q, k, v = conv(p, key + "conv_q", x), conv(p, key + "conv_k", x), conv(p, key + "conv_v", x)
    b, d, t = k.shape
    kc = d // n_heads
    q = q.view(b, n_heads, kc, t).transpose(2, 3)
    k = k.view(b, n_heads, kc, t).transpose(2, 3)
    v = v.view(b, n_heads, kc, t).transpose(2, 3)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(kc)
    # relative position j - i within +-window (embeddings zero outside): scores_local[i, j] = q_i . E_k[j - i + W]
    idx = torch.arange(t, device=q.device)
    rel = idx[None, :] - idx[:, None]
    inside = rel.abs() <= window
    Ek = p[key + "emb_rel_k"][0]                       # [2W+1, kc]
    Ev = p[key + "emb_rel_v"][0]
    Ek_full = Ek[(rel.clamp(-window, window) + window)]   # [t, t, kc]
    rl = torch.einsum("bhic,ijc->bhij", q, Ek_full) * inside
    scores = scores + rl / math.sqrt(kc)
    scores = scores.masked_fill(attn_mask == 0, -1e4)
    pa = torch.softmax(scores, dim=-1)
    if drop is not None:
        pa = drop.attn(site, pa)                        # MultiHeadAttention.drop(p_attn) (:166)
    out = torch.matmul(pa, v)
    Ev_full = Ev[(rel.clamp(-window, window) + window)] * inside[..., None]
    out = out + torch.einsum("bhij,ijc->bhic", pa, Ev_full)
    out = out.transpose(2, 3).contiguous().view(b, d, t)
    return conv(p, key + "conv_o", out)


def text_encoder(p, tokens, x_lengths, n_layers=6, n_heads=2, window=4, drop=None):
    """drop: None (eval semantics) or a Dropouts (train mode with the library's masks). The duration predictor
    reads x.detach() (:332)."""
    D = (lambda site, v, q: drop.chan(site, v, q)) if drop is not None else (lambda site, v, q: v)
    pe, pp = (drop.p, drop.pp) if drop is not None else (0.0, 0.0)
    C = p["emb.weight"].shape[1]
    x = p["emb.weight"][tokens] * math.sqrt(C)
    x = x.transpose(1, -1)
    T = x.shape[2]
    x_mask = (torch.arange(T, device=x.device)[None] < x_lengths[:, None]).unsqueeze(1).to(x.dtype)
    x_org = x
    for i in range(3):                                  # ConvReluNorm (prenet)
        x = conv(p, f"prenet.conv_layers.{i}", x * x_mask)
        x = D(1 + i, torch.relu(ln(p, f"prenet.norm_layers.{i}", x)), pp)
    x = (x_org + conv(p, "prenet.proj", x)) * x_mask
    attn_mask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
    for l in range(n_layers):                           # Encoder
        site = 16 + 8 * l
        x = x * x_mask
        y = attention(p, f"encoder.attn_layers.{l}.", x, attn_mask, n_heads, window, drop, site)
        x = ln(p, f"encoder.norm_layers_1.{l}", x + D(site + 1, y, pe))
        f = f"encoder.ffn_layers.{l}."
        hdn = D(site + 2, torch.relu(conv(p, f + "conv_1", x * x_mask)), pe)
        y = conv(p, f + "conv_2", hdn * x_mask) * x_mask
        x = ln(p, f"encoder.norm_layers_2.{l}", x + D(site + 3, y, pe))
    x = x * x_mask
    mu = conv(p, "proj_m", x) * x_mask
    x = x.detach()
    d = torch.relu(conv(p, "proj_w.conv_1", x * x_mask))
    d = D(8, ln(p, "proj_w.norm_1", d), pe)
    d = torch.relu(conv(p, "proj_w.conv_2", d * x_mask))
    d = D(9, ln(p, "proj_w.norm_2", d), pe)
    logw = conv(p, "proj_w.proj", d * x_mask) * x_mask
    return mu, logw, x_mask


def front_end(mu_x, logw, x_mask, length_scale=1.0):
    """tts.py:86-101: (w_ceil, y_lengths, y_max_length, y_mask, attn, mu_y)."""
    w = torch.exp(logw) * x_mask
    w_ceil = torch.ceil(w) * length_scale
    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
    y_max_length = int(y_lengths.max())
    ty = y_max_length
    while ty % 4:
        ty += 1
    y_mask = (torch.arange(ty, device=mu_x.device)[None] < y_lengths[:, None]).unsqueeze(1).to(x_mask.dtype)
    attn_mask = (x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1)
    cum = torch.cumsum(w_ceil.squeeze(1), 1)
    path = (torch.arange(ty, device=mu_x.device)[None, None, :] < cum[:, :, None]).to(x_mask.dtype)
    path = path - F.pad(path, (0, 0, 1, 0))[:, :-1]
    attn = (path * attn_mask).unsqueeze(1)
    mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
    return w_ceil, y_lengths, y_max_length, y_mask, attn, mu_y


def to_torch_params(sd, dtype=torch.float32):
    return {k: torch.as_tensor(v).to(dtype) for k, v in sd.items()}
