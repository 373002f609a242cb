"""ORACLE (test infrastructure only) -- the decoder restatement with the HIP library's storage points.

Only ``tests/`` (and ``__graft_entry__.smoke()`` / ``bench.py``'s ``cpu_baseline`` through ``oracle.decoder``) use
this, as the checker; the product path never imports ``oracle/``.

``oracle.decoder`` restates ``model/diffusion.py`` in fp32 (pinned to the reference's golden vectors). The library's
bf16 / fp8 modes compute the same algorithm but keep every activation between kernels in bf16 and run their convs on
bf16 (or, GT_FP8, e4m3) operands, so against the fp32 restatement a bf16 call sits ~2^-9 away -- and an fp8 call
much further, because a bf16 rounding moves a value across an e4m3 rounding boundary (a 2^-3 step) for about 1 in 32
operands, and those flips, not the arithmetic, set the distance. This module makes the restatement round where the
library rounds, so the GPU can be pinned against it at fp32-summation-order distance instead:

* every stored activation -- a Block conv's output (csrc/conv3w.hip / conv64.hip / conv.hip epilogues), a ResnetBlock
  output (rbout passes, attn_kv's RB form, conv64 IN_RB0), an attention output (conv_kernel OUT_RESID), a
  Down/Upsample output -- is bf16 (round to nearest even); the GroupNorm statistics of a conv output are those of its
  fp32 values (the epilogues sum before rounding), applied to the stored bf16 copy -- except the single-speaker
  U-Net input conv, whose output block2's conv recomputes instead of reading (conv64 IN_X0), so its GroupNorm
  normalises the fp32 values;
* a bf16 conv's operand is the bf16 rounding of its fp32 operand value (masked input, or (Mish(GN(h)) + tb) * m); an
  fp8-operand conv (GT_FP8, ``decoder.fp8_operand_conv``) quantizes that fp32 value straight to e4m3
  (``decoder.quantize_act_e4m3``: conv3w_a8.hip finish_item / conv.hip store_item_a8);
* weights: the Block, Downsample and Upsample convs' and the non-input res_convs' in bf16 (bf16 mode) or the e4m3
  dequantized ones (fp8 modes, ``decoder.fp8_params`` already applied by the caller); the attention's k / v projection
  rows in bf16; the input block's res_conv, the attention's q rows, to_out, final_conv, the MLPs in fp32, as the
  library packs them (csrc/decoder.cpp prepare);
* LinearAttention as attn_kv / attn_merge / attn_fold compute it (csrc/attn.hip): per tile of the utterance's
  flattened positions (decoder.cpp attn_tiles, by tile plan) an online softmax over 64-position sub-blocks in log2
  units, exp values and v rounded to bf16 for the context MFMA, the sums in fp32; tiles merged by their maxima;
  M_b = g W_out blockdiag(ctx^T) W_q in fp32, rounded to bf16 as the per-utterance 1x1 weight image; y = x + M_b x +
  g b_out, stored in bf16.
What remains between the GPU and this restatement is fp32 summation order and the library's exp2 / rcp forms of
Mish, GroupNorm and softmax: ~1e-6 of a value, which flips a bf16 or e4m3 rounding only for the rare value that lies
that close to a boundary.
"""
from __future__ import annotations

import math
from contextlib import contextmanager

import torch
import torch.nn.functional as F

from oracle import decoder as D

L2E = 1.44269504088896341


def r16(t):
    """bf16 storage: round to nearest even, held in the tensor's own dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


def attn_tiles(n, target):
    """decoder.cpp attn_tiles: positions per tile (a multiple of 64) and tiles per utterance."""
    tp = (n + target - 1) // target
    tp = max(64, (tp + 63) // 64 * 64)
    return tp, (n + tp - 1) // tp


class _Cfg:
    mode = None      # None | "bf16" | "bf16_w8" | "fp8"
    small = None     # tile plan: True small-batch, False throughput, None: decided by the batch (B <= 4)


@contextmanager
def product_storage(mode, small=None):
    """Within the context, ``oracle.decoder.estimator`` (and so ``reverse_diffusion``) computes with the library's
    storage points for compute mode ``mode`` ("bf16", "bf16_w8" or "fp8"; pass ``decoder.fp8_params`` weights for the
    fp8 modes). ``small``: the attention tile plan (None: the library's choice, B <= 4 -> small)."""
    assert mode in ("bf16", "bf16_w8", "fp8")
    prev = (_Cfg.mode, _Cfg.small)
    _Cfg.mode, _Cfg.small = mode, small
    D._EMU = estimator
    try:
        yield
    finally:
        _Cfg.mode, _Cfg.small = prev
        D._EMU = None if prev[0] is None else estimator


def _conv_w(p, key):
    """A Block / Down / Up / res_conv weight as the library holds it."""
    w = p[key]
    if _Cfg.mode != "bf16" and D.is_fp8_key(key):
        return w   # e4m3 dequantized by the caller (fp8_params); the library scales the accumulator, same value
    return r16(w)


def _gn_stored(y, gamma, beta, stored=True):
    """GroupNorm(8) of the bf16-stored y with the statistics of the fp32 y (conv epilogue partial sums, reduced in
    fp64: csrc/common.h gn_reduce). stored=False: y is never stored (the U-Net input conv recomputed by its consumer,
    conv64 IN_X0), so the normalised values are the fp32 ones."""
    B = y.shape[0]
    yg = y.reshape(B, D.GROUPS, -1).double()
    mean = yg.mean(-1)
    var = (yg * yg).mean(-1) - mean * mean
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    ys = (r16(y) if stored else y).reshape(B, D.GROUPS, -1).double()
    n = ((ys - mean[..., None]) * rstd[..., None]).reshape(y.shape)
    shp = (1, -1, 1, 1)
    return (n * gamma.double().reshape(shp) + beta.double().reshape(shp)).to(y.dtype)


def _block(p, key, xop, mask, taps, tap_name, a8, stored=True):
    """``Block`` (diffusion.py:49-58) on the fp32 operand value xop (already masked): bf16 operand or e4m3 (a8); the
    conv output stored in bf16 (tap), GroupNorm with the fp32 statistics, Mish, mask. stored=False: the output is
    recomputed by its consumer instead of stored (GroupNorm + Mish of the fp32 values; the tap is still bf16, as the
    library's diagnostic probe writes it)."""
    xin = D.quantize_act_e4m3(xop) if a8 else r16(xop)
    y = F.conv2d(xin, _conv_w(p, key + ".block.0.weight"), p[key + ".block.0.bias"], padding=1)
    if taps is not None and tap_name:
        taps[tap_name] = r16(y)
    return D.mish(_gn_stored(y, p[key + ".block.1.weight"], p[key + ".block.1.bias"], stored)) * mask


def _resnet(p, key, x, mask, t_emb, taps, first):
    """``ResnetBlock`` (diffusion.py:61-79); x is stored (bf16) except for the input block (fp32 mu, x_t, spk)."""
    cin, cout = x.shape[1], p[key + ".block1.block.0.weight"].shape[0]
    fp8 = _Cfg.mode == "fp8"
    # the single-speaker input block recomputes h1 inside block2's conv (decoder.cpp x0_fused): never stored
    fused_x0 = first and cin == 2 and cout == 64 and x.shape[2] % 20 == 0
    h = _block(p, key + ".block1", x * mask, mask, taps, key + ".pre1", fp8 and D.fp8_operand_conv(cin, cout),
               stored=not fused_x0)
    tb = F.linear(D.mish(t_emb), p[key + ".mlp.1.weight"], p[key + ".mlp.1.bias"])
    h = (h + tb.unsqueeze(-1).unsqueeze(-1)) * mask
    h = _block(p, key + ".block2", h, mask, taps, key + ".pre2", fp8 and D.fp8_operand_conv(cout, cout))
    if (key + ".res_conv.weight") in p:
        w = p[key + ".res_conv.weight"] if first else r16(p[key + ".res_conv.weight"])   # input block: fp32 FMAs
        res = F.conv2d(x * mask, w, p[key + ".res_conv.bias"])
    else:
        res = x * mask
    out = r16(h + res)
    if taps is not None:
        taps[key] = out
    return out


def _attention(p, key, x, taps):
    """``Residual(Rezero(LinearAttention))`` (diffusion.py:39-46, 82-110) as csrc/attn.hip computes it."""
    B, C, H, W = x.shape
    n = H * W
    w = p[key + ".fn.fn.to_qkv.weight"]
    wq, wk, wv = w[:128], r16(w[128:256]), r16(w[256:384])
    k = F.conv2d(x, wk).reshape(B, D.HEADS, D.DIM_HEAD, n)
    v = F.conv2d(x, wv).reshape(B, D.HEADS, D.DIM_HEAD, n)
    small = _Cfg.small if _Cfg.small is not None else B <= 4
    tp, nt = attn_tiles(n, 256 if small else (16 if n >= 8192 else 32))
    npad = tp * nt
    ka = F.pad(k, (0, npad - n), value=-math.inf)                           # padded positions: no part in the softmax
    vp = F.pad(v, (0, npad - n))
    nsb = tp // 64
    ka = ka.reshape(B, D.HEADS, D.DIM_HEAD, nt, nsb, 64)
    vp = vp.reshape(B, D.HEADS, D.DIM_HEAD, nt, nsb, 64)
    # running maximum of each tile over its 64-position sub-blocks in log2 units, mL = fl(max a * log2 e) (attn_kv)
    mrun = torch.cummax((ka.amax(-1).double() * L2E).float(), dim=-1).values   # [B, h, d, nt, nsb]
    arg = (ka.double() * L2E - mrun[..., None].double()).float()           # fma(a, log2 e, -mL): one rounding
    e = torch.where(torch.isfinite(ka), torch.exp2(arg), torch.zeros_like(arg))
    l_sb = e.sum(-1)                                                        # fp32 sums of the unrounded values
    ctx_sb = torch.einsum("bhdtsn,bhetsn->bhdtse", r16(e), r16(vp))         # bf16 operands, fp32 accumulate
    mlast = mrun[..., -1:]
    scale = torch.exp2(mrun - mlast)                                        # rescales as the running max moved
    l_t = (l_sb * scale).sum(-1)                                            # [B, h, d, nt]
    ctx_t = (ctx_sb * scale[..., None]).sum(-2)                             # [B, h, d, nt, e]
    m_t = mlast[..., 0]
    M = m_t.amax(-1, keepdim=True)                                          # attn_merge
    wt = torch.exp2(m_t - M)
    ctx = (ctx_t * wt[..., None]).sum(-2) / (l_t * wt).sum(-1)[..., None]   # [B, h, d, e]
    g = p[key + ".fn.g"]
    wout = p[key + ".fn.fn.to_out.weight"].reshape(C, D.HEADS, D.DIM_HEAD)
    A = g * torch.einsum("che,bhde->bchd", wout, ctx).reshape(B, C, 128)     # g W_out blockdiag(ctx^T)
    Mb = r16(torch.einsum("bcj,ji->bci", A, wq.reshape(128, C)))            # attn_fold -> bf16 weight image
    gb = g * p[key + ".fn.fn.to_out.bias"]
    y = torch.einsum("boc,bcn->bon", Mb, x.reshape(B, C, n)).reshape(x.shape) + gb.reshape(1, -1, 1, 1) + x
    y = r16(y)
    if taps is not None:
        taps[key] = y
    return y


def estimator(p, x, mask, mu, t, spk=None, n_spks=1, pe_scale=1000.0, dim=64, taps=None):
    """``GradLogPEstimator2d.forward`` (diffusion.py:174-216) with the library's storage points (module docstring)."""
    s = None
    if spk is not None:
        s = F.linear(D.mish(D.linear(p, "spk_mlp.0", spk)), p["spk_mlp.2.weight"], p["spk_mlp.2.bias"])
    t_emb = D.sinusoidal_pos_emb(t, dim, pe_scale)
    t_emb = F.linear(D.mish(D.linear(p, "mlp.0", t_emb)), p["mlp.2.weight"], p["mlp.2.bias"])
    if n_spks < 2:
        h = torch.stack([mu, x], 1)
    else:
        h = torch.stack([mu, x, s.unsqueeze(-1).repeat(1, 1, x.shape[-1])], 1)
    mask = mask.unsqueeze(1)
    hiddens, masks = [], [mask]
    for i in range(3):
        m = masks[-1]
        h = _resnet(p, f"downs.{i}.0", h, m, t_emb, taps, first=(i == 0))
        h = _resnet(p, f"downs.{i}.1", h, m, t_emb, taps, first=False)
        h = _attention(p, f"downs.{i}.2", h, taps)
        hiddens.append(h)
        if i < 2:
            h = r16(F.conv2d(h * m, _conv_w(p, f"downs.{i}.3.conv.weight"), p[f"downs.{i}.3.conv.bias"], stride=2,
                             padding=1))
            if taps is not None:
                taps[f"downs.{i}.3"] = h
        else:
            h = h * m
        masks.append(m[:, :, :, ::2])
    masks = masks[:-1]
    m = masks[-1]
    h = _resnet(p, "mid_block1", h, m, t_emb, taps, first=False)
    h = _attention(p, "mid_attn", h, taps)
    h = _resnet(p, "mid_block2", h, m, t_emb, taps, first=False)
    for i in range(2):
        m = masks.pop()
        h = torch.cat((h, hiddens.pop()), dim=1)
        h = _resnet(p, f"ups.{i}.0", h, m, t_emb, taps, first=False)
        h = _resnet(p, f"ups.{i}.1", h, m, t_emb, taps, first=False)
        h = _attention(p, f"ups.{i}.2", h, taps)
        h = r16(F.conv_transpose2d(h * m, _conv_w(p, f"ups.{i}.3.conv.weight"), p[f"ups.{i}.3.conv.bias"],
                                   stride=2, padding=1))
        if taps is not None:
            taps[f"ups.{i}.3"] = h
    h = _block(p, "final_block", h * mask, mask, taps, "final_block.pre", False)
    out = F.conv2d(h, p["final_conv.weight"], p["final_conv.bias"])
    return (out * mask).squeeze(1)
