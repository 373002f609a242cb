"""ORACLE (test infrastructure only) -- CPU restatement of the Grad-TTS reverse-diffusion decoder.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline. The product path
(``grad-tts_amd/gradtts_amd``) never calls into ``oracle/``.

This is a functional (module-free) restatement of ``/root/reference/model/diffusion.py`` in plain
torch CPU ops over a ``{state_dict key: tensor}`` dict. Each function cites the reference lines it
follows. It is pinned against golden vectors generated from the real reference
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; test ``tests/test_oracle_golden.py``).

dtype: float32 by default (parity gate fp32 max|d| <= 1e-4 * max|ref|), float64 for the
tolerance envelope.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

HEADS, DIM_HEAD, GROUPS = 4, 32, 8


def mish(x):
    """``Mish`` diffusion.py:16-18: x * tanh(softplus(x)) (softplus beta=1, threshold=20)."""
    return x * torch.tanh(F.softplus(x))


def sinusoidal_pos_emb(t, dim, scale):
    """``SinusoidalPosEmb`` diffusion.py:113-125."""
    half = dim // 2
    emb = math.log(10000) / (half - 1)
    emb = torch.exp(torch.arange(half, dtype=torch.float32) * -emb).to(t.device, t.dtype)
    emb = scale * t.unsqueeze(1) * emb.unsqueeze(0)
    return torch.cat((emb.sin(), emb.cos()), dim=-1)


def linear(p, key, x):
    return F.linear(x, p[key + ".weight"], p[key + ".bias"])


# GT_FP8 emulation (not in the reference): when set by fp8_activations(), the input of every 3x3 Block conv that runs
# on fp8 operands (fp8_operand_conv) is quantized by quantize_act_e4m3 before the conv (what csrc/conv.hip's A8 operand
# load does)
_ACT_Q = None
# oracle.emulate.product_storage: the estimator with the library's bf16 / fp8 storage points (test infrastructure)
_EMU = None


def fp8_operand_conv(cin, cout):
    """GT_FP8's fp8-operand Block convs: at least 32 input channels, except 64 -> 64 (level 0), which keeps bf16
    operands on conv64 (with the fp8 weights)."""
    return cin >= 32 and not (cin == 64 and cout == 64)


def block(p, key, x, mask, taps=None, tap_name=None):
    """``Block`` diffusion.py:49-58: Mish(GN8(conv3x3(x*mask))) * mask."""
    xin = x * mask
    if _ACT_Q is not None and fp8_operand_conv(xin.shape[1], p[key + ".block.0.weight"].shape[0]):
        xin = _ACT_Q(xin)
    y = F.conv2d(xin, p[key + ".block.0.weight"], p[key + ".block.0.bias"], padding=1)
    if taps is not None and tap_name:
        taps[tap_name] = y
    y = F.group_norm(y, GROUPS, p[key + ".block.1.weight"], p[key + ".block.1.bias"], eps=1e-5)
    return mish(y) * mask


def resnet_block(p, key, x, mask, t_emb, taps=None):
    """``ResnetBlock`` diffusion.py:61-79."""
    h = block(p, key + ".block1", x, mask, taps, key + ".pre1")
    tb = F.linear(mish(t_emb), p[key + ".mlp.1.weight"], p[key + ".mlp.1.bias"])
    h = h + tb.unsqueeze(-1).unsqueeze(-1)
    h = block(p, key + ".block2", h, mask, taps, key + ".pre2")
    if (key + ".res_conv.weight") in p:
        res = F.conv2d(x * mask, p[key + ".res_conv.weight"], p[key + ".res_conv.bias"])
    else:
        res = x * mask
    out = h + res
    if taps is not None:
        taps[key] = out
    return out


def linear_attention(p, key, x, taps=None):
    """``Residual(Rezero(LinearAttention))`` diffusion.py:39-46, 82-110."""
    b, c, hh, ww = x.shape
    qkv = F.conv2d(x, p[key + ".fn.fn.to_qkv.weight"])
    qkv = qkv.reshape(b, 3, HEADS, DIM_HEAD, hh * ww)
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    k = k.softmax(dim=-1)
    context = torch.einsum("bhdn,bhen->bhde", k, v)
    out = torch.einsum("bhde,bhdn->bhen", context, q)
    out = out.reshape(b, HEADS * DIM_HEAD, hh, ww)
    out = F.conv2d(out, p[key + ".fn.fn.to_out.weight"], p[key + ".fn.fn.to_out.bias"])
    y = out * p[key + ".fn.g"] + x
    if taps is not None:
        taps[key] = y
    return y


def estimator(p, x, mask, mu, t, spk=None, n_spks=1, pe_scale=1000.0, dim=64, taps=None):
    """``GradLogPEstimator2d.forward`` diffusion.py:174-216. x, mu: [B,80,T]; mask [B,1,T]; t [B].

    ``taps`` (optional dict) receives intermediate activations under the stage names the HIP library's
    probe uses (include/gradtts.h gt_estimator_probe).

    Inside ``oracle.emulate.product_storage(mode)`` this is the restatement with the HIP library's bf16 / fp8
    storage points instead (oracle/emulate.py)."""
    if _EMU is not None:
        return _EMU(p, x, mask, mu, t, spk, n_spks, pe_scale, dim, taps)
    s = None
    if spk is not None:
        s = F.linear(mish(linear(p, "spk_mlp.0", spk)), p["spk_mlp.2.weight"], p["spk_mlp.2.bias"])
    t_emb = sinusoidal_pos_emb(t, dim, pe_scale)
    t_emb = F.linear(mish(linear(p, "mlp.0", t_emb)), p["mlp.2.weight"], p["mlp.2.bias"])
    if n_spks < 2:
        h = torch.stack([mu, x], 1)
    else:
        h = torch.stack([mu, x, s.unsqueeze(-1).repeat(1, 1, x.shape[-1])], 1)
    mask = mask.unsqueeze(1)
    hiddens, masks = [], [mask]
    n_levels = 3
    for i in range(n_levels):
        m = masks[-1]
        h = resnet_block(p, f"downs.{i}.0", h, m, t_emb, taps)
        h = resnet_block(p, f"downs.{i}.1", h, m, t_emb, taps)
        h = linear_attention(p, f"downs.{i}.2", h, taps)
        hiddens.append(h)
        if i < n_levels - 1:   # Downsample (diffusion.py:30-36) on x*mask
            h = F.conv2d(h * m, p[f"downs.{i}.3.conv.weight"], p[f"downs.{i}.3.conv.bias"], stride=2, padding=1)
            if taps is not None:
                taps[f"downs.{i}.3"] = h
        else:                  # Identity(x*mask)
            h = h * m
        masks.append(m[:, :, :, ::2])
    masks = masks[:-1]
    m = masks[-1]
    h = resnet_block(p, "mid_block1", h, m, t_emb, taps)
    h = linear_attention(p, "mid_attn", h, taps)
    h = resnet_block(p, "mid_block2", h, m, t_emb, taps)
    for i in range(n_levels - 1):
        m = masks.pop()
        h = torch.cat((h, hiddens.pop()), dim=1)
        h = resnet_block(p, f"ups.{i}.0", h, m, t_emb, taps)
        h = resnet_block(p, f"ups.{i}.1", h, m, t_emb, taps)
        h = linear_attention(p, f"ups.{i}.2", h, taps)
        h = F.conv_transpose2d(h * m, p[f"ups.{i}.3.conv.weight"], p[f"ups.{i}.3.conv.bias"], stride=2, padding=1)
        if taps is not None:
            taps[f"ups.{i}.3"] = h
    h = block(p, "final_block", h, mask, taps, "final_block.pre")
    out = F.conv2d(h * mask, p["final_conv.weight"], p["final_conv.bias"])
    return (out * mask).squeeze(1)


def get_noise(t, beta_init, beta_term, cumulative=False):
    """``get_noise`` diffusion.py:219-224."""
    if cumulative:
        return beta_init * t + 0.5 * (beta_term - beta_init) * (t ** 2)
    return beta_init + (beta_term - beta_init) * t


@torch.no_grad()
def reverse_diffusion(p, z, mask, mu, n_timesteps, spk=None, n_spks=1, beta_min=0.05, beta_max=20.0,
                      pe_scale=1000.0, dim=64):
    """``Diffusion.reverse_diffusion`` diffusion.py:254-268 (deterministic Euler; ``stoc`` is ignored there)."""
    h = 1.0 / n_timesteps
    xt = z * mask
    for i in range(n_timesteps):
        t = (1.0 - (i + 0.5) * h) * torch.ones(z.shape[0], dtype=z.dtype)
        noise_t = get_noise(t.unsqueeze(-1).unsqueeze(-1), beta_min, beta_max)
        dxt = 0.5 * (mu - xt - estimator(p, xt, mask, mu, t, spk, n_spks, pe_scale, dim))
        dxt = dxt * noise_t * h
        xt = (xt - dxt) * mask
    return xt


def forward_diffusion(x0, mask, mu, t, z, beta_min=0.05, beta_max=20.0):
    """``Diffusion.forward_diffusion`` diffusion.py:244-252 with the noise ``z`` passed in (the reference draws it
    with torch.randn at :249-250)."""
    time = t.unsqueeze(-1).unsqueeze(-1)
    cum_noise = get_noise(time, beta_min, beta_max, cumulative=True)
    mean = x0 * torch.exp(-0.5 * cum_noise) + mu * (1.0 - torch.exp(-0.5 * cum_noise))
    variance = 1.0 - torch.exp(-cum_noise)
    xt = mean + z * torch.sqrt(variance)
    return xt * mask, z * mask


@torch.no_grad()
def loss_t(p, x0, mask, mu, t, z, spk=None, n_spks=1, beta_min=0.05, beta_max=20.0, pe_scale=1000.0, dim=64,
           n_feats=80):
    """``Diffusion.loss_t`` diffusion.py:274-281 (forward value) with the noise passed in."""
    xt, z = forward_diffusion(x0, mask, mu, t, z, beta_min, beta_max)
    time = t.unsqueeze(-1).unsqueeze(-1)
    cum_noise = get_noise(time, beta_min, beta_max, cumulative=True)
    noise_estimation = estimator(p, xt, mask, mu, t, spk, n_spks, pe_scale, dim)
    noise_estimation = noise_estimation * torch.sqrt(1.0 - torch.exp(-cum_noise))
    loss = torch.sum((noise_estimation + z) ** 2) / (torch.sum(mask) * n_feats)
    return loss, xt


def loss_t_grads(sd, x0, mask, mu, t, z, spk=None, n_spks=1, dtype=torch.float64, beta_min=0.05, beta_max=20.0):
    """``Diffusion.loss_t`` (diffusion.py:274-281) differentiated by torch.autograd in `dtype` (numpy inputs):
    returns (loss, {param name: grad}, d mu, d spk or None) -- the gradients ``loss.backward()`` gives the
    reference's training step (train.py:109-113)."""
    d = lambda a: torch.as_tensor(a).to(dtype)
    p = {k: torch.as_tensor(v).to(dtype).requires_grad_() for k, v in sd.items()}
    mu_t = d(mu).requires_grad_()
    spk_t = d(spk).requires_grad_() if n_spks != 1 and spk is not None else None
    x0_t, mask_t, t_t, z_t = d(x0), d(mask), d(t), d(z)
    with torch.enable_grad():
        xt, zm = forward_diffusion(x0_t, mask_t, mu_t, t_t, z_t, beta_min, beta_max)
        cum = get_noise(t_t[:, None, None], beta_min, beta_max, cumulative=True)
        ne = estimator(p, xt, mask_t, mu_t, t_t, spk_t, n_spks) * torch.sqrt(1.0 - torch.exp(-cum))
        loss = torch.sum((ne + zm) ** 2) / (torch.sum(mask_t) * 80)
        loss.backward()
    return float(loss.detach()), {k: (v.grad.numpy() if v.grad is not None else np.zeros(v.shape)) for k, v in p.items()}, \
        mu_t.grad.numpy(), (spk_t.grad.numpy() if spk_t is not None else None)


def grad_probe(name, shape):
    """Fixed pseudo-random direction of the gradient digests in tests/golden/loss_*.npz (make_golden_train_lik.py)."""
    seed = int.from_bytes(name.encode()[:8].ljust(8, b"\0"), "little") ^ 0x5EED
    return np.random.default_rng(seed).standard_normal(shape)


def grad_digest(grads, names):
    """(sum of squares, projection onto grad_probe) per parameter, in `names` order, fp64."""
    gsq = np.array([float((np.asarray(grads[k], np.float64) ** 2).sum()) for k in names])
    gproj = np.array([float((np.asarray(grads[k], np.float64) * grad_probe(k, np.shape(grads[k]))).sum())
                      for k in names])
    return gsq, gproj


def log_prior(mu_x, y, n_feats=80):
    """The log-prior that ``GradTTS.compute_loss`` aligns with MAS, model/tts.py:143-149 (three matmuls + const)."""
    const = -0.5 * math.log(2 * math.pi) * n_feats
    factor = -0.5 * torch.ones(mu_x.shape, dtype=mu_x.dtype)
    y_square = torch.matmul(factor.transpose(1, 2), y ** 2)
    y_mu_double = torch.matmul(2.0 * (factor * mu_x).transpose(1, 2), y)
    mu_square = torch.sum(factor * (mu_x ** 2), 1).unsqueeze(-1)
    return y_square - y_mu_double + mu_square + const


def to_torch_params(sd, dtype=torch.float32):
    return {k: torch.as_tensor(v).to(dtype) for k, v in sd.items()}


# ---- fp8 weights (BASELINE.json config 5) ----------------------------------------
# Not in the reference (which is fp32 throughout): the W8 build quantizes the 3x3 convs
# (``Block.block[0]``, diffusion.py:52), ``Downsample.conv`` (:33) and ``Upsample.conv`` (:24) to OCP
# e4m3 per output channel. Parity for that mode is "the reference run with the dequantized weights":
# fp8_params() returns the state dict with those weights replaced by q * scale.
E4M3_MAX = 448.0


def is_fp8_key(key):
    """The weights the W8 build stores as fp8 (include/gradtts.h GT_BF16_W8)."""
    return key.endswith(".block.0.weight") or (key.startswith(("downs.", "ups.")) and key.endswith(".3.conv.weight"))


def fp8_axis(key):
    """Output-channel axis: Conv2d [Cout, Cin, kh, kw] -> 0; ConvTranspose2d [Cin, Cout, kh, kw] -> 1."""
    return 1 if key.startswith("ups.") and key.endswith(".3.conv.weight") else 0


def quantize_e4m3(w, axis):
    """Per-output-channel e4m3: scale = amax / 448 in fp32 (1 for an all-zero channel),
    q = (w / scale).to(float8_e4m3fn) (round to nearest even). Returns (q as uint8 codes, scale [C])."""
    w = torch.as_tensor(w, dtype=torch.float32)
    red = tuple(d for d in range(w.dim()) if d != axis)
    amax = w.abs().amax(dim=red)
    scale = torch.where(amax > 0, amax / torch.tensor(E4M3_MAX, dtype=torch.float32), torch.ones_like(amax))
    shape = [1] * w.dim()
    shape[axis] = -1
    q = (w / scale.reshape(shape)).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale


def dequantize_e4m3(q, scale, axis):
    shape = [1] * q.dim()
    shape[axis] = -1
    return q.view(torch.float8_e4m3fn).to(torch.float32) * scale.reshape(shape)


def fp8_params(sd):
    """State dict as the W8 build sees it: fp8 weights dequantized to fp32, everything else unchanged."""
    out = {}
    for k, v in sd.items():
        v = torch.as_tensor(v, dtype=torch.float32)
        if is_fp8_key(k):
            ax = fp8_axis(k)
            q, s = quantize_e4m3(v, ax)
            v = dequantize_e4m3(q, s, ax)
        out[k] = v
    return out


def quantize_act_e4m3(x, block=32):
    """GT_FP8 conv-operand quantization (csrc/conv.hip store_item_a8): x [B, C, F, T] -> e4m3 values with one
    power-of-two scale 2^k per (utterance, position, block of 32 channels); k is the least integer with
    max|x| / 2^k <= 448 (clamped at -126; an all-zero block stays zero), q = (x / 2^k).to(float8_e4m3fn) * 2^k."""
    B, C, H, W = x.shape
    g = x.reshape(B, C // block, block, H, W)
    amax = g.abs().amax(dim=2, keepdim=True)
    m, e = torch.frexp(amax)                      # amax = m 2^e, m in [0.5, 1): 2m 2^(e-1), 2m in [1, 2)
    k = torch.where(2 * m > 1.75, e - 8, e - 9).clamp(min=-126)
    s = torch.ldexp(torch.ones_like(amax), k)
    return ((g / s).to(torch.float8_e4m3fn).to(x.dtype) * s).reshape(x.shape)


class fp8_activations:
    """Context: the oracle's Block convs see GT_FP8's quantized operands (use with fp8_params weights)."""

    def __enter__(self):
        global _ACT_Q
        self.prev, _ACT_Q = _ACT_Q, quantize_act_e4m3
        return self

    def __exit__(self, *exc):
        global _ACT_Q
        _ACT_Q = self.prev
        return False
