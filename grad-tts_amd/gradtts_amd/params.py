"""Parameter inventory of the Grad-TTS score U-Net and a deterministic synthetic-weight generator.

The inventory enumerates the ``state_dict`` keys (and shapes) that the reference
``GradLogPEstimator2d`` registers, so checkpoints saved by the reference
(``train.py:174-175``) load into this package unchanged:

* ``spk_mlp.{0,2}``              -- ``model/diffusion.py:139-141`` (only if n_spks > 1 or n_spks == -1)
* ``mlp.{0,2}``                  -- ``model/diffusion.py:143-144``
* ``downs.{i}.{0,1,2,3}``        -- ``model/diffusion.py:146-158``
* ``mid_block1/mid_attn/mid_block2`` -- ``model/diffusion.py:160-163``
* ``ups.{i}.{0,1,2,3}``          -- ``model/diffusion.py:165-170``
* ``final_block``, ``final_conv`` -- ``model/diffusion.py:171-172``

No trained checkpoint exists in this environment, so tests and the
benchmark use :func:`synthetic_state_dict`: a framework-free numpy PCG64 stream that
reproduces bit-identically on every host with the same numpy.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

DIM_MULTS = (1, 2, 4)
HEADS = 4
DIM_HEAD = 32
GROUPS = 8


def level_dims(dim: int, n_spks: int):
    """Channel plan ``dims`` of ``model/diffusion.py:146``."""
    cin = 2 + (1 if n_spks > 1 else 0)
    return [cin] + [dim * m for m in DIM_MULTS]


def uses_spk_mlp(n_spks: int) -> bool:
    """``model/diffusion.py:139``: the speaker MLP exists for n_spks > 1 or n_spks == -1."""
    return n_spks > 1 or n_spks == -1


def _resnet(prefix, din, dout, dim, out):
    out[prefix + "mlp.1.weight"] = (dout, dim)
    out[prefix + "mlp.1.bias"] = (dout,)
    out[prefix + "block1.block.0.weight"] = (dout, din, 3, 3)
    out[prefix + "block1.block.0.bias"] = (dout,)
    out[prefix + "block1.block.1.weight"] = (dout,)
    out[prefix + "block1.block.1.bias"] = (dout,)
    out[prefix + "block2.block.0.weight"] = (dout, dout, 3, 3)
    out[prefix + "block2.block.0.bias"] = (dout,)
    out[prefix + "block2.block.1.weight"] = (dout,)
    out[prefix + "block2.block.1.bias"] = (dout,)
    if din != dout:
        out[prefix + "res_conv.weight"] = (dout, din, 1, 1)
        out[prefix + "res_conv.bias"] = (dout,)


def _attn(prefix, c, out):
    hidden = HEADS * DIM_HEAD
    out[prefix + "fn.g"] = (1,)
    out[prefix + "fn.fn.to_qkv.weight"] = (3 * hidden, c, 1, 1)
    out[prefix + "fn.fn.to_out.weight"] = (c, hidden, 1, 1)
    out[prefix + "fn.fn.to_out.bias"] = (c,)


def estimator_param_shapes(dim: int = 64, n_spks: int = 1, spk_emb_dim: int = 64,
                           n_feats: int = 80) -> "OrderedDict[str, tuple]":
    """Ordered ``{key: shape}`` of ``GradLogPEstimator2d.state_dict()`` (registration order)."""
    out: "OrderedDict[str, tuple]" = OrderedDict()
    if uses_spk_mlp(n_spks):
        out["spk_mlp.0.weight"] = (spk_emb_dim * 4, spk_emb_dim)
        out["spk_mlp.0.bias"] = (spk_emb_dim * 4,)
        out["spk_mlp.2.weight"] = (n_feats, spk_emb_dim * 4)
        out["spk_mlp.2.bias"] = (n_feats,)
    out["mlp.0.weight"] = (dim * 4, dim)
    out["mlp.0.bias"] = (dim * 4,)
    out["mlp.2.weight"] = (dim, dim * 4)
    out["mlp.2.bias"] = (dim,)
    dims = level_dims(dim, n_spks)
    in_out = list(zip(dims[:-1], dims[1:]))
    for i, (din, dout) in enumerate(in_out):
        p = f"downs.{i}."
        _resnet(p + "0.", din, dout, dim, out)
        _resnet(p + "1.", dout, dout, dim, out)
        _attn(p + "2.", dout, out)
        if i < len(in_out) - 1:
            out[p + "3.conv.weight"] = (dout, dout, 3, 3)
            out[p + "3.conv.bias"] = (dout,)
    # `downs` and `ups` ModuleLists are registered before the mid blocks (diffusion.py:147-148),
    # so the up path precedes mid_* in state_dict order.
    for i, (din, dout) in enumerate(reversed(in_out[1:])):
        p = f"ups.{i}."
        _resnet(p + "0.", dout * 2, din, dim, out)
        _resnet(p + "1.", din, din, dim, out)
        _attn(p + "2.", din, out)
        out[p + "3.conv.weight"] = (din, din, 4, 4)   # ConvTranspose2d: [in, out, kH, kW]
        out[p + "3.conv.bias"] = (din,)
    mid = dims[-1]
    _resnet("mid_block1.", mid, mid, dim, out)
    _attn("mid_attn.", mid, out)
    _resnet("mid_block2.", mid, mid, dim, out)
    out["final_block.block.0.weight"] = (dim, dim, 3, 3)
    out["final_block.block.0.bias"] = (dim,)
    out["final_block.block.1.weight"] = (dim,)
    out["final_block.block.1.bias"] = (dim,)
    out["final_conv.weight"] = (1, dim, 1, 1)
    out["final_conv.bias"] = (1,)
    return out


def _fan_in(shape):
    return int(shape[1] * int(np.prod(shape[2:]))) if len(shape) > 1 else int(shape[0])


def synthetic_state_dict(seed: int = 0, dim: int = 64, n_spks: int = 1, spk_emb_dim: int = 64,
                         n_feats: int = 80, rezero_g: float = 0.02) -> "OrderedDict[str, np.ndarray]":
    """Deterministic synthetic weights (float32) for the estimator.

    * conv / linear weights and their biases ~ U(-1/sqrt(fan_in), +1/sqrt(fan_in)) (torch's default bound);
    * GroupNorm affine: weight = 1 + 0.1*U(-1,1), bias = 0.1*U(-1,1) (exercises the affine path);
    * Rezero ``g`` = ``rezero_g`` (0.02: attention is active and N<=1000 stays finite).

    Keys are visited in registration order with one PCG64 stream seeded by ``seed``.
    """
    rng = np.random.default_rng(seed)
    shapes = estimator_param_shapes(dim, n_spks, spk_emb_dim, n_feats)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    last_fan = 1
    for key, shape in shapes.items():
        if key.endswith(".g"):
            arr = np.full(shape, rezero_g, dtype=np.float64)
        elif ".block.1." in key:  # GroupNorm affine (Block: Sequential(conv, GN, Mish))
            u = rng.uniform(-1.0, 1.0, size=shape)
            arr = (1.0 + 0.1 * u) if key.endswith("weight") else 0.1 * u
        elif key.endswith("weight"):
            last_fan = _fan_in(shape)
            b = 1.0 / np.sqrt(last_fan)
            arr = rng.uniform(-b, b, size=shape)
        else:  # bias of the preceding weight
            b = 1.0 / np.sqrt(last_fan)
            arr = rng.uniform(-b, b, size=shape)
        out[key] = np.ascontiguousarray(arr.astype(np.float32))
    return out


def state_dict_sha256(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(np.asarray(v, dtype=np.float32)).tobytes())
    return h.hexdigest()


def synthetic_inputs(seed: int, B: int, T: int, n_feats: int = 80, lengths=None, spk_emb_dim: int = 64,
                     temperature: float = 1.0):
    """Synthetic decoder inputs: mu ~ N(0,1), z = mu + N(0,1)/temperature, mask from lengths."""
    rng = np.random.default_rng(seed)
    mu = rng.standard_normal((B, n_feats, T)).astype(np.float32)
    z = (mu + rng.standard_normal((B, n_feats, T)).astype(np.float32) / np.float32(temperature)).astype(np.float32)
    if lengths is None:
        lengths = [T] * B
    mask = np.zeros((B, 1, T), dtype=np.float32)
    for b, L in enumerate(lengths):
        mask[b, 0, :L] = 1.0
    spk = rng.standard_normal((B, spk_emb_dim)).astype(np.float32)
    return mu, z, mask, spk


def fix_len_compatibility(length: int, num_downsamplings_in_unet: int = 2) -> int:
    """Round a frame count up to a multiple of 4 (``model/utils.py:13-17``)."""
    m = 2 ** num_downsamplings_in_unet
    return ((int(length) + m - 1) // m) * m


def estimator_flops(B: int, T: int, n_spks: int = 1) -> int:
    """Algorithmic FLOPs of one estimator call (measured with torch flop_counter)."""
    if n_spks > 1:
        return B * (134_256_640 * T + 368_640)
    return B * (134_154_240 * T + 294_912)


# ---- text encoder (model/text_encoder.py:285-335; GradTTS builds it speaker-agnostic, tts.py:49-51) ----------
def text_encoder_param_shapes(n_vocab: int = 149, n_feats: int = 80, n_channels: int = 192,
                              filter_channels: int = 768, filter_channels_dp: int = 256, n_heads: int = 2,
                              n_layers: int = 6, kernel_size: int = 3, window_size: int = 4):
    """state_dict keys and shapes of the reference TextEncoder, in its registration order (the order
    tests/golden/gradtts_layout.json records from the real module, without the ``encoder.`` prefix)."""
    C, kc = n_channels, n_channels // n_heads
    out = OrderedDict()
    out["emb.weight"] = (n_vocab, C)
    for i in range(3):
        out[f"prenet.conv_layers.{i}.weight"] = (C, C, 5)
        out[f"prenet.conv_layers.{i}.bias"] = (C,)
    for i in range(3):
        out[f"prenet.norm_layers.{i}.gamma"] = (C,)
        out[f"prenet.norm_layers.{i}.beta"] = (C,)
    out["prenet.proj.weight"] = (C, C, 1)
    out["prenet.proj.bias"] = (C,)
    for l in range(n_layers):
        p = f"encoder.attn_layers.{l}."
        out[p + "emb_rel_k"] = (1, 2 * window_size + 1, kc)
        out[p + "emb_rel_v"] = (1, 2 * window_size + 1, kc)
        for n in ("conv_q", "conv_k", "conv_v", "conv_o"):
            out[p + n + ".weight"] = (C, C, 1)
            out[p + n + ".bias"] = (C,)
    for l in range(n_layers):
        out[f"encoder.norm_layers_1.{l}.gamma"] = (C,)
        out[f"encoder.norm_layers_1.{l}.beta"] = (C,)
    for l in range(n_layers):
        p = f"encoder.ffn_layers.{l}."
        out[p + "conv_1.weight"] = (filter_channels, C, kernel_size)
        out[p + "conv_1.bias"] = (filter_channels,)
        out[p + "conv_2.weight"] = (C, filter_channels, kernel_size)
        out[p + "conv_2.bias"] = (C,)
    for l in range(n_layers):
        out[f"encoder.norm_layers_2.{l}.gamma"] = (C,)
        out[f"encoder.norm_layers_2.{l}.beta"] = (C,)
    out["proj_m.weight"] = (n_feats, C, 1)
    out["proj_m.bias"] = (n_feats,)
    Fd = filter_channels_dp
    out["proj_w.conv_1.weight"] = (Fd, C, kernel_size)
    out["proj_w.conv_1.bias"] = (Fd,)
    out["proj_w.norm_1.gamma"] = (Fd,)
    out["proj_w.norm_1.beta"] = (Fd,)
    out["proj_w.conv_2.weight"] = (Fd, Fd, kernel_size)
    out["proj_w.conv_2.bias"] = (Fd,)
    out["proj_w.norm_2.gamma"] = (Fd,)
    out["proj_w.norm_2.beta"] = (Fd,)
    out["proj_w.proj.weight"] = (1, Fd, 1)
    out["proj_w.proj.bias"] = (1,)
    return out


def synthetic_text_encoder_state_dict(seed: int = 0, **kw) -> "OrderedDict[str, np.ndarray]":
    """Deterministic synthetic TextEncoder weights (float32), one PCG64 stream in key order:
    convs U(-1/sqrt(fan_in), +) (torch's default bound; the prenet projection too, which the reference zero-inits,
    so the path is exercised); LayerNorm gamma = 1 + 0.1 U(-1,1), beta = 0.1 U(-1,1); the embedding
    U(-sqrt(3/C), +) (the variance of the reference's N(0, 1/C)); relative embeddings U(-1/sqrt(k_c), +)."""
    rng = np.random.default_rng(seed)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    last_fan = 1
    for key, shape in text_encoder_param_shapes(**kw).items():
        if key.endswith((".gamma", ".beta")):
            u = rng.uniform(-1.0, 1.0, size=shape)
            arr = (1.0 + 0.1 * u) if key.endswith("gamma") else 0.1 * u
        elif key == "emb.weight":
            arr = rng.uniform(-1.0, 1.0, size=shape) * np.sqrt(3.0 / shape[1])
        elif "emb_rel" in key:
            b = 1.0 / np.sqrt(shape[-1])
            arr = rng.uniform(-b, b, size=shape)
        elif key.endswith("weight"):
            last_fan = _fan_in(shape)
            b = 1.0 / np.sqrt(last_fan)
            arr = rng.uniform(-b, b, size=shape)
        else:
            b = 1.0 / np.sqrt(last_fan)
            arr = rng.uniform(-b, b, size=shape)
        out[key] = np.ascontiguousarray(arr.astype(np.float32))
    return out


# ---- HiFi-GAN generator (hifi-gan/models.py:77-128; checkpts/hifigan-config.json, V1) -------------------------
HIFIGAN_V1 = {"resblock": "1", "upsample_rates": [8, 8, 2, 2], "upsample_kernel_sizes": [16, 16, 4, 4],
              "upsample_initial_channel": 512, "resblock_kernel_sizes": [3, 7, 11],
              "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]], "num_mels": 80}
# HiFi-GAN V3 (the published config_v3.json of the HiFi-GAN repository; not shipped in the reference, whose models.py
# builds it with ResBlock2, models.py:53-74 / :84)
HIFIGAN_V3 = {"resblock": "2", "upsample_rates": [8, 8, 4], "upsample_kernel_sizes": [16, 16, 8],
              "upsample_initial_channel": 256, "resblock_kernel_sizes": [3, 5, 7],
              "resblock_dilation_sizes": [[1, 2], [2, 6], [3, 12]], "num_mels": 80}


def _wn(out, key, w_shape, g_dim0):
    out[key + ".bias"] = (w_shape[1] if key.startswith("ups.") else w_shape[0],)
    out[key + ".weight_g"] = (g_dim0, 1, 1)
    out[key + ".weight_v"] = tuple(w_shape)


def vocoder_param_shapes(h=None):
    """Generator state_dict keys and shapes in registration order (weight_norm puts bias, weight_g, weight_v)."""
    h = h or HIFIGAN_V1
    out = OrderedDict()
    c0 = h["upsample_initial_channel"]
    _wn(out, "conv_pre", (c0, h.get("num_mels", 80), 7), c0)
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        cin, cout = c0 // 2 ** i, c0 // 2 ** (i + 1)
        _wn(out, f"ups.{i}", (cin, cout, k), cin)   # ConvTranspose1d weight [in][out][k]; weight_norm dim 0 = in
    n = 0
    for i in range(len(h["upsample_rates"])):
        ch = c0 // 2 ** (i + 1)
        for k, d in zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"]):
            parts = ("convs1", "convs2") if str(h["resblock"]) == "1" else ("convs",)
            for part in parts:
                for m in range(len(d)):
                    _wn(out, f"resblocks.{n}.{part}.{m}", (ch, ch, k), ch)
            n += 1
    _wn(out, "conv_post", (1, c0 // 2 ** len(h["upsample_rates"]), 7), 1)
    return out


def synthetic_vocoder_state_dict(seed: int = 0, h=None) -> "OrderedDict[str, np.ndarray]":
    """Deterministic synthetic Generator weights (float32), one PCG64 stream in key order: weight_v
    U(-1/sqrt(fan_in), +), weight_g = ||v|| over all but dim 0 times 1 + 0.1 U(-1,1) (so the weight-norm scale is
    exercised), bias U(-1/sqrt(fan_in), +)."""
    rng = np.random.default_rng(seed)
    shapes = vocoder_param_shapes(h)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    keys = list(shapes)
    for i in range(0, len(keys), 3):
        kb, kg, kv = keys[i], keys[i + 1], keys[i + 2]
        vs = shapes[kv]
        fan = vs[0] * vs[2] if kb.startswith("ups.") else vs[1] * vs[2]
        bnd = 1.0 / np.sqrt(fan)
        bias = rng.uniform(-bnd, bnd, size=shapes[kb])
        v = rng.uniform(-bnd, bnd, size=vs)
        norm = np.sqrt((v.reshape(vs[0], -1) ** 2).sum(1)).reshape(vs[0], 1, 1)
        g = norm * (1.0 + 0.1 * rng.uniform(-1.0, 1.0, size=norm.shape))
        out[kb], out[kg], out[kv] = (np.ascontiguousarray(a.astype(np.float32)) for a in (bias, g, v))
    return out
