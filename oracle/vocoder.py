"""CPU restatement of the reference's HiFi-GAN generator (hifi-gan/models.py:13-128, V1 configuration of
checkpts/hifigan-config.json) -- TEST INFRASTRUCTURE ONLY: imported by tests/ (never by the product). Pinned to
tests/golden/voc_*.npz (tests/golden/make_golden_vocoder.py ran the reference itself).

* weight      torch.nn.utils.weight_norm's weight = g * v / ||v|| (norm over all dims but 0), as
              remove_weight_norm() bakes it (inference.py:76)
* resblock1   models.py:13-48: 3 x [leaky_relu(0.1) -> dilated conv -> leaky_relu(0.1) -> conv -> + x]
* resblock2   models.py:53-74: per dilation [leaky_relu(0.1) -> dilated conv -> + x] (h["resblock"] == "2", V3)
* generator   models.py:77-110: conv_pre, per stage leaky_relu(0.1) -> ConvTranspose1d -> mean of the resblocks,
              leaky_relu (slope 0.01, the default) -> conv_post -> tanh
"""
import torch
import torch.nn.functional as F

from gradtts_amd.params import HIFIGAN_V1


def weight(p, key):
    v, g = p[key + ".weight_v"], p[key + ".weight_g"]
    norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape(-1, 1, 1)
    return v * (g / norm)


def generator(p, mel, h=None):
    h = h or HIFIGAN_V1
    x = F.conv1d(mel, weight(p, "conv_pre"), p["conv_pre.bias"], padding=3)
    nk = len(h["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = F.leaky_relu(x, 0.1)
        x = F.conv_transpose1d(x, weight(p, f"ups.{i}"), p[f"ups.{i}.bias"], stride=u, padding=(k - u) // 2)
        xs = None
        for j, (kk, dd) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            n = i * nk + j
            y = x
            for m, d in enumerate(dd):
                xt = F.leaky_relu(y, 0.1)
                if str(h["resblock"]) == "2":
                    xt = F.conv1d(xt, weight(p, f"resblocks.{n}.convs.{m}"), p[f"resblocks.{n}.convs.{m}.bias"],
                                  dilation=d, padding=(kk * d - d) // 2)
                    y = xt + y
                    continue
                xt = F.conv1d(xt, weight(p, f"resblocks.{n}.convs1.{m}"), p[f"resblocks.{n}.convs1.{m}.bias"],
                              dilation=d, padding=(kk * d - d) // 2)
                xt = F.leaky_relu(xt, 0.1)
                xt = F.conv1d(xt, weight(p, f"resblocks.{n}.convs2.{m}"), p[f"resblocks.{n}.convs2.{m}.bias"],
                              padding=(kk - 1) // 2)
                y = xt + y
            xs = y if xs is None else xs + y
        x = xs / nk
    x = F.leaky_relu(x)
    x = F.conv1d(x, weight(p, "conv_post"), p["conv_post.bias"], padding=3)
    return torch.tanh(x)


def to_torch_params(sd, dtype=torch.float32):
    return {k: torch.as_tensor(v).to(dtype) for k, v in sd.items()}
