"""CPU experiment (oracle only): what would fp8 (OCP e4m3) ACTIVATIONS cost in accuracy on top of the fp8 weights of
BASELINE config 5? v_mfma_*_f8f6f4 needs both operands in fp8, so a real fp8-MFMA conv would quantize every conv input
(the 3x3 / Downsample / Upsample operands) to e4m3 with a scale per utterance and 16-channel K chunk (the granularity a
producer epilogue or the consumer's operand load can compute). The sampler output is compared with the fp32
reference (the oracle is pinned to the real reference) for:

  w8        fp8 weights, fp32 activations         (the dequantized-weight oracle the W8 tests gate against)
  w8_bf16   fp8 weights, bf16-rounded conv inputs (what the shipped W8 kernels compute)
  w8_a8c16  fp8 weights, e4m3 conv inputs, scale per (utterance, 16-channel chunk)
  w8_a8c    fp8 weights, e4m3 conv inputs, scale per (utterance, channel)

usage: python tools/fp8_act_envelope.py [N=50] [T=64]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "grad-tts_amd")]
from gradtts_amd.params import synthetic_inputs, synthetic_state_dict  # noqa: E402
from oracle import decoder as odec  # noqa: E402

E4M3_MAX = 448.0


def q_e4m3(x, group):
    """x [B, C, H, W] -> e4m3-rounded with a scale per (b, channel group of `group`) (amax / 448)."""
    B, C = x.shape[:2]
    g = x.reshape(B, C // group, group, *x.shape[2:])
    amax = g.abs().amax(dim=tuple(range(2, g.dim())), keepdim=True)
    s = torch.where(amax > 0, amax / E4M3_MAX, torch.ones_like(amax))
    q = (g / s).to(torch.float8_e4m3fn).to(torch.float32) * s
    return q.reshape(x.shape)


def run(mode, p, z, mask, mu, N):
    conv2d, convt = F.conv2d, F.conv_transpose2d

    def quant(x):
        if mode == "w8_bf16":
            return x.to(torch.bfloat16).to(torch.float32)
        if mode == "w8_a8c16":
            return q_e4m3(x, 16) if x.shape[1] % 16 == 0 else x.to(torch.bfloat16).to(torch.float32)
        if mode == "w8_a8c":
            return q_e4m3(x, 1)
        return x

    def qconv2d(x, w, b=None, stride=1, padding=0, *a, **k):
        if w.shape[-1] == 3:   # the fp8-weight convs: Block 3x3, Downsample
            x = quant(x)
        return conv2d(x, w, b, stride, padding, *a, **k)

    def qconvt(x, w, b=None, stride=1, padding=0, *a, **k):
        return convt(quant(x), w, b, stride, padding, *a, **k)

    F.conv2d, F.conv_transpose2d = qconv2d, qconvt
    try:
        with torch.no_grad():
            return odec.reverse_diffusion(p, z, mask, mu, N).numpy()
    finally:
        F.conv2d, F.conv_transpose2d = conv2d, convt


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    sd = synthetic_state_dict(seed=0)
    p32 = odec.to_torch_params(sd)
    p8 = odec.fp8_params(sd)
    mu, z, mask, _ = synthetic_inputs(7, 2, T, lengths=[T, T - T // 4])
    mu, z, mask = (torch.from_numpy(a) for a in (mu, z, mask))
    with torch.no_grad():
        ref = odec.reverse_diffusion(p32, z, mask, mu, N).numpy()
    scale = np.abs(ref).max()
    print(f"N={N} T={T}: |ref| max {scale:.1f}")
    for mode in ("w8", "w8_bf16", "w8_a8c16", "w8_a8c"):
        y = run(mode, p8, z, mask, mu, N)
        e = np.abs(y - ref)
        print(f"{mode:9s} rel-to-max err vs fp32: max {e.max() / scale:.3e}  mean {e.mean() / scale:.3e}", flush=True)


if __name__ == "__main__":
    main()
