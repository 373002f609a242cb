"""The throughput plan's 1x1 convs on conv1s_kernel (csrc/conv1s.hip): ResnetBlock.res_conv with the block output
(model/diffusion.py:70, 77-78) and the folded attention output with its residual (diffusion.py:108).

conv1s keeps conv_kernel's MFMA sequence per accumulator (32x32x16 bf16, weights as A, 16-channel k-steps in ascending
order) and its epilogue arithmetic, so with 0/1 masks a decoder on conv1s must give the same BITS as one on conv_kernel
(GT_CONV1S=0) -- stage activations, the estimator and the sampler -- on ragged batches whose frame counts leave partial
64-frame tiles at every level. A fractional mask (C-ABI callers only: the Python boundary rejects it) is applied to
the fp32 accumulator instead of the bf16 operand (m W x + b = W (x m) + b per position): agreement within the
plan-agreement gate. The launch lists prove which kernel ran."""
import ctypes
import json

import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder, probe, rel_err, report
from gradtts_amd import _lib
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu

# stages whose output a 1x1 conv forms: res_conv + block output (downs.1.0, downs.2.0, ups.0.0 and ups.1.0 with their
# concatenated inputs) and the attention output + residual (downs.1.2, downs.2.2, mid_attn, ups.0.2; the level-0
# attentions are the fused attn_down / attn_up passes)
STAGES = [("downs.1.0", 128, 40), ("downs.1.2", 128, 40), ("downs.2.0", 256, 20), ("downs.2.2", 256, 20),
          ("mid_attn", 256, 20), ("ups.0.0", 128, 20), ("ups.0.2", 128, 20), ("ups.1.0", 64, 40)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _decoder(monkeypatch, c1s, dtype, small=0):
    monkeypatch.setenv("GT_CONV1S", str(c1s))
    dec, _ = make_decoder(1, 31, dtype)
    _lib.check(_lib.lib().gt_decoder_set_small_batch(dec.estimator._native(), small), "gt_decoder_set_small_batch")
    return dec


def _launches(dec, fn):
    L = _lib.lib()
    h = dec.estimator._native()
    _lib.check(L.gt_decoder_profile_enable(h, 1), "gt_decoder_profile_enable")
    out = fn()
    torch.cuda.synchronize()
    buf = ctypes.create_string_buffer(1 << 20)
    _lib.check(L.gt_decoder_profile_read(h, buf, len(buf)), "gt_decoder_profile_read")
    _lib.check(L.gt_decoder_profile_enable(h, 0), "gt_decoder_profile_enable")
    return out, [r["kernel"] for r in json.loads(buf.value.decode())]


@pytest.mark.parametrize("dtype", [torch.bfloat16, "fp8"], ids=["bf16", "fp8"])
@pytest.mark.parametrize("B,T,lengths,parts", [(3, 132, [132, 97, 40], 0), (2, 256, None, 0), (2, 256, [256, 170], 1),
                                               (3, 132, [132, 97, 40], 3)])
def test_conv1s_bit_identical_to_conv_kernel(monkeypatch, dtype, B, T, lengths, parts):
    """parts: workgroups per (utterance, channel tile) (GT_CONV1S_PARTS; 0 = the launch's own choice, which at these
    batch sizes gives every workgroup one or two stages): 1 and 3 run the stage ring through many wraps, as B = 32 does."""
    if parts:
        monkeypatch.setenv("GT_CONV1S_PARTS", str(parts))
    mu, z, mask, _ = synthetic_inputs(61, B, T, lengths=lengths)
    t = np.linspace(0.85, 0.15, B).astype(np.float32)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(t), None)
    res = {}
    for c1s in (1, 0):
        dec = _decoder(monkeypatch, c1s, dtype)
        est, names = _launches(dec, lambda: dec.estimator(*args))
        # (one entry per kernel and shape: downs.2.2 and mid_attn share theirs)
        n1 = sum(n.startswith("conv1s_kernel<") for n in names)
        assert n1 == (7 if c1s else 0), names   # 4 res_convs + 4 attention outputs
        outs = {"estimator": est.cpu().numpy(), "sampler N=2": dec(args[0], args[1], args[2], 2).cpu().numpy()}
        for st, C, F in STAGES:
            _, pr = probe(dec.estimator, dtype, *args, st, (B, C, F, (T + 3) // 4 if F == 20 else (T + 1) // 2))
            outs[st] = pr.cpu().numpy()
        res[c1s] = outs
    for name in res[1]:
        a, b = res[1][name], res[0][name]
        assert np.isfinite(a).all(), name
        diff = float(np.mean(a != b))
        report(f"conv1s vs conv_kernel {name} ({'bf16' if dtype is torch.bfloat16 else dtype}, B={B}, T={T}, "
               f"parts={parts}): fraction of elements not bit-identical", diff, 0.0)


def test_conv1s_fractional_mask(monkeypatch):
    """C-ABI caller with a fractional mask: m W x + b in fp32 against conv_kernel's W bf16(x m) + b."""
    B, T = 3, 128
    mu, z, mask, _ = synthetic_inputs(63, B, T, lengths=[128, 100, 60])
    frac = (mask * np.random.default_rng(9).uniform(0.25, 1.0, mask.shape)).astype(np.float32)
    t = np.linspace(0.9, 0.3, B).astype(np.float32)
    args = (_cuda(z), _cuda(frac), _cuda(mu), _cuda(t), None)
    outs = {}
    for c1s in (1, 0):
        dec = _decoder(monkeypatch, c1s, torch.bfloat16)
        (score, y), names = _launches(dec, lambda: probe(dec.estimator, torch.bfloat16, *args, "downs.1.0", (B, 128, 40, 64)))
        assert any(n.startswith("conv1s_kernel<") for n in names) == bool(c1s)
        outs[c1s] = (score.cpu().numpy(), y.cpu().numpy())
    for i, name in enumerate(("estimator", "downs.1.0")):
        assert np.isfinite(outs[1][i]).all()
        report(f"conv1s vs conv_kernel {name}, fractional mask (C ABI)", rel_err(outs[1][i], outs[0][i]), 2e-2)


@pytest.mark.parametrize("B,T", [(1, 96), (2, 512)])
def test_conv1s_small_plan(monkeypatch, B, T):
    """The small-batch plan takes conv1s too (one stage per workgroup at B = 1): same bits as its conv_kernel 1-row
    tiles, so the small plan stays batch-invariant."""
    mu, z, mask, _ = synthetic_inputs(64, B, T)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(np.linspace(0.5, 0.3, B).astype(np.float32)), None)
    outs = {}
    for c1s in (1, 0):
        dec = _decoder(monkeypatch, c1s, torch.bfloat16, small=16)
        est, names = _launches(dec, lambda: dec.estimator(*args))
        assert any(n.startswith("conv1s_kernel<") for n in names) == bool(c1s)
        assert any(n.startswith("conv_kernel<bf16,2,") for n in names) == (not c1s)
        outs[c1s] = (est.cpu().numpy(), dec(args[0], args[1], args[2], 2).cpu().numpy())
    for i, name in enumerate(("estimator", "sampler N=2")):
        report(f"conv1s vs conv_kernel {name}, small plan B={B} T={T}: fraction of elements not bit-identical",
               float(np.mean(outs[1][i] != outs[0][i])), 0.0)
