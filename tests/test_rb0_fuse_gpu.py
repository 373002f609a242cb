"""The first ResnetBlock's output formed inside the next block's conv (csrc/conv64.hip IN_RB0, decoder.cpp conv3_stats).

downs.0.0's output r0 = Mish(GN(h2)) * m + res_conv(x * m) over the 2-3 U-Net input channels (model/diffusion.py:70-79,
181-184) used to be written by its own elementwise pass (rbout_input_kernel) and read back by downs.0.1's block1 conv.
Now that conv (conv64 IN_RB0) forms r0 per staged item from h2 with the pass's fp32 operations and writes it once per
position for the residual of downs.0.1. So a decoder built with GT_RB0_FUSE=1 (the default) must give bit-identical
estimator outputs, samples and stage probes ("downs.0.0" = r0 as written by the conv, "downs.0.1.pre1" = the conv's
own output, "downs.0.1") to one built with GT_RB0_FUSE=0, on ragged batches (masked frames carry r0 = res_conv bias:
written, but staged as zeros), T not a multiple of 32 (partial column segments), 247 speakers (3 input channels) and
on both tile plans (the small plan walks one-tile segments: the halo rows of a segment are not its own to write), and
with fp8 weights (bf16_w8, fp8: the 64 -> 64 level-0 convs keep bf16 operands on conv64, accumulating from bias / scale)."""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder, probe
from gradtts_amd import _lib
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n_spks,B,T,lengths,small,dtype", [(1, 3, 132, [132, 100, 44], False, torch.bfloat16),
                                                           (247, 2, 96, [96, 61], False, torch.bfloat16),
                                                           (1, 2, 76, [76, 50], True, torch.bfloat16),
                                                           (247, 1, 132, None, True, torch.bfloat16),
                                                           (1, 3, 132, [132, 100, 44], False, "bf16_w8"),
                                                           (247, 2, 96, [96, 61], True, "fp8")])
def test_rb0_fused_bit_identical(monkeypatch, n_spks, B, T, lengths, small, dtype):
    mu, z, mask, spk = synthetic_inputs(37, B, T, lengths=lengths)
    t = np.linspace(0.9, 0.2, B).astype(np.float32)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(t), _cuda(spk) if n_spks > 1 else None)
    res = {}
    for fuse in (1, 0):
        monkeypatch.setenv("GT_RB0_FUSE", str(fuse))
        dec, _ = make_decoder(n_spks, 17, dtype)
        _lib.check(_lib.lib().gt_decoder_set_small_batch(dec.estimator._native(), 16 if small else 0),
                   "gt_decoder_set_small_batch")
        z_, m_, mu_, t_, s_ = args
        est = dec.estimator(z_, m_, mu_, t_, s_)
        y = dec(z_, m_, mu_, 3, spk=s_)
        outs = [est.cpu(), y.cpu()]
        for st in ("downs.0.0", "downs.0.1.pre1", "downs.0.1"):
            _, pr = probe(dec.estimator, dtype, z_, m_, mu_, t_, s_, st, (B, 64, 80, T))
            outs.append(pr.cpu())
        torch.cuda.synchronize()
        res[fuse] = outs
    for a, b_, name in zip(res[1], res[0], ("estimator", "sampler N=3", "downs.0.0", "downs.0.1.pre1", "downs.0.1")):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b_), f"{name}: max |diff| {float((a - b_).abs().max())}"


@pytest.mark.parametrize("small,dtype", [(False, torch.bfloat16), (True, torch.bfloat16), (False, "fp8")],
                         ids=["bf16", "bf16-small", "fp8"])
def test_rb0_fused_fractional_mask_c_abi(monkeypatch, small, dtype):
    """A C-ABI caller (no boundary mask check) with a fractional mask: the fused IN_RB0 operand is bf16(r0) * m rounded
    to bf16 -- the unfused IN_MASK conv's operand -- so both builds still give the same bits (gradtts.h: a consistent
    result on every kernel path)."""
    B, T = 3, 132
    mu, z, mask, _ = synthetic_inputs(38, B, T, lengths=[132, 100, 44])
    frac = (mask * np.random.default_rng(9).uniform(0.25, 1.0, mask.shape)).astype(np.float32)
    t = np.linspace(0.9, 0.2, B).astype(np.float32)
    args = (_cuda(z), _cuda(frac), _cuda(mu), _cuda(t), None)
    res = {}
    for fuse in (1, 0):
        monkeypatch.setenv("GT_RB0_FUSE", str(fuse))
        dec, _ = make_decoder(1, 17, dtype)
        _lib.check(_lib.lib().gt_decoder_set_small_batch(dec.estimator._native(), 16 if small else 0),
                   "gt_decoder_set_small_batch")
        outs = []
        for st in ("downs.0.1.pre1", "downs.0.1"):
            y, pr = probe(dec.estimator, dtype, *args, st, (B, 64, 80, T))
            outs += [pr.cpu(), y.cpu()]
        res[fuse] = outs
    for a, b_, name in zip(res[1], res[0], ("downs.0.1.pre1", "estimator", "downs.0.1", "estimator (2)")):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b_), f"{name}: max |diff| {float((a - b_).abs().max())}"
