"""attn_down_kernel (csrc/attn_down.hip): the level-0 attention output and the Downsample after it in one pass.

The kernel performs the same operations in the same order as conv_kernel CONV1/OUT_RESID followed by conv_kernel
CONV3_S2/IN_MASK, so a decoder built with GT_ATTN_DS=1 (the default) must produce bit-identical estimator outputs,
samples and downsample outputs to one built with GT_ATTN_DS=0, on ragged batches (frames past an utterance's length
masked; T not a multiple of 64: a partial last 32-frame output tile) and with 247 speakers. The fused path's
downsample output is also checked against the fp32 oracle (the "downs.0.3" stage probe takes the fused path; probing
"downs.0.2", the attention output the fused path never writes, falls back to the two launches)."""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder, probe, rel_err, report
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n_spks,B,T,lengths,dtype", [(1, 3, 132, [132, 100, 44], torch.bfloat16),
                                                     (247, 2, 512, [512, 301], torch.bfloat16),
                                                     (1, 4, 64, None, torch.bfloat16),
                                                     (1, 3, 132, [132, 100, 44], "bf16_w8"), (247, 2, 96, [96, 71], "fp8")])
def test_attn_down_bit_identical(monkeypatch, n_spks, B, T, lengths, dtype):
    """(bf16_w8 / fp8: the Downsample's fp8 weights -- their e4m3 values in the fragment image, the per-channel scale in
    the epilogue as conv_kernel W8 applies it)"""
    mu, z, mask, spk = synthetic_inputs(23, B, T, lengths=lengths)
    t = np.linspace(0.9, 0.2, B).astype(np.float32)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(t), _cuda(spk) if n_spks > 1 else None)
    res = {}
    for ds in (1, 0):
        monkeypatch.setenv("GT_ATTN_DS", str(ds))
        dec, _ = make_decoder(n_spks, 11, dtype)
        z_, m_, mu_, t_, s_ = args
        est = dec.estimator(z_, m_, mu_, t_, s_)
        y = dec(z_, m_, mu_, 3, spk=s_)
        _, lvl1 = probe(dec.estimator, dtype, z_, m_, mu_, t_, s_, "downs.0.3", (B, 64, 40, T // 2))
        _, att1 = probe(dec.estimator, dtype, z_, m_, mu_, t_, s_, "downs.1.2", (B, 128, 40, T // 2))
        _, lvl2 = probe(dec.estimator, dtype, z_, m_, mu_, t_, s_, "downs.1.3", (B, 128, 20, T // 4))
        torch.cuda.synchronize()
        res[ds] = (est.cpu(), y.cpu(), lvl1.cpu(), att1.cpu(), lvl2.cpu())
    for a, b_, name in zip(res[1], res[0], ("estimator", "sampler N=3", "downs.0.3", "downs.1.2", "downs.1.3")):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b_), f"{name}: max |diff| {float((a - b_).abs().max())}"


def test_attn_down_stage_vs_oracle():
    from oracle import decoder as odec
    dec, sd = make_decoder(1, 3, torch.bfloat16)
    B, T = 3, 132
    mu, z, mask, _ = synthetic_inputs(31, B, T, lengths=[132, 100, 44])
    t = np.linspace(0.7, 0.2, B).astype(np.float32)
    taps = {}
    with torch.no_grad():
        odec.estimator(odec.to_torch_params(sd), torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu),
                       torch.from_numpy(t), None, n_spks=1, taps=taps)
    args = [_cuda(a) for a in (z, mask, mu, t)]
    for st in ("downs.0.2", "downs.0.3", "downs.1.2", "downs.1.3"):
        r = taps[st].numpy()
        _, pr = probe(dec.estimator, torch.bfloat16, *args, None, st, r.shape)
        report(f"attn_down stage {st}", rel_err(pr.cpu().numpy(), r), 2e-2)


@pytest.mark.parametrize("n_spks,B,T,lengths,dtype", [(1, 3, 132, [132, 100, 44], torch.bfloat16),
                                                     (247, 2, 512, [512, 301], torch.bfloat16), (1, 2, 72, None, torch.bfloat16),
                                                     (1, 3, 132, [132, 100, 44], "bf16_w8"), (247, 2, 72, None, "fp8")])
def test_attn_up_bit_identical(monkeypatch, n_spks, B, T, lengths, dtype):
    """attn_up_kernel (ups.1's attention output + Upsample, one pass) against the two launches (GT_ATTN_US=0): the
    estimator, a 3-step sample and the level-0 upsample output ("ups.1.3") bit-identical; T = 132 / 72: partial
    32-frame coarse tiles."""
    mu, z, mask, spk = synthetic_inputs(29, B, T, lengths=lengths)
    t = np.linspace(0.85, 0.25, B).astype(np.float32)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(t), _cuda(spk) if n_spks > 1 else None)
    res = {}
    for us in (1, 0):
        monkeypatch.setenv("GT_ATTN_US", str(us))
        dec, _ = make_decoder(n_spks, 13, dtype)
        z_, m_, mu_, t_, s_ = args
        est = dec.estimator(z_, m_, mu_, t_, s_)
        y = dec(z_, m_, mu_, 3, spk=s_)
        _, up = probe(dec.estimator, dtype, z_, m_, mu_, t_, s_, "ups.1.3", (B, 64, 80, T))
        torch.cuda.synchronize()
        res[us] = (est.cpu(), y.cpu(), up.cpu())
    for a, b_, name in zip(res[1], res[0], ("estimator", "sampler N=3", "ups.1.3")):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b_), f"{name}: max |diff| {float((a - b_).abs().max())}"
