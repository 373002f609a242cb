"""Wide-tile 3x3 convs (csrc/conv3w.hip, include/gradtts.h gt_decoder_set_wide_conv) on the bf16 throughput plan.

conv3w runs the level-1/2 Block convs (model/diffusion.py:52: Cout 64/128/256, Cin % 32 == 0; the GroupNorm-input
block2 convs, the masked-input block1 convs and the skip-concat convs of the up path) as one 8-wave workgroup per CU that
owns every output channel of a 10- or 20-row x 32-frame tile. Checked here, always on the throughput plan
(gt_decoder_set_small_batch(dec, 0)):
  * every U-Net stage against the fp32 oracle (bf16 stage gate 2e-2, as test_decoder_gpu.py) on ragged batches whose
    level-2 rows end in partial 32-frame tiles (T = 132: 33 frames at level 2) and with 247 speakers;
  * the sampler output against the conv_kernel path (GT_CONV3W off) and against the oracle: the two paths differ only
    in fp32 accumulation order and GroupNorm partition (gate: the bf16 sampler gate 1e-2);
  * fractional mask values (outside the decoder's {0, 1} mask contract) rejected at the boundary;
  * determinism and batch invariance at the bench shape are in test_decoder_gpu.py
    (test_bench_shape_deterministic_and_batch_invariant), which now runs conv3w.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import STAGES, make_decoder, probe, rel_err, report
from gradtts_amd import _lib
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu

STAGE_TOL = 2e-2
BF16_REV_TOL = 1e-2


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _plan(dec, wide):
    L = _lib.lib()
    h = dec.estimator._native()
    _lib.check(L.gt_decoder_set_small_batch(h, 0), "gt_decoder_set_small_batch")
    _lib.check(L.gt_decoder_set_wide_conv(h, 1 if wide else 0), "gt_decoder_set_wide_conv")


@pytest.mark.parametrize("n_spks,B,T,lengths", [(1, 3, 132, [132, 100, 44]), (247, 2, 96, [96, 61])])
def test_wide_conv_every_stage_matches_oracle(n_spks, B, T, lengths):
    from oracle import decoder as odec
    dec, sd = make_decoder(n_spks, 3, torch.bfloat16)
    _plan(dec, True)
    mu, z, mask, spk = synthetic_inputs(31, B, T, lengths=lengths)
    t = np.linspace(0.7, 0.2, B).astype(np.float32)
    p = odec.to_torch_params(sd)
    taps = {}
    spk_t = torch.from_numpy(spk) if n_spks > 1 else None
    with torch.no_grad():
        ref = odec.estimator(p, torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu), torch.from_numpy(t),
                             spk_t, n_spks=n_spks, taps=taps).numpy()
    args = [_cuda(a) for a in (z, mask, mu, t)]
    spk_c = _cuda(spk) if n_spks > 1 else None
    bad = []
    for st in STAGES:
        r = taps[st].numpy()
        out, pr = probe(dec.estimator, torch.bfloat16, *args, spk_c, st, r.shape)
        e = rel_err(pr.cpu().numpy(), r)
        if not report(f"conv3w stage {st} n_spks={n_spks} B={B} T={T}", e, STAGE_TOL, gate=False):
            bad.append(f"{st}: {e:.3e}")
    report(f"conv3w estimator n_spks={n_spks} B={B} T={T}", rel_err(out.cpu().numpy(), ref), 1.92e-2)
    assert not bad, "stage mismatches: " + ", ".join(bad)


@pytest.mark.parametrize("B,T,lengths", [(5, 256, [256, 256, 200, 130, 64]), (6, 80, None)])
def test_wide_conv_sampler_agrees_with_conv_kernel_and_oracle(B, T, lengths):
    from oracle import decoder as odec
    dec, sd = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = synthetic_inputs(41, B, T, lengths=lengths)
    zc, mc, muc = _cuda(z), _cuda(mask), _cuda(mu)
    _plan(dec, True)
    yw = dec(zc, mc, muc, 4).cpu().numpy()
    _plan(dec, False)
    yk = dec(zc, mc, muc, 4).cpu().numpy()
    with torch.no_grad():
        ref = odec.reverse_diffusion(odec.to_torch_params(sd), torch.from_numpy(z), torch.from_numpy(mask),
                                     torch.from_numpy(mu), 4).numpy()
    assert np.isfinite(yw).all()
    report(f"conv3w vs conv_kernel sampler N=4 B={B} T={T}", rel_err(yw, yk), BF16_REV_TOL)
    report(f"conv3w sampler N=4 B={B} T={T} vs oracle", rel_err(yw, ref), BF16_REV_TOL)
    report(f"conv_kernel sampler N=4 B={B} T={T} vs oracle", rel_err(yk, ref), BF16_REV_TOL)


def test_fractional_mask_rejected_at_the_boundary():
    """The decoder's contract is {0, 1} masks (sequence_mask, model/utils.py:6-10): the fused kernels compute the
    reference's double masking (Mish(GN(h)) * m + tb) * m (model/diffusion.py:56-58, 74-77) as one multiply, which is
    exact for 0/1 masks and ~0.6 off the reference for fractional ones (measured in round 4 on both conv paths). Such a
    mask is rejected with an error by the estimator, the sampler (torch.ops.gradtts, csrc/torch_ops.cpp) and the training
    loss, instead of being decoded wrongly; a 0/1 mask of the same shape still runs."""
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    B, T = 3, 64
    mu, z, mask, _ = synthetic_inputs(51, B, T, lengths=[64, 50, 30])
    frac = (mask * np.random.default_rng(5).uniform(0.25, 1.0, mask.shape)).astype(np.float32)
    t = np.linspace(0.9, 0.3, B).astype(np.float32)
    zc, muc, tc = _cuda(z), _cuda(mu), _cuda(t)
    with pytest.raises(RuntimeError, match="0 or 1"):
        dec.estimator(zc, _cuda(frac), muc, tc)
    with pytest.raises(RuntimeError, match="0 or 1"):
        dec(zc, _cuda(frac), muc, 2)
    with pytest.raises(RuntimeError, match="0 or 1"):
        dec.loss_t(zc, _cuda(frac), muc, tc)
    y = dec(zc, _cuda(mask), muc, 2)
    assert torch.isfinite(y).all()


def test_wide_conv_deterministic_large_batch():
    """B = 40 (more tiles than CUs at level 2: two rounds of the 256-workgroup grid): two runs bit-identical, and
    utterances 30..39 bit-identical to the same utterances decoded alone as a batch of 10."""
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    _plan(dec, True)
    mu, z, mask, _ = synthetic_inputs(61, 40, 256)
    zc, mc, muc = _cuda(z), _cuda(mask), _cuda(mu)
    y1 = dec(zc, mc, muc, 2)
    y2 = dec(zc, mc, muc, 2)
    sub = dec(zc[30:].contiguous(), mc[30:].contiguous(), muc[30:].contiguous(), 2)
    assert torch.isfinite(y1).all()
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    assert torch.equal(y1[30:], sub), float((y1[30:] - sub).abs().max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, "fp8"], ids=["bf16", "fp8"])
def test_fractional_mask_c_abi_paths_agree(dtype):
    """A caller of the C ABI itself (no boundary check there) may still pass a fractional mask: conv3w's items then
    read their mask values again (pm_of, the path 0/1 masks never take) and compute x * m as conv_kernel does. The
    estimator through gt_estimator_probe with conv3w on and off agrees within the bf16 gate (both paths compute
    (Mish(GN(h)) + tb) * m, the single-multiply form the boundary's 0/1 contract makes exact). fp8: conv3w_a8 against
    conv_kernel's A8 tiles, the mask values read back from LDS (s_pm) before the quantization; the two fp8 paths differ
    by e4m3 rounding flips (their GroupNorm statistics sum in different orders), so the gate is test_fp8_gpu.py's
    plan-agreement gate (5e-2), and the same comparison with the 0/1 mask is reported beside it."""
    B, T = 3, 128
    mu, z, mask, _ = synthetic_inputs(52, B, T, lengths=[128, 100, 60])
    frac = (mask * np.random.default_rng(6).uniform(0.25, 1.0, mask.shape)).astype(np.float32)
    t = np.linspace(0.9, 0.3, B).astype(np.float32)
    name = "bf16" if dtype is torch.bfloat16 else dtype
    for label, m in (("fractional", frac), ("0/1", mask)) if name == "fp8" else (("fractional", frac),):
        a = [_cuda(v) for v in (z, m, mu, t)]
        outs = []
        for wide in (True, False):
            dec, _ = make_decoder(1, 0, dtype)
            _plan(dec, wide)
            y, _ = probe(dec.estimator, dtype, *a, None, "downs.1.1", (B, 128, 40, T // 2))
            outs.append(y.cpu().numpy())
        assert np.isfinite(outs[0]).all()
        report(f"conv3w vs conv_kernel estimator, {label} mask (C ABI, {name})", rel_err(outs[0], outs[1]),
               STAGE_TOL if name == "bf16" else 5e-2)
