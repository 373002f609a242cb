"""Small-batch tile plan (decoder.cpp small_plan, include/gradtts.h gt_decoder_set_small_batch).

bf16 calls on at most 4 utterances run 1-row (128-wide) / 2-row (64-wide) conv tiles and one-tile conv64
segments, so that a single utterance fills the GPU. Checked here:
  * the plan is batch-invariant on its own: an utterance decoded alone, in a pair, or in a batch of 4 gives
    bit-identical mels (GroupNorm partial slots and attention tiles depend only on the utterance's shape);
  * the two plans agree within the bf16 sampler gate (1e-2) -- they differ only in how the
    GroupNorm partial sums are partitioned (fp32 rounding), printed as PARITY lines;
  * the throughput plan (forced on small batches with gt_decoder_set_small_batch(dec, 0)) still meets the
    reference-pinned bf16 gates on the golden fixtures (the default run of test_decoder_gpu.py now takes the
    small plan at those batch sizes);
  * small-plan latency at B = 1, T = 512 is printed next to the throughput plan's (no timing gate);
  * split-K of the small plan's 128-wide 3x3 convs is deterministic and agrees with the unsplit tiles.
"""
import time

import numpy as np
import pytest
import torch

from conftest import gpu_available, load_golden
from gpu_util import make_decoder, rel_err, report
from gradtts_amd import _lib
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu

BF16_REV_TOL = 1e-2


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _inputs(seed, B, T, lengths=None):
    mu, z, mask, spk = synthetic_inputs(seed, B, T, lengths=lengths)
    return [torch.from_numpy(a).cuda() for a in (mu, z, mask, spk)]


def _set_small(dec, max_b):
    L = _lib.lib()
    _lib.check(L.gt_decoder_set_small_batch(dec.estimator._native(), max_b), "gt_decoder_set_small_batch")


def test_small_plan_batch_invariant():
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = _inputs(21, 4, 256, lengths=[256, 200, 120, 64])
    y4 = dec(z, mask, mu, 3)
    y1 = dec(z[1:2].contiguous(), mask[1:2].contiguous(), mu[1:2].contiguous(), 3)
    y2 = dec(z[2:4].contiguous(), mask[2:4].contiguous(), mu[2:4].contiguous(), 3)
    assert torch.isfinite(y4).all()
    assert torch.equal(y4[1:2], y1), float((y4[1:2] - y1).abs().max())
    assert torch.equal(y4[2:4], y2), float((y4[2:4] - y2).abs().max())


@pytest.mark.parametrize("T", [80, 96, 1040])
def test_small_plan_batch_invariant_ragged_tiles(T):
    """T % 64 in 1..32: the small plan's 2-row 64-wide level-0 tiles write 40*ceil(T/64) GroupNorm partials per
    utterance, more than conv64's 20*ceil(T/32); every utterance of a batch of 4 must still equal its B = 1 decode
    (the stats slots are sized for the largest producer of either plan)."""
    for dt in (torch.bfloat16, "bf16_w8"):
        dec, _ = make_decoder(1, 0, dt)
        lengths = [T, T - 4, T - 12, max(4, T - 40)]
        mu, z, mask, _ = _inputs(31, 4, T, lengths=lengths)
        y4 = dec(z, mask, mu, 2)
        assert torch.isfinite(y4).all()
        for b in range(4):
            sl = slice(b, b + 1)
            y1 = dec(z[sl].contiguous(), mask[sl].contiguous(), mu[sl].contiguous(), 2)
            assert torch.equal(y4[sl], y1), (dt, T, b, float((y4[sl] - y1).abs().max()))


@pytest.mark.parametrize("B,T,N", [(1, 512, 10), (3, 256, 10), (4, 128, 10)])
def test_plans_agree(B, T, N):
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    lengths = [T - 16 * i for i in range(B)]
    mu, z, mask, _ = _inputs(5 + B, B, T, lengths=lengths)
    y_small = dec(z, mask, mu, N).cpu().numpy()
    _set_small(dec, 0)
    y_tput = dec(z, mask, mu, N).cpu().numpy()
    assert np.isfinite(y_small).all() and np.isfinite(y_tput).all()
    report(f"small vs throughput plan bf16 B={B} T={T} N={N}", rel_err(y_small, y_tput), BF16_REV_TOL)


@pytest.mark.parametrize("name", ["reverse_s1_N10.npz", "reverse_s247_N10.npz", "reverse_s1_N50.npz"])
def test_throughput_plan_bf16_matches_reference(name):
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), torch.bfloat16)
    _set_small(dec, 0)
    spk = torch.from_numpy(g["spk"]).cuda() if n_spks != 1 else None
    c = lambda k: torch.from_numpy(np.ascontiguousarray(g[k])).cuda()
    y = dec(c("z"), c("mask"), c("mu"), int(g["n_timesteps"]), False, spk).cpu().numpy()
    report(f"reverse bf16 throughput plan {name}", rel_err(y, g["out"]), BF16_REV_TOL)


def test_throughput_plan_every_stage_bf16():
    """Every U-Net stage vs the oracle on the throughput plan (forced at the fixture's batch size): the tiles the
    bench runs (5-row tiles, 32-channel 1x1 chunks, the ResnetBlock output formed in attn_kv, conv64 column
    segments), which the default small-batch plan does not run at the fixtures' sizes. bf16 stage gate 2e-2, as
    test_decoder_gpu's."""
    from conftest import load_golden
    from gpu_util import STAGES, probe
    from oracle import decoder as odec
    g = load_golden("estimator_s1_T132.npz")
    dec, sd = make_decoder(1, 0, torch.bfloat16)
    _set_small(dec, 0)
    p = odec.to_torch_params(sd)
    taps = {}
    with torch.no_grad():
        odec.estimator(p, torch.from_numpy(g["x"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["mu"]),
                       torch.from_numpy(g["t"]), None, taps=taps)
    args = [torch.from_numpy(np.ascontiguousarray(g[k])).cuda() for k in ("x", "mask", "mu", "t")]
    bad = []
    for st in STAGES:
        ref = taps[st].numpy()
        _, pr = probe(dec.estimator, torch.bfloat16, *args, None, st, ref.shape)
        e = rel_err(pr.cpu().numpy(), ref)
        if not report(f"stage {st} bf16 throughput plan", e, 2e-2, gate=False):
            bad.append(f"{st}: {e:.3e}")
    assert not bad, "stage mismatches: " + ", ".join(bad)


def test_throughput_plan_speaker_input_conv_bf16():
    """n_spks = 247 (the input conv takes 3 channels: mu, x_t, spk) on ragged lengths: throughput plan vs small plan."""
    dec, _ = make_decoder(247, 0, torch.bfloat16)
    B, T = 3, 128
    mu, z, mask, spk = _inputs(31, B, T, lengths=[128, 100, 60])   # spk: speaker embeddings [B, 64]
    y_small = dec(z, mask, mu, 4, False, spk).cpu().numpy()
    _set_small(dec, 0)
    y_tput = dec(z, mask, mu, 4, False, spk).cpu().numpy()
    assert np.isfinite(y_tput).all()
    report(f"small vs throughput plan bf16 n_spks=247 B={B} T={T} N=4", rel_err(y_small, y_tput), BF16_REV_TOL)


def test_w8_small_plan_batch_invariant_and_agrees():
    """fp8-weight calls (config 5) on at most 4 utterances take the small-batch tiles too: batch-invariant within
    the plan, and within the bf16 sampler gate of the throughput plan."""
    dec, _ = make_decoder(1, 0, "bf16_w8")
    mu, z, mask, _ = _inputs(23, 4, 256, lengths=[256, 200, 120, 64])
    y4 = dec(z, mask, mu, 3)
    y1 = dec(z[1:2].contiguous(), mask[1:2].contiguous(), mu[1:2].contiguous(), 3)
    assert torch.isfinite(y4).all()
    assert torch.equal(y4[1:2], y1), float((y4[1:2] - y1).abs().max())
    _set_small(dec, 0)
    y4t = dec(z, mask, mu, 3)
    report("w8 small vs throughput plan B=4 T=256 N=3", rel_err(y4.cpu().numpy(), y4t.cpu().numpy()), BF16_REV_TOL)


@pytest.mark.parametrize("mode", ["bf16_w8", "fp8", torch.bfloat16])
def test_latency_b1_report(mode):
    """Config 5 latency (fp8 weights / fp8 operands; bf16 for comparison), B = 1, T = 512: small plan vs throughput
    plan, ms per Euler step."""
    dec, _ = make_decoder(1, 0, mode)
    mu, z, mask, _ = _inputs(3, 1, 512)
    N = 20

    def run():
        dec(z, mask, mu, N)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = dec(z, mask, mu, N)
        torch.cuda.synchronize()
        return y, (time.perf_counter() - t0) / N * 1e3

    y_s, ms_s = run()
    _set_small(dec, 0)
    y_t, ms_t = run()
    print(f"LATENCY {mode} B=1 T=512: small plan {ms_s:.3f} ms per step, throughput plan {ms_t:.3f} ms per step "
          f"({512 / (1000 * ms_s) * 1e3:.0f} vs {512 / (1000 * ms_t) * 1e3:.0f} mel-frames/s for 1000-step decodes)")
    assert torch.isfinite(y_s).all() and torch.isfinite(y_t).all()


@pytest.mark.parametrize("mode", [torch.bfloat16, "bf16_w8", "fp8"])
def test_split_k_deterministic_and_agrees(monkeypatch, mode):
    """Split-K of the small plan's 128-wide 3x3 convs (conv.hip ConvCfg::SK: the last of a tile's workgroups adds the
    fp32 partials in split order and re-arms the tile's counter), for bf16, fp8-weight and fp8-operand tiles: repeated
    decodes are bit-identical whichever workgroup finishes last, a second decoder on the same workspace sizes sees
    zeroed counters, and the result agrees with the unsplit tiles (GT_SK_TARGET=0) within the bf16 sampler gate
    (fp8 operands: the per-block scales are per position and chunk, so splitting K changes no quantization).
    B = 1, T = 512: level-2 tiles split 3-4 ways."""
    mu, z, mask, _ = _inputs(41, 1, 512, lengths=[480])
    dec, _ = make_decoder(1, 0, mode)
    ya = dec(z, mask, mu, 4)
    yb = dec(z, mask, mu, 4)
    assert torch.isfinite(ya).all()
    assert torch.equal(ya, yb), float((ya - yb).abs().max())
    monkeypatch.setenv("GT_SK_TARGET", "0")
    dec0, _ = make_decoder(1, 0, mode)
    y0 = dec0(z, mask, mu, 4)
    report(f"small plan split-K vs unsplit {mode} B=1 T=512 N=4", rel_err(ya.cpu().numpy(), y0.cpu().numpy()),
           BF16_REV_TOL)
