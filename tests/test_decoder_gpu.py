"""GPU parity of the HIP decoder (through the C ABI via the drop-in modules) against
(a) golden vectors produced by the real reference (tests/golden, make_golden.py) and
(b) the oracle (oracle/decoder.py, itself pinned to those vectors) on larger / other shapes.

Tolerances (written here; rel = max|d| / max|ref|):
  * fp32 compute: 1e-4 (the reference's own fp32-vs-fp64 spread reaches 3.4e-5 at N = 50);
  * bf16 sampler: 1e-2; the reference's own bf16 autocast is 2.2-3.9e-3 from its fp32 output on
    these fixtures (tests/golden/ref_bf16_envelope.json, made by make_bf16_envelope.py from the reference);
  * bf16, one estimator call: 1.25 x the reference's own bf16-autocast error on the same fixture (1.07-1.92e-2:
    a single call is dominated by the bf16 rounding of its inputs and activations, which the reference's bf16
    path has too); on oracle-only shapes the envelope's largest value over the five fixtures (1.92e-2) for the
    max element, and 1e-2 for the 99.9th percentile (a single call's max is one sensitive element: an fp32 res_conv
    for the first ResnetBlock, which lowered every U-Net stage's error, moved it from 1.23e-2 to 1.56e-2 on the
    B = 3, T = 256 case -- tools/diag_stage_err.py; measured, not kept for speed reasons).
Every check prints its achieved error (PARITY lines in the log).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, gpu_available, load_golden
from gpu_util import STAGES, make_decoder, probe, rel_err, report

pytestmark = pytest.mark.gpu

FP32_TOL = 1e-4
BF16_EST_TOL = 1.92e-2       # oracle-only shapes: the reference's largest bf16 envelope over the estimator fixtures
BF16_EST_P999_TOL = 1e-2     # ... and the 99.9th percentile of |d| / max|ref|
BF16_REV_TOL = 1e-2
with open(os.path.join(GOLDEN, "ref_bf16_envelope.json")) as _f:
    REF_BF16 = json.load(_f)


def bf16_est_gate(name):
    return 1.25 * REF_BF16[name]["ref_bf16_vs_f32"]

EST = ["estimator_s1.npz", "estimator_s247.npz", "estimator_sm1.npz", "estimator_s1_T132.npz", "estimator_s1_T20.npz"]
REV = ["reverse_s1_N1.npz", "reverse_s1_N2.npz", "reverse_s1_N10.npz", "reverse_s1_N50.npz", "reverse_s247_N10.npz",
       "reverse_s1_N10_alone_T100.npz"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("name", EST)
@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_estimator_matches_reference(name, cdt):
    tol = FP32_TOL if cdt == torch.float32 else bf16_est_gate(name)
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), cdt)
    spk = _cuda(g["spk"]) if n_spks != 1 else None
    y = dec.estimator(_cuda(g["x"]), _cuda(g["mask"]), _cuda(g["mu"]), _cuda(g["t"]), spk).cpu().numpy()
    assert np.isfinite(y).all()
    report(f"estimator {name} {cdt}", rel_err(y, g["out"]), tol)


@pytest.mark.parametrize("name", REV)
def test_reverse_diffusion_fp32_matches_reference(name):
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), torch.float32)
    spk = _cuda(g["spk"]) if n_spks != 1 else None
    y = dec(_cuda(g["z"]), _cuda(g["mask"]), _cuda(g["mu"]), int(g["n_timesteps"]), False, spk).cpu().numpy()
    report(f"reverse fp32 {name}", rel_err(y, g["out"]), FP32_TOL)


@pytest.mark.parametrize("name", ["reverse_s1_N10.npz", "reverse_s247_N10.npz", "reverse_s1_N50.npz"])
def test_reverse_diffusion_bf16_matches_reference(name):
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), torch.bfloat16)
    spk = _cuda(g["spk"]) if n_spks != 1 else None
    y = dec(_cuda(g["z"]), _cuda(g["mask"]), _cuda(g["mu"]), int(g["n_timesteps"]), False, spk).cpu().numpy()
    report(f"reverse bf16 {name}", rel_err(y, g["out"]), BF16_REV_TOL)


def test_padding_dependence_reproduced():
    """Same utterance alone (T=100) vs padded in a batch (T=128) differ in the reference (GN and
    attention statistics include padded frames); the HIP path must reproduce BOTH results."""
    gb = load_golden("reverse_s1_N10.npz")
    ga = load_golden("reverse_s1_N10_alone_T100.npz")
    dec, _ = make_decoder(1, 0, torch.float32)
    yb = dec(_cuda(gb["z"]), _cuda(gb["mask"]), _cuda(gb["mu"]), 10).cpu().numpy()
    ya = dec(_cuda(ga["z"]), _cuda(ga["mask"]), _cuda(ga["mu"]), 10).cpu().numpy()
    assert rel_err(yb, gb["out"]) <= FP32_TOL and rel_err(ya, ga["out"]) <= FP32_TOL
    assert np.max(np.abs(yb[1, :, :100] - ya[0])) > 1e-2


@pytest.mark.parametrize("cdt,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_every_stage_matches_oracle(cdt, tol):
    """Intermediate activations of every U-Net stage vs the oracle (localises any mismatch)."""
    from oracle import decoder as odec
    g = load_golden("estimator_s1_T132.npz")
    dec, sd = make_decoder(1, 0, cdt)
    p = odec.to_torch_params(sd)
    taps = {}
    with torch.no_grad():
        odec.estimator(p, torch.from_numpy(g["x"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["mu"]),
                       torch.from_numpy(g["t"]), None, taps=taps)
    args = [_cuda(g[k]) for k in ("x", "mask", "mu", "t")]
    bad = []
    for st in STAGES:
        ref = taps[st].numpy()
        _, pr = probe(dec.estimator, cdt, *args, None, st, ref.shape)
        e = rel_err(pr.cpu().numpy(), ref)
        if not report(f"stage {st} {cdt}", e, tol, gate=False):
            bad.append(f"{st}: {e:.3e}")
    assert not bad, "stage mismatches: " + ", ".join(bad)


@pytest.mark.parametrize("B,T,lengths", [(3, 256, [256, 200, 64]), (2, 516, [516, 300])])
def test_estimator_vs_oracle_other_shapes(B, T, lengths):
    from oracle import decoder as odec
    from gradtts_amd.params import synthetic_inputs
    dec, sd = make_decoder(1, 1, torch.float32)
    mu, z, mask, _ = synthetic_inputs(7, B, T, lengths=lengths)
    t = np.linspace(0.9, 0.1, B).astype(np.float32)
    ref = odec.estimator(odec.to_torch_params(sd), torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu),
                         torch.from_numpy(t)).numpy()
    y32 = dec.estimator(_cuda(z), _cuda(mask), _cuda(mu), _cuda(t)).cpu().numpy()
    report(f"estimator fp32 B={B} T={T}", rel_err(y32, ref), FP32_TOL)
    dec.compute_dtype = torch.bfloat16
    y16 = dec.estimator(_cuda(z), _cuda(mask), _cuda(mu), _cuda(t)).cpu().numpy()
    d = np.abs(y16.astype(np.float64) - ref) / np.abs(ref).max()
    report(f"estimator bf16 B={B} T={T} (p99.9)", float(np.quantile(d, 0.999)), BF16_EST_P999_TOL)
    report(f"estimator bf16 B={B} T={T}", rel_err(y16, ref), BF16_EST_TOL)


@pytest.mark.parametrize("B,T,lengths,scale", [(2, 256, [256, 190], 10.0), (2, 256, [256, 190], 30.0),
                                              (1, 1024, [1000], 30.0)])
def test_attention_large_logits_fp32(B, T, lengths, scale):
    """LinearAttention's softmax over n = F*T positions (diffusion.py:95) with large logits: k rows of every
    to_qkv scaled by `scale` (|k| reaches the hundreds), Rezero g = 0.5 so the attention term is large. The online
    softmax runs per position tile in log2 units (attn.hip) and its per-tile rescale factors must cancel exactly
    when tiles with different running maxima merge. A peaked softmax is ill-conditioned (at scale 300 the
    reference's own fp32 result is 4.5e-2 from fp64), so the check is against the fp64 oracle, gated at
    max(1e-4, 4 x the oracle's own fp32-vs-fp64 error on the same inputs)."""
    from oracle import decoder as odec
    from gradtts_amd.diffusion import Diffusion
    from gradtts_amd.params import synthetic_inputs, synthetic_state_dict
    sd = synthetic_state_dict(seed=2)
    for k in list(sd):
        if k.endswith("to_qkv.weight"):
            w = sd[k].copy()
            w[128:256] *= scale
            sd[k] = w
        elif k.endswith("fn.g"):
            sd[k] = np.full_like(sd[k], 0.5)
    dec = Diffusion(80, 64, 1, 64, 0.05, 20, 1000, compute_dtype=torch.float32)
    dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    dec = dec.cuda()
    mu, z, mask, _ = synthetic_inputs(17, B, T, lengths=lengths)
    t = np.linspace(0.8, 0.3, B).astype(np.float32)
    ins = [torch.from_numpy(a) for a in (z, mask, mu, t)]
    with torch.no_grad():
        r32 = odec.estimator(odec.to_torch_params(sd), *ins).numpy()
        r64 = odec.estimator({k: v.double() for k, v in odec.to_torch_params(sd).items()},
                             *(a.double() for a in ins)).numpy()
    cond = rel_err(r32, r64)
    y = dec.estimator(_cuda(z), _cuda(mask), _cuda(mu), _cuda(t)).cpu().numpy()
    report(f"attention k x{scale:g} fp32 B={B} T={T} vs fp64 oracle (oracle fp32: {cond:.1e})", rel_err(y, r64),
           max(FP32_TOL, 4 * cond))


@pytest.mark.parametrize("cdt", [torch.bfloat16, torch.float32])
def test_bench_shape_deterministic_and_batch_invariant(cdt):
    """BASELINE config 2 shape (B=32, T=512): finite, bit-identical across runs, and each utterance
    bit-identical to the same utterance decoded in a smaller batch (what an 8-GPU shard computes).
    GroupNorm partial sums are per utterance and reduced in a fixed order, and attention tiles depend only on
    T, so no result depends on atomic order or batch composition. The sub-batch (9 utterances) stays above the
    small-batch plan's threshold (4), so both decodes use the throughput tiles (test_small_batch_gpu.py covers
    the small plan)."""
    from gradtts_amd.params import synthetic_inputs
    dec, _ = make_decoder(1, 0, cdt)
    mu, z, mask, _ = synthetic_inputs(1234, 32, 512)
    zc, mc, muc = _cuda(z), _cuda(mask), _cuda(mu)
    y1 = dec(zc, mc, muc, 3)
    y2 = dec(zc, mc, muc, 3)
    assert torch.isfinite(y1).all()
    sub = dec(zc[5:14].contiguous(), mc[5:14].contiguous(), muc[5:14].contiguous(), 3)
    assert torch.equal(y1, y2), (y1 - y2).abs().max().item()
    assert torch.equal(y1[5:14], sub), (y1[5:14] - sub).abs().max().item()


def test_concurrent_streams_match_one_stream():
    """Two decodes in flight on two HIP streams (each half of a batch) give the same mels as one call on one
    stream: the module's cached scratch is per stream, and the arithmetic is batch-invariant (halves of 5
    utterances: above the small-batch plan's threshold, like the whole batch)."""
    from gradtts_amd.params import synthetic_inputs
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = synthetic_inputs(77, 10, 256)
    zc, mc, muc = _cuda(z), _cuda(mask), _cuda(mu)
    full = dec(zc, mc, muc, 4)
    cur = torch.cuda.current_stream()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for i, st in enumerate(streams):
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            s = slice(5 * i, 5 * i + 5)
            outs.append(dec(zc[s], mc[s], muc[s], 4))
    for st in streams:
        cur.wait_stream(st)
    assert torch.equal(torch.cat(outs), full)


# ---- GT_BF16_W8: fp8 e4m3 weights for the 3x3 / Downsample / Upsample convs, bf16 activations
# (BASELINE.json config 5). Oracle = the reference algorithm run with the dequantized weights
# (oracle.decoder.fp8_params, whose quantizer is bit-identical to the library's: test_fp8_cpu.py);
# tolerances are the bf16 ones. The quantization itself moves one estimator call by ~8e-2 and an
# N = 100 sampler output by ~3e-2 relative to the fp32 weights (synthetic weights).
W8 = "bf16_w8"
W8_STAGE_TOL = 2e-2
# One W8 estimator call: the max element may reach 1.5 x the reference's own bf16 envelope, and the 99.9th
# percentile must stay under 1 x. Measured on estimator_s247: one sensitive element (b=1, f=58, t=25) is the
# max in every build, at 1.39e-2 or 1.96e-2 depending only on the fp32 summation order of the GroupNorm
# partials (two builds, same box), while the 2nd-largest (1.1-1.3e-2), p99.9 (1.01e-2) and mean (1.57e-3) are
# unchanged (tools/diag_w8.py).
W8_EST_MAX_X, W8_EST_P999_X = 1.5, 1.0


@pytest.mark.parametrize("name", EST)
def test_w8_estimator_matches_oracle_dequantized(name):
    from oracle import decoder as odec
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, sd = make_decoder(n_spks, int(g["seed_w"]), W8)
    spk = g["spk"] if n_spks != 1 else None
    with torch.no_grad():
        ref = odec.estimator(odec.fp8_params(sd), *(torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")),
                             torch.from_numpy(spk) if spk is not None else None, n_spks).numpy()
    y = dec.estimator(_cuda(g["x"]), _cuda(g["mask"]), _cuda(g["mu"]), _cuda(g["t"]),
                      _cuda(spk) if spk is not None else None).cpu().numpy()
    env = bf16_est_gate(name) / 1.25   # the reference's own bf16-autocast error on this fixture
    d = np.abs(y.astype(np.float64) - ref) / np.abs(ref).max()
    report(f"w8 estimator {name} vs dequantized oracle (p99.9)", float(np.quantile(d, 0.999)), W8_EST_P999_X * env)
    report(f"w8 estimator {name} vs dequantized oracle", rel_err(y, ref), W8_EST_MAX_X * env)


def test_w8_every_stage_matches_oracle_dequantized():
    from oracle import decoder as odec
    g = load_golden("estimator_s1_T132.npz")
    dec, sd = make_decoder(1, 0, W8)
    taps = {}
    with torch.no_grad():
        odec.estimator(odec.fp8_params(sd), torch.from_numpy(g["x"]), torch.from_numpy(g["mask"]),
                       torch.from_numpy(g["mu"]), torch.from_numpy(g["t"]), None, taps=taps)
    args = [_cuda(g[k]) for k in ("x", "mask", "mu", "t")]
    bad = []
    for st in STAGES:
        ref = taps[st].numpy()
        _, pr = probe(dec.estimator, W8, *args, None, st, ref.shape)
        e = rel_err(pr.cpu().numpy(), ref)
        if not report(f"w8 stage {st}", e, W8_STAGE_TOL, gate=False):
            bad.append(f"{st}: {e:.3e}")
    assert not bad, "stage mismatches: " + ", ".join(bad)


def test_w8_sampler_N1000_matches_oracle_dequantized():
    """Config 5's step count (n_timesteps = 1000) on a small ragged batch the CPU oracle finishes in ~1 min."""
    from oracle import decoder as odec
    from gradtts_amd.params import synthetic_inputs
    dec, sd = make_decoder(1, 0, W8)
    mu, z, mask, _ = synthetic_inputs(11, 2, 16, lengths=[16, 12])
    torch.set_num_threads(min(16, torch.get_num_threads()))
    ref = odec.reverse_diffusion(odec.fp8_params(sd), torch.from_numpy(z), torch.from_numpy(mask),
                                 torch.from_numpy(mu), 1000).numpy()
    y = dec(_cuda(z), _cuda(mask), _cuda(mu), 1000).cpu().numpy()
    report("w8 reverse N=1000 vs dequantized oracle", rel_err(y, ref), BF16_REV_TOL)


def test_w8_bench_shape_deterministic_and_batch_invariant():
    from gradtts_amd.params import synthetic_inputs
    dec, _ = make_decoder(1, 0, W8)
    mu, z, mask, _ = synthetic_inputs(1234, 32, 512)
    zc, mc, muc = _cuda(z), _cuda(mask), _cuda(mu)
    y1 = dec(zc, mc, muc, 3)
    y2 = dec(zc, mc, muc, 3)
    assert torch.isfinite(y1).all()
    # 5 utterances: above the small-batch plan's threshold (4), so both decodes use the throughput tiles
    sub = dec(zc[5:10].contiguous(), mc[5:10].contiguous(), muc[5:10].contiguous(), 3)
    assert torch.equal(y1, y2) and torch.equal(y1[5:10], sub)
    dec.compute_dtype = torch.bfloat16
    y16 = dec(zc, mc, muc, 3)
    assert rel_err(y1.cpu().numpy(), y16.cpu().numpy()) <= 0.1   # quantization moves it, but not far
