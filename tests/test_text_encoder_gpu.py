"""Text encoder + GradTTS.forward front-end on the MI355X, against the reference's own outputs
(tests/golden/te_*.npz from make_golden_tts.py) and the pinned oracle (oracle/text_encoder.py).

Tolerances (written here): encoder mu_x / logw fp32 vs the reference's fp64 2e-5 x max|ref| (and vs its fp32
2e-5); x_mask exact; the front-end (durations, y_lengths, generate_path, mu_y) exact given the same encoder
outputs; full GradTTS.forward (encoder + front-end + N = 5 decoder, fp32) vs the oracle chain 1e-4 x max|ref|.
"""
import os

import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import rel_err, report
from gradtts_amd.params import synthetic_state_dict, synthetic_text_encoder_state_dict
from gradtts_amd.text_encoder import TextEncoder, align_durations

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def make_encoder(seed):
    enc = TextEncoder(149, 80, 192, 768, 256, 2, 6, 3, 0.1, 4)
    sd = synthetic_text_encoder_state_dict(seed)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return enc.cuda().eval(), sd   # eval: the reference's inference semantics (no dropout)


@pytest.mark.parametrize("name", ["te_B3_T37", "te_B2_T130"])
def test_text_encoder_matches_reference_golden(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    enc, _ = make_encoder(int(g["weights_seed"]))
    with torch.no_grad():   # the inference pass (gt_text_encoder_forward)
        mu, logw, xm = enc(torch.from_numpy(g["tokens"]).cuda(), torch.from_numpy(g["x_lengths"]).cuda())
    # with gradients the training pass runs (gt_text_encoder_forward_train; eval mode: no dropout): same values
    mu_t, logw_t, _ = enc.eval()(torch.from_numpy(g["tokens"]).cuda(), torch.from_numpy(g["x_lengths"]).cuda())
    report(f"text encoder training-pass mu_x {name} vs fp64 reference", rel_err(mu_t.detach().cpu().numpy(),
                                                                                g["mu_x_f64"]), 2e-5)
    report(f"text encoder training-pass logw {name} vs fp64 reference", rel_err(logw_t.detach().cpu().numpy(),
                                                                                g["logw_f64"]), 2e-5)
    torch.cuda.synchronize()
    report(f"text encoder mu_x {name} vs fp64 reference", rel_err(mu.cpu().numpy(), g["mu_x_f64"]), 2e-5)
    report(f"text encoder logw {name} vs fp64 reference", rel_err(logw.cpu().numpy(), g["logw_f64"]), 2e-5)
    report(f"text encoder mu_x {name} vs fp32 reference", rel_err(mu.cpu().numpy(), g["mu_x_f32"]), 2e-5)
    assert np.array_equal(xm.cpu().numpy(), g["x_mask_f32"])


@pytest.mark.parametrize("name", ["te_B3_T37", "te_B2_T130"])
@pytest.mark.parametrize("ls", [1.0, 1.25])
def test_front_end_exact_on_reference_encoder_outputs(name, ls):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    c = lambda a: torch.from_numpy(a).cuda()
    mu_y, y_mask, attn, y_lengths, y_max, w_ceil = align_durations(c(g["mu_x_f32"]), c(g["logw_f32"]),
                                                                   c(g["x_mask_f32"]), ls)
    k = f"ls{int(ls * 100)}"
    # exp on the device vs the reference's CPU exp may differ by an ulp; ceil flips only if w sits on an integer
    w = g[f"{k}_w"]
    assert np.min(np.abs(w - np.round(w))[g["x_mask_f32"] > 0]) > 1e-5
    assert np.array_equal(w_ceil.cpu().numpy(), g[f"{k}_w_ceil"][:, 0])
    assert np.array_equal(y_lengths.cpu().numpy(), g[f"{k}_y_lengths"]) and y_max == int(g[f"{k}_y_max_length"])
    assert np.array_equal(y_mask.cpu().numpy(), g[f"{k}_y_mask"])
    assert np.array_equal(attn.cpu().numpy().astype(np.uint8), g[f"{k}_attn"])
    assert np.array_equal(mu_y.cpu().numpy(), g[f"{k}_mu_y"])


@pytest.mark.parametrize("n_spks", [1, 247])
def test_gradtts_forward_matches_oracle_chain(n_spks):
    from oracle import decoder as odec, text_encoder as ote
    from gradtts_amd.tts import GradTTS
    m = GradTTS(149, n_spks, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000).eval()
    esd = synthetic_text_encoder_state_dict(2)
    dsd = synthetic_state_dict(seed=0, n_spks=n_spks)
    m.encoder.load_state_dict({k: torch.from_numpy(v) for k, v in esd.items()}, strict=True)
    m.decoder.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in dsd.items()}, strict=True)
    spk_ids, spk_vec = None, None
    if n_spks > 1:   # speaker embedding table (tts.py:46) with seeded values; ids looked up as tts.py:78 does
        table = torch.from_numpy(np.random.default_rng(5).standard_normal((n_spks, 64)).astype(np.float32))
        m.spk_emb.weight.data.copy_(table)
        spk_ids = torch.tensor([3, 200])
        spk_vec = table[spk_ids]
    m = m.cuda()
    rng = np.random.default_rng(4)
    B, Tx = 2, 29
    tokens = torch.from_numpy(rng.integers(0, 149, (B, Tx)))
    lengths = torch.tensor([29, 21])
    drawn = []
    randn_like = torch.randn_like

    def record(*a, **k):   # the z draw inside forward (tts.py:102), reused by the oracle chain
        drawn.append(randn_like(*a, **k))
        return drawn[-1]

    torch.randn_like = record
    try:
        enc_out, dec_out, attn = m(tokens.cuda(), lengths.cuda(), n_timesteps=5,
                                   spk=spk_ids.cuda() if spk_ids is not None else None)
    finally:
        torch.randn_like = randn_like
    assert len(drawn) == 1
    # oracle chain: encoder -> front-end -> the same z draw -> reverse diffusion
    mu_x, logw, xm = ote.text_encoder(ote.to_torch_params(esd), tokens, lengths)
    w_ceil, y_len, y_max, y_mask, r_attn, mu_y = ote.front_end(mu_x, logw, xm)
    z = mu_y + drawn[0].cpu()
    r_dec = odec.reverse_diffusion(odec.to_torch_params(dsd), z, y_mask, mu_y, 5, spk_vec, n_spks)
    # the reference slices attn's TEXT axis with y_max_length (tts.py:108): kept as is
    assert enc_out.shape[-1] == y_max and attn.shape == r_attn[:, :, :y_max].shape
    assert np.array_equal(attn.cpu().numpy(), r_attn[:, :, :y_max].numpy())
    report(f"GradTTS.forward encoder outputs n_spks={n_spks}", rel_err(enc_out.cpu().numpy(),
                                                                       mu_y[:, :, :y_max].numpy()), 2e-5)
    report(f"GradTTS.forward decoder outputs (N=5) n_spks={n_spks}",
           rel_err(dec_out.cpu().numpy(), r_dec[:, :, :y_max].numpy()), 1e-4)


def test_text_encoder_speed_vs_torch_eager():
    """Report (no gate): encoder + front-end at B = 32, Tx = 150 against the reference's encoder run eagerly
    (oracle restatement, torch on the same GPU)."""
    import time
    from oracle import text_encoder as ote
    enc, sd = make_encoder(3)
    B, Tx = 32, 150
    rng = np.random.default_rng(6)
    tokens = torch.from_numpy(rng.integers(0, 149, (B, Tx))).cuda()
    lengths = torch.from_numpy(rng.integers(100, Tx + 1, B)).cuda()
    lengths[0] = Tx
    p = {k: v.cuda() for k, v in ote.to_torch_params(sd).items()}

    def ours():
        mu, logw, xm = enc(tokens, lengths)
        return align_durations(mu, logw, xm)

    def eager():
        mu, logw, xm = ote.text_encoder(p, tokens, lengths)
        return ote.front_end(mu, logw, xm)

    def timed(f, n=10):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    with torch.no_grad():   # inference (GradTTS.forward is no_grad)
        ms_ours, ms_eager = timed(ours), timed(eager)
    report(f"text encoder + front-end B={B} Tx={Tx}: ours {ms_ours:.2f} ms, torch eager {ms_eager:.2f} ms; "
           f"ratio eager/ours", ms_eager / ms_ours, 0.0, gate=False, ms_ours=ms_ours, ms_eager=ms_eager)
