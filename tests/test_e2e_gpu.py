"""End-to-end inference: text -> GradTTS.forward (text encoder, durations, alignment, N-step
decoder) -> HiFi-GAN -> audio, every stage on the MI355X, against the oracle chain (oracle/text_encoder.py ->
oracle/decoder.py -> oracle/vocoder.py) with the same noise draw. Gate (fp32): audio 1e-4 x max|ref|. Plus the
end-to-end real-time factor (report only)."""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import rel_err, report
from gradtts_amd.params import (HIFIGAN_V1, synthetic_state_dict, synthetic_text_encoder_state_dict,
                                synthetic_vocoder_state_dict)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def build(compute_dtype=torch.float32, vocoder_dtype=torch.float32):
    from gradtts_amd.tts import GradTTS
    from gradtts_amd.vocoder import Generator
    m = GradTTS(149, 1, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000, compute_dtype=compute_dtype)
    esd, dsd, vsd = synthetic_text_encoder_state_dict(2), synthetic_state_dict(seed=0), synthetic_vocoder_state_dict(7)
    m.encoder.load_state_dict({k: torch.from_numpy(v) for k, v in esd.items()}, strict=True)
    m.decoder.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in dsd.items()}, strict=True)
    voc = Generator(HIFIGAN_V1, compute_dtype=vocoder_dtype)
    voc.load_state_dict({k: torch.from_numpy(v) for k, v in vsd.items()}, strict=True)
    voc.remove_weight_norm()
    return m.cuda().eval(), voc.cuda().eval(), (esd, dsd, vsd)   # eval: inference semantics (no dropout)


def run(m, voc, tokens, lengths, n_timesteps, drawn=None):
    randn_like = torch.randn_like
    if drawn is not None:
        def record(*a, **k):
            drawn.append(randn_like(*a, **k))
            return drawn[-1]
        torch.randn_like = record
    try:
        enc, dec, attn = m(tokens, lengths, n_timesteps=n_timesteps)
    finally:
        torch.randn_like = randn_like
    return voc(dec), dec


def test_text_to_audio_matches_oracle_chain():
    from oracle import decoder as odec, text_encoder as ote, vocoder as ov
    m, voc, (esd, dsd, vsd) = build()
    rng = np.random.default_rng(21)
    tokens = torch.from_numpy(rng.integers(0, 149, (2, 23)))
    lengths = torch.tensor([23, 16])
    drawn = []
    audio, dec = run(m, voc, tokens.cuda(), lengths.cuda(), 3, drawn)
    mu_x, logw, xm = ote.text_encoder(ote.to_torch_params(esd), tokens, lengths)
    _, _, y_max, y_mask, _, mu_y = ote.front_end(mu_x, logw, xm)
    z = mu_y + drawn[0].cpu()
    r_dec = odec.reverse_diffusion(odec.to_torch_params(dsd), z, y_mask, mu_y, 3)[:, :, :y_max]
    r_audio = ov.generator(ov.to_torch_params(vsd), r_dec)
    assert audio.shape == r_audio.shape
    report("text -> audio (N=3, fp32) vs oracle chain", rel_err(audio.cpu().numpy(), r_audio.numpy()), 1e-4)


@pytest.mark.parametrize("B,Tx,N,dtype", [(1, 120, 50, torch.bfloat16), (32, 120, 50, torch.bfloat16)])
def test_end_to_end_rtf(B, Tx, N, dtype):
    """Report (no gate): wall time per stage and the real-time factor (wall / seconds of audio at 22.05 kHz)."""
    import time
    from gradtts_amd.text_encoder import align_durations
    m, voc, _ = build(dtype, dtype)
    rng = np.random.default_rng(22)
    tokens = torch.from_numpy(rng.integers(0, 149, (B, Tx))).cuda()
    lengths = torch.full((B,), Tx, dtype=torch.int64).cuda()

    def once():
        t0 = time.perf_counter()
        mu_x, logw, xm = m.encoder(tokens, lengths)
        mu_y, y_mask, attn, _, y_max, _ = align_durations(mu_x, logw, xm)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        z = mu_y + torch.randn_like(mu_y)
        dec = m.decoder(z, y_mask, mu_y, N)[:, :, :y_max]
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        audio = voc(dec)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        return (t1 - t0, t2 - t1, t3 - t2), audio.shape[-1]

    once()
    times, n_samples = once()
    total = sum(times)
    sec = B * n_samples / 22050
    report(f"end-to-end B={B} Tx={Tx} N={N} decoder + vocoder {str(dtype)[6:]}: encoder+align {times[0] * 1e3:.1f} ms, decoder "
           f"{times[1] * 1e3:.1f} ms, vocoder {times[2] * 1e3:.1f} ms; {sec:.1f} s of audio, RTF", total / sec, 0.0,
           gate=False, ms=[t * 1e3 for t in times], audio_s=sec)
