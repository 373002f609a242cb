"""HiFi-GAN generator (the vocoder) on the MI355X against the reference Generator's own outputs
(tests/golden/voc_*.npz, made by make_golden_vocoder.py from the real hifi-gan/models.py) and the pinned oracle.

Tolerances (written here): audio fp32 vs the reference's fp64 1e-5 x max|ref| (fp32 MFMA convs in a different
summation order through 4 stages x 18 resblock convs); larger random shapes vs the fp32 oracle 1e-5. The bf16
throughput mode (operands rounded to bf16, fp32 accumulation): 2e-2 x max|ref| against fp64, error printed."""
import os

import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import rel_err, report
from gradtts_amd.params import HIFIGAN_V1, HIFIGAN_V3, synthetic_vocoder_state_dict
from gradtts_amd.vocoder import Generator

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def make_vocoder(seed, compute_dtype=torch.float32, h=HIFIGAN_V1):
    g = Generator(h, compute_dtype=compute_dtype)
    sd = synthetic_vocoder_state_dict(seed, h)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    g.remove_weight_norm()
    return g.cuda().eval(), sd


@pytest.mark.parametrize("name,h", [("voc_B2_T6", HIFIGAN_V1), ("voc_B1_T13", HIFIGAN_V1),
                                    ("voc3_B2_T7", HIFIGAN_V3)])   # voc3: HiFi-GAN V3, ResBlock2
def test_vocoder_matches_reference_golden(name, h):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    voc, _ = make_vocoder(int(g["weights_seed"]), h=h)
    audio = voc(torch.from_numpy(g["mel"]).cuda())
    torch.cuda.synchronize()
    assert audio.shape == g["audio_f64"].shape
    report(f"vocoder audio {name} vs fp64 reference", rel_err(audio.cpu().numpy(), g["audio_f64"]), 1e-5)
    report(f"vocoder audio {name} vs fp32 reference", rel_err(audio.cpu().numpy(), g["audio_f32"]), 1e-5)


@pytest.mark.parametrize("name,h", [("voc_B2_T6", HIFIGAN_V1), ("voc_B1_T13", HIFIGAN_V1),
                                    ("voc3_B2_T7", HIFIGAN_V3)])
def test_vocoder_bf16_mode_within_envelope(name, h):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    voc, _ = make_vocoder(int(g["weights_seed"]), torch.bfloat16, h)
    audio = voc(torch.from_numpy(g["mel"]).cuda())
    report(f"vocoder bf16 mode audio {name} vs fp64 reference", rel_err(audio.cpu().numpy(), g["audio_f64"]), 2e-2)


def test_vocoder_matches_oracle_longer():
    from oracle import vocoder as ov
    voc, sd = make_vocoder(3)
    rng = np.random.default_rng(8)
    mel = (rng.standard_normal((2, 80, 37)) * 2.0 - 5.0).astype(np.float32)
    audio = voc(torch.from_numpy(mel).cuda()).cpu().numpy()
    ref = ov.generator(ov.to_torch_params(sd, torch.float64), torch.from_numpy(mel).double()).numpy()
    report("vocoder audio B=2 T=37 vs fp64 oracle", rel_err(audio, ref), 1e-5)


def test_vocoder_speed_vs_torch_eager():
    """Report (no gate): 2 s of audio per utterance (172 frames), B = 16, against the reference Generator's
    algorithm eagerly on the same GPU (oracle restatement: torch conv1d / conv_transpose1d, MIOpen, fp32)."""
    import time
    from oracle import vocoder as ov
    voc, sd = make_vocoder(4)
    B, T = 16, 172
    mel = torch.randn(B, 80, T, device="cuda") * 2.0 - 5.0
    p = {k: v.cuda() for k, v in ov.to_torch_params(sd).items()}

    def timed(f, n=5):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    voc16, _ = make_vocoder(4, torch.bfloat16)
    with torch.no_grad():
        ms_ours = timed(lambda: voc(mel))
        ms_bf16 = timed(lambda: voc16(mel))
        ms_eager = timed(lambda: ov.generator(p, mel))
    sec = B * T * 256 / 22050
    report(f"vocoder B={B} T={T} ({sec:.1f} s of audio): ours fp32 {ms_ours:.1f} ms (RTF {ms_ours / 1e3 / sec:.5f}), "
           f"ours bf16 {ms_bf16:.1f} ms (RTF {ms_bf16 / 1e3 / sec:.5f}), torch eager fp32 {ms_eager:.1f} ms; "
           f"ratio eager/ours-fp32", ms_eager / ms_ours, 0.0, gate=False, ms_ours=ms_ours, ms_bf16=ms_bf16,
           ms_eager=ms_eager)
