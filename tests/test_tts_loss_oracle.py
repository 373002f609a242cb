"""The compute_loss oracle (oracle/tts_loss.py) against the reference's own GradTTS.compute_loss
(tests/golden/tts_loss_*.npz from tests/golden/make_golden_tts_loss.py), and the dropout-mask restatement.
CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from gradtts_amd.params import state_dict_sha256, synthetic_state_dict, synthetic_text_encoder_state_dict
from oracle import tts_loss
from oracle.decoder import grad_digest
from oracle.text_encoder import dropout_keep


def fixture_inputs(g):
    enc = synthetic_text_encoder_state_dict(int(g["seed_enc"]))
    dec = synthetic_state_dict(seed=int(g["seed_dec"]))
    sd = {f"encoder.{k}": v for k, v in enc.items()}
    sd.update({f"decoder.estimator.{k}": v for k, v in dec.items()})
    assert state_dict_sha256(sd) == str(g["weights_sha256"])
    return enc, dec


def run_oracle(g, mas, dtype=torch.float64, drop=None):
    enc, dec = fixture_inputs(g)
    ep, dp = tts_loss.params(enc, dtype), tts_loss.params(dec, dtype)
    out_size = int(g["out_size"])
    dur, prior, diff, attn = tts_loss.compute_loss(ep, dp, g["tokens"], g["x_lengths"], g["y"], g["y_lengths"],
                                                   g["offsets"], out_size if out_size > 0 else None, g["t"], g["z"],
                                                   mas, drop=drop, dtype=dtype)
    (dur + prior + diff).backward()
    grads = {f"encoder.{k}": v.grad.numpy() for k, v in ep.items()}
    grads.update({f"decoder.estimator.{k}": v.grad.numpy() for k, v in dp.items()})
    return np.array([float(dur), float(prior), float(diff)]), grads, attn


@pytest.mark.parametrize("name", ["tts_loss_B2.npz", "tts_loss_B3_nocut.npz", "tts_loss_B2_short.npz"])
def test_oracle_compute_loss_matches_reference(name, mas_oracle):
    g = load_golden(name)
    losses, grads, _ = run_oracle(g, mas_oracle)
    np.testing.assert_allclose(losses, g["losses_f64"], rtol=1e-10, atol=0)
    names = [str(n) for n in g["param_names"]]
    gsq, gproj = grad_digest(grads, names)
    np.testing.assert_allclose(gsq, g["gsq_f64"], rtol=1e-8, atol=1e-30)
    np.testing.assert_allclose(gproj, g["gproj_f64"], rtol=1e-7, atol=1e-12 * np.abs(g["gproj_f64"]).max())
    for k in g:
        if k.startswith("full__"):
            np.testing.assert_allclose(grads[k[6:]], g[k], rtol=1e-8, atol=1e-14)


def test_dropout_keep_rate_and_determinism():
    idx = np.arange(1 << 20)
    for p in (0.1, 0.5):
        s = dropout_keep(1234, 17, idx, p)
        assert set(np.unique(s)) == {0.0, 1.0 / (1.0 - p)}
        rate = float((s > 0).mean())
        assert abs(rate - (1 - p)) < 4e-3, rate
        np.testing.assert_array_equal(s, dropout_keep(1234, 17, idx, p))
        assert (s != dropout_keep(1234, 18, idx, p)).mean() > 0.5 * 2 * p * (1 - p)   # sites are independent
    np.testing.assert_array_equal(dropout_keep(5, 1, idx[:10], 0.0), np.ones(10))
