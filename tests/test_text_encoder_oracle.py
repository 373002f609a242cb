"""The text-encoder oracle (oracle/text_encoder.py) against the reference's own outputs
(tests/golden/te_*.npz, made by tests/golden/make_golden_tts.py from the real model/text_encoder.py).
Gates: fp64 restatement vs fp64 reference 1e-10 x max|ref|; fp32 vs fp32 1e-5; front-end exact."""
import os

import numpy as np
import pytest
import torch

from gradtts_amd.params import state_dict_sha256, synthetic_text_encoder_state_dict

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("name", ["te_B3_T37", "te_B2_T130"])
def test_oracle_matches_reference_golden(name):
    from oracle import text_encoder as ote
    g = np.load(os.path.join(GOLD, name + ".npz"))
    sd = synthetic_text_encoder_state_dict(int(g["weights_seed"]))
    assert state_dict_sha256(sd) == str(g["weights_sha256"])
    tok, xl = torch.from_numpy(g["tokens"]), torch.from_numpy(g["x_lengths"])
    for tag, dt, tol in (("f64", torch.float64, 1e-10), ("f32", torch.float32, 1e-5)):
        mu, logw, xm = ote.text_encoder(ote.to_torch_params(sd, dt), tok, xl)
        assert _rel(mu.numpy(), g[f"mu_x_{tag}"]) <= tol
        assert _rel(logw.numpy(), g[f"logw_{tag}"]) <= tol
        assert np.array_equal(xm.numpy(), g[f"x_mask_{tag}"])
    for ls in (1.0, 1.25):
        k = f"ls{int(ls * 100)}"
        w_ceil, y_len, y_max, y_mask, attn, mu_y = ote.front_end(torch.from_numpy(g["mu_x_f32"]),
                                                                 torch.from_numpy(g["logw_f32"]),
                                                                 torch.from_numpy(g["x_mask_f32"]), ls)
        assert np.array_equal(w_ceil.numpy(), g[f"{k}_w_ceil"])
        assert np.array_equal(y_len.numpy(), g[f"{k}_y_lengths"]) and y_max == int(g[f"{k}_y_max_length"])
        assert np.array_equal(attn.numpy().astype(np.uint8), g[f"{k}_attn"])
        assert np.array_equal(mu_y.numpy(), g[f"{k}_mu_y"])
