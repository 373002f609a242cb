"""Pin the oracle (oracle/decoder.py, oracle/mas.c) against golden vectors from the real reference.

CPU only.  Tolerances: fp32 restatement vs fp32 reference max|d| <= 1e-4 * max|ref|.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from gradtts_amd.params import synthetic_state_dict, state_dict_sha256
from oracle import decoder as odec

EST = ["estimator_s1.npz", "estimator_s247.npz", "estimator_sm1.npz", "estimator_s1_T132.npz",
       "estimator_s1_T20.npz"]


def _params(g):
    sd = synthetic_state_dict(seed=int(g["seed_w"]), n_spks=int(g["n_spks"]))
    assert state_dict_sha256(sd) == str(g["weights_sha256"]), "synthetic weights drifted from the fixture"
    return odec.to_torch_params(sd)


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("name", EST)
def test_oracle_estimator_matches_reference(name):
    g = load_golden(name)
    p = _params(g)
    n_spks = int(g["n_spks"])
    spk = torch.from_numpy(g["spk"]) if n_spks != 1 else None
    with torch.no_grad():
        y = odec.estimator(p, torch.from_numpy(g["x"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["mu"]),
                           torch.from_numpy(g["t"]), spk, n_spks=n_spks).numpy()
    assert _rel(y, g["out"]) <= 1e-5
    assert _rel(g["out"], g["out_f64"]) <= 1e-4   # the fixture's own fp32-vs-fp64 envelope


@pytest.mark.parametrize("name", ["reverse_s1_N1.npz", "reverse_s1_N2.npz", "reverse_s1_N10.npz",
                                  "reverse_s247_N10.npz", "reverse_s1_N10_alone_T100.npz"])
def test_oracle_reverse_diffusion_matches_reference(name):
    g = load_golden(name)
    p = _params(g)
    n_spks = int(g["n_spks"])
    spk = torch.from_numpy(g["spk"]) if n_spks != 1 else None
    y = odec.reverse_diffusion(p, torch.from_numpy(g["z"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["mu"]),
                               int(g["n_timesteps"]), spk, n_spks=n_spks).numpy()
    assert _rel(y, g["out"]) <= 1e-4


def test_padding_dependence_is_real():
    """the same utterance alone vs zero-padded inside a batch differs (GN/attention stats)."""
    batched = load_golden("reverse_s1_N10.npz")["out"][1, :, :100]
    alone = load_golden("reverse_s1_N10_alone_T100.npz")["out"][0]
    assert np.max(np.abs(batched - alone)) > 1e-2


@pytest.mark.parametrize("name", ["mas_random.npz", "mas_ties.npz", "mas_logprior.npz"])
def test_mas_oracle_bit_exact_vs_reference(name, mas_oracle):
    g = load_golden(name)
    value, mask = g["value"], g["mask"]
    t_x = mask.sum(1)[:, 0].astype(np.int32)
    t_y = mask.sum(2)[:, 0].astype(np.int32)
    path, _ = mas_oracle((value * mask).astype(np.float32), t_x, t_y)
    np.testing.assert_array_equal(path, g["path"].astype(np.int32))


def test_mas_known_answers(mas_oracle):
    # t_x == t_y -> identity diagonal; t_x == 1 -> row 0 all ones
    v = np.random.default_rng(0).standard_normal((2, 12, 12)).astype(np.float32)
    p, _ = mas_oracle(v, [12, 1], [12, 12])
    np.testing.assert_array_equal(p[0], np.eye(12, dtype=np.int32))
    assert p[1, 0].sum() == 12 and p[1, 1:].sum() == 0


def test_mas_oracle_vs_reference_build_random(mas_oracle):
    """900 random cases against the reference's own core.pyx compiled into oracle/_ref (if built)."""
    import importlib.util
    import os
    import sysconfig
    from conftest import REPO
    so = os.path.join(REPO, "oracle", "_ref", "core" + sysconfig.get_config_var("EXT_SUFFIX"))
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built (make -C oracle ref needs /root/reference)")
    spec = importlib.util.spec_from_file_location("core", so)
    core = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(core)
    rng = np.random.default_rng(123)
    for it in range(900):
        b = int(rng.integers(1, 4))
        txm, tym = int(rng.integers(1, 30)), int(rng.integers(1, 60))
        t_x = rng.integers(1, txm + 1, b).astype(np.int32)
        t_y = np.array([rng.integers(tx, max(tx, tym) + 1) for tx in t_x], np.int32)
        tym = max(tym, int(t_y.max()))
        if it % 2:
            v = rng.integers(-3, 4, (b, txm, tym)).astype(np.float32)
        else:
            v = rng.standard_normal((b, txm, tym)).astype(np.float32)
        ref_paths = np.zeros((b, txm, tym), np.int32)
        ref_v = v.copy()
        core.maximum_path_c(ref_paths, ref_v, t_x, t_y)
        paths, vals = mas_oracle(v, t_x, t_y)
        np.testing.assert_array_equal(paths, ref_paths)
        np.testing.assert_array_equal(vals, ref_v)
