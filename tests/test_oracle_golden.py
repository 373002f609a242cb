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


# ---- (f1) training loss and its gradients, (f3) likelihood: fixtures from the real reference
# (tests/golden/make_golden_train_lik.py: Diffusion.loss_t + loss.backward(); n_best likelihood_fn / drift_fn /
# get_div_fn with the reference SPEECHSDE)

def _grad_digest_err(gsq, gproj, rsq, rproj):
    """Relative error of the per-parameter gradient digests: sqrt(sum g^2) within 1e-3 of the reference norm, the
    projection onto a random direction within 1e-3 of it (plus 1e-3 of the largest norm: biases ahead of a
    GroupNorm have an exact gradient of 0)."""
    rn = np.sqrt(rsq)
    floor = 1e-3 * rn.max()
    e_norm = np.abs(np.sqrt(gsq) - rn) / (rn + floor)
    e_proj = np.abs(gproj - rproj) / (rn + floor)
    return float(max(e_norm.max(), e_proj.max()))


@pytest.mark.parametrize("name", ["loss_s1.npz", "loss_s247.npz"])
def test_oracle_loss_and_gradients_match_reference(name):
    g = load_golden(name)
    p = _params(g)
    sd = {k: v.numpy() for k, v in p.items()}
    n_spks = int(g["n_spks"])
    spk = g["spk"] if n_spks != 1 else None
    args = (g["x0"], g["mask"], g["mu"], g["t"])
    # fp32 forward value against the reference's fp32 loss_t
    loss32, xt = odec.loss_t(p, *(torch.from_numpy(a) for a in args), torch.from_numpy(g["z"]),
                             torch.from_numpy(spk) if spk is not None else None, n_spks)
    assert abs(float(loss32) - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))
    assert _rel(xt.numpy(), g["xt"]) <= 1e-6
    # fp64 autograd against the reference's fp64 loss.backward()
    loss, grads, dmu, dspk = odec.loss_t_grads(sd, *args, g["z"], spk, n_spks)
    assert abs(loss - float(g["loss_f64"])) <= 1e-10 * abs(float(g["loss_f64"]))
    names = [str(n) for n in g["param_names"]]
    gsq, gproj = odec.grad_digest(grads, names)
    assert _grad_digest_err(gsq, gproj, g["gsq_f64"], g["gproj_f64"]) <= 1e-8
    assert _rel(dmu, g["dmu_f64"]) <= 1e-9
    if spk is not None:
        assert _rel(dspk, g["dspk_f64"]) <= 1e-9
    for k in list(g):
        if k.startswith("full_f64__"):
            assert _rel(grads[k[len("full_f64__"):]], g[k]) <= 1e-9, k
    # the reference's own fp32-vs-fp64 envelope of the digest (what an fp32 implementation can reach)
    assert _grad_digest_err(g["gsq"], g["gproj"], g["gsq_f64"], g["gproj_f64"]) <= 1e-4


@pytest.mark.parametrize("name", ["lik_s1_E3.npz", "lik_s247_E2.npz"])
def test_oracle_likelihood_matches_reference(name):
    from oracle import likelihood as olik
    g = load_golden(name)
    p = _params(g)
    n_spks = int(g["n_spks"])
    c = lambda k: torch.from_numpy(np.ascontiguousarray(g[k]))
    spk = c("spk") if n_spks != 1 else None
    B = g["x"].shape[0]
    tv = torch.full((B,), float(g["t_eval"]))
    drift = olik.drift_fn(p, c("x"), c("mask"), c("mu"), tv, spk, n_spks)
    div = olik.div_fn(p, c("x"), c("mask"), c("mu"), tv, c("eps"), spk, n_spks)
    assert _rel(drift.detach().numpy(), g["drift"]) <= 1e-5
    assert float(np.max(np.abs(div.numpy() - g["div"]) / np.abs(g["div"]))) <= 1e-4
    # the whole euler > 0 likelihood (likelihood.py:99-115) in fp32, as the reference evaluates it
    bpd, pl, dl, z = olik.likelihood_euler(p, c("x"), c("mask"), c("mu"), c("eps"), int(g["n_euler"]), spk, n_spks,
                                           dtype=torch.float32)
    assert _rel(z.numpy(), g["z"]) <= 1e-5
    assert float(np.max(np.abs(dl.numpy() - g["delta_logp"]) / np.abs(g["delta_logp"]))) <= 1e-4
    assert float(np.max(np.abs(bpd.numpy() - g["bpd"]) / np.abs(g["bpd"]))) <= 1e-5
    assert float(np.max(np.abs(pl.numpy() - g["prior_logp"]) / np.abs(g["prior_logp"]))) <= 1e-5
