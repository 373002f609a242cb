"""Likelihood rescoring path on the MI355X against the oracle (oracle/likelihood.py: the
reference's drift_fn / div_fn / Euler loop, n_best/likelihood/likelihood.py:27-133, sde_lib.py:256-297, with
torch.autograd through oracle.decoder.estimator in fp64).

Tolerances (written here): estimator output fp32 1e-5 x max|ref|; VJP and drift 2e-5 x max|ref| (fp32 forward +
backward against fp64); divergence 1e-4 relative; Euler likelihood (3 steps) delta_logp and bpd 1e-4 relative,
z 1e-5 x max|ref|.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder, rel_err, report
from gradtts_amd import _lib
from gradtts_amd.diffusion import _stream_ptr
from gradtts_amd.likelihood import SPEECHSDE, _Evaluator as _Ev, get_div_fn, get_fused_div_fn, get_likelihood_fn
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _case(seed, B, T, lengths, n_spks):
    mu, z, mask, spk = synthetic_inputs(seed, B, T, lengths=lengths)
    rng = np.random.default_rng(seed + 7)
    x = (mu + rng.standard_normal(mu.shape)).astype(np.float32)
    eps = (rng.integers(0, 2, mu.shape) * 2 - 1).astype(np.float32)
    t = rng.uniform(0.05, 0.95, B).astype(np.float32)
    return x, mu, mask, eps, t, (spk if n_spks > 1 else None)


@pytest.mark.parametrize("n_spks,B,T,lengths", [(1, 2, 32, [32, 20]), (247, 2, 24, [24, 17])])
def test_estimator_vjp_matches_autograd(n_spks, B, T, lengths):
    from oracle import decoder as odec, likelihood as olik
    x, mu, mask, v, t, spk = _case(3, B, T, lengths, n_spks)
    dec, sd = make_decoder(n_spks, 0, torch.float32)
    est = dec.estimator
    c = lambda a: torch.from_numpy(a).cuda()
    h = est._native()
    L = _lib.lib()
    score = torch.empty(B, 80, T, device="cuda")
    vjp = torch.empty(B, 80, T, device="cuda")
    ws = torch.empty(L.gt_estimator_vjp_workspace_bytes(h, B, T), dtype=torch.uint8, device="cuda")
    s_d = c(spk) if spk is not None else None
    args = [c(a) for a in (x, mask, mu, t, v)]
    _lib.check(L.gt_estimator_vjp(h, args[0].data_ptr(), args[1].data_ptr(), args[2].data_ptr(), args[3].data_ptr(),
                                  s_d.data_ptr() if s_d is not None else None, args[4].data_ptr(), B, T,
                                  score.data_ptr(), vjp.data_ptr(), ws.data_ptr(), ws.numel(),
                                  _stream_ptr(torch.device("cuda"))), "gt_estimator_vjp")
    d = lambda a: torch.from_numpy(a).double() if a is not None else None
    p = {k: v_.double() for k, v_ in odec.to_torch_params(sd).items()}
    rs, rg = olik.estimator_vjp(p, d(x), d(mask), d(mu), d(t), d(v), d(spk), n_spks)
    report(f"estimator (vjp pass) n_spks={n_spks}", rel_err(score.cpu().numpy(), rs.numpy()), 1e-5)
    report(f"estimator VJP n_spks={n_spks}", rel_err(vjp.cpu().numpy(), rg.numpy()), 2e-5)


@pytest.mark.parametrize("n_spks", [1, 247])
def test_drift_and_divergence_match_oracle(n_spks):
    from oracle import decoder as odec, likelihood as olik
    B, T = 2, 32
    x, mu, mask, eps, t, spk = _case(5, B, T, [32, 26], n_spks)
    dec, sd = make_decoder(n_spks, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda() if a is not None else None
    sde = SPEECHSDE(0.05, 20.0, 1000, c(mu), c(spk), c(mask))
    from gradtts_amd.likelihood import _Evaluator
    drift, div = _Evaluator(dec.estimator, sde).drift_div(c(x), c(t), c(eps))
    d = lambda a: torch.from_numpy(a).double() if a is not None else None
    p = {k: v_.double() for k, v_ in odec.to_torch_params(sd).items()}
    rd = olik.drift_fn(p, d(x), d(mask), d(mu), d(t), d(spk), n_spks)
    rdiv = olik.div_fn(p, d(x), d(mask), d(mu), d(t), d(eps), d(spk), n_spks)
    report(f"likelihood drift n_spks={n_spks}", rel_err(drift.cpu().numpy(), rd.detach().numpy()), 2e-5)
    report(f"likelihood divergence n_spks={n_spks}", float(np.max(np.abs(div.cpu().numpy() - rdiv.numpy()) /
                                                                    np.abs(rdiv.numpy()))), 1e-4)
    # the fused entry point under its own name returns the same divergence
    div2 = get_fused_div_fn(dec.estimator, sde)(c(x), c(t), c(eps))
    assert torch.equal(div, div2)
    # the reference's own formulation, get_div_fn(fn) with torch.autograd through the estimator (its backward is
    # the device VJP) around the reference's drift_fn (likelihood.py:61-68), gives the same divergence
    rsde = sde.reverse(lambda xx, tt: dec.estimator(xx, c(mask), c(mu), tt, c(spk)), probability_flow=True)
    div3 = get_div_fn(lambda xx, tt: rsde.sde(xx * c(mask), tt)[0] * c(mask))(c(x), c(t), c(eps))
    report(f"get_div_fn(fn) autograd vs fused divergence n_spks={n_spks}",
           float((div3 - div).abs().max() / div.abs().max()), 1e-5)


def test_likelihood_euler_matches_oracle():
    from oracle import decoder as odec, likelihood as olik
    B, T, N = 2, 24, 3
    x, mu, mask, eps, _, _ = _case(9, B, T, [24, 15], 1)
    dec, sd = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    sde = SPEECHSDE(0.05, 20.0, 1000, c(mu), None, c(mask))
    bpd, pl, dl, z = get_likelihood_fn(sde, euler=N)(dec.estimator, c(x), epsilon=c(eps))
    p = {k: v_.double() for k, v_ in odec.to_torch_params(sd).items()}
    rbpd, rpl, rdl, rz = olik.likelihood_euler(p, torch.from_numpy(x), torch.from_numpy(mask), torch.from_numpy(mu),
                                               torch.from_numpy(eps), N)
    report("likelihood Euler z", rel_err(z.cpu().numpy(), rz.numpy()), 1e-5)
    report("likelihood Euler delta_logp", float(np.max(np.abs(dl.cpu().numpy() - rdl.numpy()) / np.abs(rdl.numpy()))),
           1e-4)
    report("likelihood Euler bpd", float(np.max(np.abs(bpd.cpu().numpy() - rbpd.numpy()) / np.abs(rbpd.numpy()))),
           1e-4)
    assert torch.isfinite(bpd).all()


def test_likelihood_blackbox_rk45_runs_and_agrees_with_euler():
    """The solve_ivp branch drives the same evaluation; at a loose tolerance its likelihood agrees with a fine
    Euler integration of the same ODE (both ours) to the ODE-solver accuracy."""
    B, T = 1, 16
    x, mu, mask, eps, _, _ = _case(11, B, T, None, 1)
    dec, _ = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    sde = SPEECHSDE(0.05, 20.0, 1000, c(mu), None, c(mask))
    bpd_rk, _, dl_rk, _ = get_likelihood_fn(sde, rtol=1e-4, atol=1e-4)(dec.estimator, c(x), epsilon=c(eps))
    bpd_eu, _, dl_eu, _ = get_likelihood_fn(sde, euler=200)(dec.estimator, c(x), epsilon=c(eps))
    assert torch.isfinite(bpd_rk).all()
    report("likelihood RK45 vs Euler-200 bpd", float(abs(bpd_rk - bpd_eu).max() / abs(bpd_eu).max()), 2e-2)


def test_likelihood_speed_vs_torch_eager():
    """Report (no gate) the n-best rescoring workload of the reference (n_best/config/generate_scores.yaml:
    n_euler = 10; a batch of 16 hypotheses of 172 frames) against the reference's own algorithm run eagerly on the
    same GPU (torch autograd for the divergence, numpy fp64 state between steps as likelihood.py:92-107)."""
    import time
    from oracle import decoder as odec, likelihood as olik
    B, T, N = 16, 172, 10
    x, mu, mask, eps, _, _ = _case(13, B, T, None, 1)
    dec, sd = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    sde = SPEECHSDE(0.05, 20.0, 1000, c(mu), None, c(mask))
    fn = get_likelihood_fn(sde, euler=N)
    ours = lambda: fn(dec.estimator, c(x), epsilon=c(eps))
    p = {k: v_.cuda() for k, v_ in odec.to_torch_params(sd).items()}
    mu_d, mask_d, eps_d = c(mu), c(mask), c(eps)

    def eager():
        y = np.concatenate([(x * mask).reshape(-1).astype(np.float64), np.zeros((B,))])
        for i in range(N):
            t = (i + 0.5) / N
            sample = torch.from_numpy(y[:-B].reshape(x.shape)).cuda().float()
            vt = torch.ones(B, device="cuda") * t
            dr = olik.drift_fn(p, sample, mask_d, mu_d, vt)
            dv = olik.div_fn(p, sample, mask_d, mu_d, vt, eps_d)
            y = y + np.concatenate([dr.detach().cpu().numpy().reshape(-1), dv.cpu().numpy()]) * (1 / N)
        return y

    def timed(f, n=3):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    ms_ours, ms_eager = timed(ours), timed(eager)
    report(f"likelihood B={B} T={T} n_euler={N}: ours {ms_ours:.1f} ms, torch eager {ms_eager:.1f} ms; "
           f"ratio eager/ours", ms_eager / ms_ours, 0.0, gate=False, ms_ours=ms_ours, ms_eager=ms_eager)


def test_get_score_model_and_rescoring_chain(mas_oracle):
    """GradTTS.get_score_model (tts.py:196-254: encoder, log-prior + MAS, mu_y = attn^T mu_x) and the rescoring
    call of n_best (get_score_parallel.py:68-85: SPEECHSDE + get_likelihood_fn(euler) on the score model) against
    the oracle chain (oracle text encoder -> log-prior -> C MAS oracle -> oracle likelihood, fp64)."""
    from oracle import decoder as odec, likelihood as olik, text_encoder as ote
    from gradtts_amd.params import synthetic_text_encoder_state_dict
    from gradtts_amd.tts import GradTTS
    m = GradTTS(149, 1, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000).eval()
    esd, dsd = synthetic_text_encoder_state_dict(2), None
    dec, dsd = make_decoder(1, 0, torch.float32)
    m.encoder.load_state_dict({k: torch.from_numpy(v) for k, v in esd.items()}, strict=True)
    m.decoder.estimator.load_state_dict(dec.estimator.state_dict(), strict=True)
    m = m.cuda()
    rng = np.random.default_rng(31)
    B, Tx, Ty = 2, 15, 40
    tokens = torch.from_numpy(rng.integers(0, 149, (B, Tx)))
    x_lengths, y_lengths = torch.tensor([15, 11]), torch.tensor([40, 32])
    y = torch.from_numpy((rng.standard_normal((B, 80, Ty)) * 0.5).astype(np.float32))
    score_model, mu_y, spk, y_mask = m.get_score_model(tokens.cuda(), x_lengths.cuda(), y.cuda(), y_lengths.cuda())
    mu_x, _, xm = ote.text_encoder(ote.to_torch_params(esd), tokens, x_lengths)
    ym = (torch.arange(Ty)[None] < y_lengths[:, None]).unsqueeze(1).float()
    lp = (odec.log_prior(mu_x, y) * (xm.transpose(1, 2) * ym)).numpy()
    path, _ = mas_oracle(lp, x_lengths.numpy(), y_lengths.numpy())
    r_mu_y = torch.matmul(torch.from_numpy(path).float().transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
    report("get_score_model mu_y", rel_err(mu_y.cpu().numpy(), r_mu_y.numpy()), 2e-5)
    eps = torch.from_numpy((rng.integers(0, 2, (B, 80, Ty)) * 2 - 1).astype(np.float32))
    sde = SPEECHSDE(0.05, 20.0, 1000, mu_y, spk, y_mask)
    bpd, _, dl, _ = get_likelihood_fn(sde, lambda x: x, rtol=1e-3, atol=1e-3, euler=2)(score_model, y.cuda(),
                                                                                      epsilon=eps.cuda())
    p = {k: v_.double() for k, v_ in odec.to_torch_params(dsd).items()}
    rbpd, _, rdl, _ = olik.likelihood_euler(p, y, ym, r_mu_y, eps, 2)
    report("rescoring bpd (get_score_model + euler 2)", float(np.max(np.abs(bpd.cpu().numpy() - rbpd.numpy()) /
                                                                      np.abs(rbpd.numpy()))), 1e-4)


@pytest.mark.parametrize("name", ["lik_s1_E3.npz", "lik_s247_E2.npz"])
def test_likelihood_matches_reference_fixture(name):
    """Against the REAL reference (tests/golden/make_golden_train_lik.py: n_best likelihood_fn with euler steps, the
    reference SPEECHSDE and Rademacher probe; one drift_fn / get_div_fn evaluation), fp32 as the reference runs:
    drift 2e-5 x max, divergence 1e-4 rel, z 2e-5 x max, delta_logp / prior_logp / bpd 1e-4 rel -- through the fused
    device path and through the reference's own autograd formulation (get_div_fn(fn) over the estimator)."""
    from conftest import load_golden
    from gradtts_amd.tts import ScoreModel
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), torch.float32)
    c = lambda k: torch.from_numpy(np.ascontiguousarray(g[k])).cuda()
    spk = c("spk") if n_spks != 1 else None
    mu, mask, x, eps = c("mu"), c("mask"), c("x"), c("eps")
    sde = SPEECHSDE(beta_min=0.05, beta_max=20.0, N=1000, mu=mu, spk=spk, mask=mask)
    model = ScoreModel(dec.estimator, mask, mu, spk)
    rel = lambda a, b: float(np.max(np.abs(a - b) / np.abs(b)))
    B = x.shape[0]
    tv = torch.full((B,), float(g["t_eval"]), device="cuda")
    drift, div = _Ev(model, sde).drift_div(x, tv, eps)
    report(f"likelihood drift vs reference {name}", rel_err(drift.cpu().numpy(), g["drift"]), 2e-5)
    report(f"likelihood div vs reference {name}", rel(div.cpu().numpy(), g["div"]), 1e-4)
    rsde = sde.reverse(model, probability_flow=True)
    div_ag = get_div_fn(lambda xx, tt: rsde.sde(xx * mask, tt)[0] * mask)(x.clone(), tv, eps)
    report(f"likelihood get_div_fn(fn) autograd vs reference {name}", rel(div_ag.cpu().numpy(), g["div"]), 1e-4)
    bpd, pl, dl, z = get_likelihood_fn(sde, lambda v: v, euler=int(g["n_euler"]))(model, x, epsilon=eps)
    report(f"likelihood z vs reference {name}", rel_err(z.cpu().numpy(), g["z"]), 2e-5)
    report(f"likelihood delta_logp vs reference {name}", rel(dl.cpu().numpy(), g["delta_logp"]), 1e-4)
    report(f"likelihood prior_logp vs reference {name}", rel(pl.cpu().numpy(), g["prior_logp"]), 1e-4)
    report(f"likelihood bpd vs reference {name}", rel(bpd.cpu().numpy(), g["bpd"]), 1e-4)
