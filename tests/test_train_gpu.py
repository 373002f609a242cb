"""Training-path forward values on the MI355X, against the oracle restatements
(oracle/decoder.py: forward_diffusion / loss_t / log_prior, citing model/diffusion.py:244-287 and model/tts.py:141-152)
and the C MAS oracle.

Tolerances (written here): forward_diffusion fp32 elementwise 1e-6 x max|ref| (expf/sqrtf ulp differences);
loss_t fp32 rel 1e-5, bf16 rel 1e-2 (the score's bf16 envelope, summed); log-prior fp32 1e-6 x max|ref|;
alignment paths bit-exact against the C MAS oracle run on the same log-prior.
Training step (gt_diffusion_loss_grad, fp32): loss rel 1e-5; every parameter gradient, d mu and d spk against
torch.autograd through the oracle in fp64: max|g - ref| <= 2e-4 x (max|ref| of that tensor + 1e-3 x the largest
max|ref| over all tensors) -- the floor covers the conv biases feeding a GroupNorm, whose exact gradient is 0.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder, rel_err, report
from gradtts_amd.alignment import mas_alignment
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _data(seed, B, T, lengths):
    mu, z, mask, spk = synthetic_inputs(seed, B, T, lengths=lengths)
    rng = np.random.default_rng(seed + 1)
    x0 = (mu + 0.5 * rng.standard_normal(mu.shape)).astype(np.float32)
    noise = rng.standard_normal(mu.shape).astype(np.float32)
    t = rng.uniform(1e-5, 1 - 1e-5, B).astype(np.float32)
    return x0, mu, mask, noise, t, spk


def test_forward_diffusion_matches_oracle():
    from oracle import decoder as odec
    x0, mu, mask, z, t, _ = _data(3, 3, 96, [96, 60, 88])
    dec, _ = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    xt, zm = dec.forward_diffusion(c(x0), c(mask), c(mu), c(t), z=c(z))
    rxt, rzm = odec.forward_diffusion(*(torch.from_numpy(a) for a in (x0, mask, mu, t, z)))
    report("forward_diffusion xt fp32", rel_err(xt.cpu().numpy(), rxt.numpy()), 1e-6)
    assert np.array_equal(zm.cpu().numpy(), rzm.numpy())


@pytest.mark.parametrize("cdt,tol,n_spks", [(torch.float32, 1e-5, 1), (torch.bfloat16, 1e-2, 1),
                                            (torch.float32, 1e-5, 247)])
def test_loss_t_matches_oracle(cdt, tol, n_spks):
    from oracle import decoder as odec
    x0, mu, mask, z, t, spk = _data(5, 2, 64, [64, 44])
    dec, sd = make_decoder(n_spks, 0, cdt)
    c = lambda a: torch.from_numpy(a).cuda()
    s = c(spk) if n_spks > 1 else None
    with torch.no_grad():   # forward value in the compute dtype (with gradients the fp32 training step runs)
        loss, xt = dec.loss_t(c(x0), c(mask), c(mu), c(t), s, z=c(z))
    rloss, rxt = odec.loss_t(odec.to_torch_params(sd), *(torch.from_numpy(a) for a in (x0, mask, mu, t, z)),
                             torch.from_numpy(spk) if n_spks > 1 else None, n_spks)
    report(f"loss_t {cdt} n_spks={n_spks} (loss {float(loss):.5f} vs {float(rloss):.5f})",
           abs(float(loss) - float(rloss)) / abs(float(rloss)), tol)
    report(f"loss_t xt {cdt}", rel_err(xt.cpu().numpy(), rxt.numpy()), 1e-6)


def _oracle_grads(sd, x0, mask, mu, t, z, spk, n_spks):
    """torch.autograd through the oracle's loss_t in fp64 (oracle/decoder.py, diffusion.py:274-281)."""
    from oracle import decoder as odec
    d = lambda a: torch.from_numpy(a).double()
    p = {k: v.double().requires_grad_() for k, v in odec.to_torch_params(sd).items()}
    mu_t = d(mu).requires_grad_()
    spk_t = d(spk).requires_grad_() if n_spks > 1 else None
    x0_t, mask_t, t_t, z_t = d(x0), d(mask), d(t), d(z)
    xt, zm = odec.forward_diffusion(x0_t, mask_t, mu_t, t_t, z_t)
    cum = odec.get_noise(t_t[:, None, None], 0.05, 20.0, cumulative=True)
    ne = odec.estimator(p, xt, mask_t, mu_t, t_t, spk_t, n_spks) * torch.sqrt(1.0 - torch.exp(-cum))
    loss = torch.sum((ne + zm) ** 2) / (torch.sum(mask_t) * 80)
    loss.backward()
    return float(loss), {k: v.grad.numpy() for k, v in p.items()}, mu_t.grad.numpy(), \
        (spk_t.grad.numpy() if spk_t is not None else None)


@pytest.mark.parametrize("n_spks,B,T,lengths", [(1, 2, 64, [64, 44]), (247, 2, 32, [32, 21]), (1, 1, 40, [40])])
def test_training_step_gradients_match_autograd(n_spks, B, T, lengths):
    x0, mu, mask, z, t, spk = _data(9 + n_spks, B, T, lengths)
    dec, sd = make_decoder(n_spks, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    mu_d = c(mu).requires_grad_()
    s = c(spk).requires_grad_() if n_spks > 1 else None
    loss, _ = dec.loss_t(c(x0), c(mask), mu_d, c(t), s, z=c(z))
    loss.backward()
    rloss, rgrads, rdmu, rdspk = _oracle_grads(sd, x0, mask, mu, t, z, spk, n_spks)
    report(f"train loss n_spks={n_spks} B={B} T={T}", abs(float(loss) - rloss) / abs(rloss), 1e-5)
    gmax = max(float(np.abs(g).max()) for g in rgrads.values())
    params = dict(dec.estimator.named_parameters())
    worst, worst_name = 0.0, None
    for name, rg in rgrads.items():
        g = params[name].grad
        assert g is not None, name
        g = g.detach().cpu().numpy().astype(np.float64)
        err = float(np.abs(g - rg).max()) / (float(np.abs(rg).max()) + 1e-3 * gmax)
        if err > worst:
            worst, worst_name = err, name
    report(f"train param grads n_spks={n_spks} B={B} T={T} (worst {worst_name})", worst, 2e-4)
    report(f"train d mu n_spks={n_spks}", rel_err(mu_d.grad.cpu().numpy(), rdmu), 2e-4)
    if n_spks > 1:
        report(f"train d spk n_spks={n_spks}", rel_err(s.grad.cpu().numpy(), rdspk), 2e-4)


def test_training_step_deterministic_and_optimizer_step():
    """Two identical calls give bit-identical gradients; an SGD step on them lowers the loss on the same draw and
    the next call picks up the updated parameters (the handle re-syncs on the parameters' versions)."""
    x0, mu, mask, z, t, _ = _data(13, 2, 64, [64, 50])
    dec, _ = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    args = (c(x0), c(mask), c(mu), c(t))
    params = list(dec.estimator.parameters())
    grads = []
    for _ in range(2):
        dec.zero_grad(set_to_none=True)
        loss, _ = dec.loss_t(*args, z=c(z))
        loss.backward()
        grads.append([p.grad.clone() for p in params])
    assert all(torch.equal(a, b) for a, b in zip(*grads))
    opt = torch.optim.SGD(params, lr=1e-3)
    opt.step()
    with torch.no_grad():
        loss2, _ = dec.loss_t(*args, z=c(z))
    assert float(loss2) < float(loss), (float(loss2), float(loss))


def test_compute_loss_seeded_deterministic_with_backward():
    x0, mu, mask, _, _, _ = _data(7, 2, 64, [64, 52])
    dec, _ = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    torch.manual_seed(11)
    l1, _ = dec.compute_loss(c(x0), c(mask), c(mu))
    torch.manual_seed(11)
    l2, _ = dec.compute_loss(c(x0), c(mask), c(mu))
    assert torch.isfinite(l1) and torch.equal(l1, l2)
    assert l1.requires_grad
    l1.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in dec.estimator.parameters())


@pytest.mark.parametrize("B,Tx,Ty", [(3, 37, 150), (2, 130, 400), (4, 61, 1000)])
def test_log_prior_alignment(B, Tx, Ty, mas_oracle):
    from oracle import decoder as odec
    rng = np.random.default_rng(Tx)
    mu_x = rng.standard_normal((B, 80, Tx)).astype(np.float32)
    tx = np.maximum(1, (Tx * rng.uniform(0.5, 1.0, B)).astype(int)); tx[0] = Tx
    ty = np.maximum(tx, (Ty * rng.uniform(0.6, 1.0, B)).astype(int)); ty[0] = Ty
    x_mask = (np.arange(Tx)[None] < tx[:, None]).astype(np.float32)
    y_mask = (np.arange(Ty)[None] < ty[:, None]).astype(np.float32)
    # y: mu_x expanded over random durations plus noise (a realistic log-prior landscape)
    idx = np.sort(rng.integers(0, Tx, (B, Ty)), axis=1)
    y = (np.take_along_axis(mu_x, idx[:, None, :], axis=2) + 0.3 * rng.standard_normal((B, 80, Ty))).astype(np.float32)
    attn, lp = mas_alignment(torch.from_numpy(mu_x).cuda(), torch.from_numpy(y).cuda(),
                             torch.from_numpy(x_mask[:, None]).cuda(), torch.from_numpy(y_mask[:, None]).cuda(),
                             return_log_prior=True)
    attn_mask = x_mask[:, :, None] * y_mask[:, None, :]
    ref_lp = (odec.log_prior(torch.from_numpy(mu_x), torch.from_numpy(y)).numpy() * attn_mask).astype(np.float32)
    lp = lp.cpu().numpy()
    report(f"log_prior B={B} Tx={Tx} Ty={Ty}", rel_err(lp, ref_lp), 1e-6)
    path_same_lp, _ = mas_oracle(lp, tx, ty)                    # MAS oracle on our log-prior: bit-exact
    assert np.array_equal(attn.cpu().numpy().astype(np.int32), path_same_lp)
    path_ref_lp, _ = mas_oracle(ref_lp, tx, ty)                 # ... and on the oracle's own log-prior
    agree = float((path_ref_lp == path_same_lp).mean())
    report(f"alignment B={B} Tx={Tx} Ty={Ty} path agreement with the oracle log-prior", 1.0 - agree, 1e-3)


def test_training_step_speed_vs_torch_eager():
    """Report (no gate) the training-step time at the reference's training shape (params.py: batch 16, out_size
    2 s = 172 frames) against torch eager autograd of the same loss on the same GPU (MIOpen convs, fp32)."""
    import time
    from oracle import decoder as odec
    B, T = 16, 172
    x0, mu, mask, z, t, _ = _data(21, B, T, None)
    dec, sd = make_decoder(1, 0, torch.float32)
    c = lambda a: torch.from_numpy(a).cuda()
    args = (c(x0), c(mask), c(mu), c(t))
    zz = c(z)

    def ours():
        dec.zero_grad(set_to_none=True)
        loss, _ = dec.loss_t(*args, z=zz)
        loss.backward()

    p = {k: v.cuda().requires_grad_() for k, v in odec.to_torch_params(sd).items()}
    x0_t, mask_t, mu_t, t_t = args

    def eager():
        for v in p.values():
            v.grad = None
        xt, zm = odec.forward_diffusion(x0_t, mask_t, mu_t, t_t, zz)
        cum = odec.get_noise(t_t[:, None, None], 0.05, 20.0, cumulative=True)
        ne = odec.estimator(p, xt, mask_t, mu_t, t_t) * torch.sqrt(1.0 - torch.exp(-cum))
        loss = torch.sum((ne + zm) ** 2) / (torch.sum(mask_t) * 80)
        loss.backward()

    def timed(fn, n=5):
        fn(); fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    ms_ours, ms_eager = timed(ours), timed(eager)
    frames = B * T
    report(f"training step B={B} T={T}: ours {ms_ours:.2f} ms ({frames / ms_ours * 1e3:.0f} frames/s), torch eager "
           f"{ms_eager:.2f} ms ({frames / ms_eager * 1e3:.0f} frames/s); ratio eager/ours", ms_eager / ms_ours, 0.0,
           gate=False, ms_ours=ms_ours, ms_eager=ms_eager)


@pytest.mark.parametrize("name", ["loss_s1.npz", "loss_s247.npz"])
def test_training_step_matches_reference_fixture(name):
    """The training step against the REAL reference (tests/golden/make_golden_train_lik.py: Diffusion.loss_t +
    loss.backward() in fp64 with the same noise): loss rel 1e-5 against the reference's fp32 value; every parameter
    gradient's digest (norm and random projection, oracle.decoder.grad_digest) within 2e-4 of the reference's fp64
    gradients relative to that tensor's norm (+ 1e-3 of the largest norm); d mu / d spk 2e-4."""
    from conftest import load_golden
    from oracle import decoder as odec
    g = load_golden(name)
    n_spks = int(g["n_spks"])
    dec, _ = make_decoder(n_spks, int(g["seed_w"]), torch.float32)
    c = lambda k: torch.from_numpy(np.ascontiguousarray(g[k])).cuda()
    mu_d = c("mu").requires_grad_()
    s = c("spk").requires_grad_() if n_spks > 1 else None
    loss, xt = dec.loss_t(c("x0"), c("mask"), mu_d, c("t"), s, z=c("z"))
    loss.backward()
    report(f"train loss vs reference {name}", abs(float(loss) - float(g["loss"])) / abs(float(g["loss"])), 1e-5)
    report(f"train xt vs reference {name}", rel_err(xt.detach().cpu().numpy(), g["xt"]), 1e-6)
    names = [str(n) for n in g["param_names"]]
    params = dict(dec.estimator.named_parameters())
    grads = {k: params[k].grad.detach().cpu().numpy().astype(np.float64) for k in names}
    gsq, gproj = odec.grad_digest(grads, names)
    rn = np.sqrt(g["gsq_f64"])
    floor = 1e-3 * rn.max()
    err = np.maximum(np.abs(np.sqrt(gsq) - rn), np.abs(gproj - g["gproj_f64"])) / (rn + floor)
    report(f"train param grad digests vs reference {name} (worst {names[int(err.argmax())]})", float(err.max()), 2e-4)
    for k in list(g):
        if k.startswith("full_f64__"):
            report(f"train grad {k[10:]} vs reference", rel_err(grads[k[10:]], g[k]), 2e-4)
    report(f"train d mu vs reference {name}", rel_err(mu_d.grad.cpu().numpy(), g["dmu_f64"]), 2e-4)
    if n_spks > 1:
        report(f"train d spk vs reference {name}", rel_err(s.grad.cpu().numpy(), g["dspk_f64"]), 2e-4)
