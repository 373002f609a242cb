"""Training-path forward values on the MI355X, against the oracle restatements
(oracle/decoder.py: forward_diffusion / loss_t / log_prior, citing model/diffusion.py:244-287 and model/tts.py:141-152)
and the C MAS oracle.

Tolerances (written here): forward_diffusion fp32 elementwise 1e-6 x max|ref| (expf/sqrtf ulp differences);
loss_t fp32 rel 1e-5, bf16 rel 1e-2 (the score's bf16 envelope, summed); log-prior fp32 1e-6 x max|ref|;
alignment paths bit-exact against the C MAS oracle run on the same log-prior.
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
    loss, xt = dec.loss_t(c(x0), c(mask), c(mu), c(t), s, z=c(z))
    rloss, rxt = odec.loss_t(odec.to_torch_params(sd), *(torch.from_numpy(a) for a in (x0, mask, mu, t, z)),
                             torch.from_numpy(spk) if n_spks > 1 else None, n_spks)
    report(f"loss_t {cdt} n_spks={n_spks} (loss {float(loss):.5f} vs {float(rloss):.5f})",
           abs(float(loss) - float(rloss)) / abs(float(rloss)), tol)
    report(f"loss_t xt {cdt}", rel_err(xt.cpu().numpy(), rxt.numpy()), 1e-6)


def test_compute_loss_seeded_deterministic_and_backward_raises():
    x0, mu, mask, _, _, _ = _data(7, 2, 64, [64, 52])
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    c = lambda a: torch.from_numpy(a).cuda()
    torch.manual_seed(11)
    l1, _ = dec.compute_loss(c(x0), c(mask), c(mu))
    torch.manual_seed(11)
    l2, _ = dec.compute_loss(c(x0), c(mask), c(mu))
    assert torch.isfinite(l1) and torch.equal(l1, l2)
    assert l1.requires_grad
    with pytest.raises(NotImplementedError, match="backward"):
        l1.backward()


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
