"""CPU restatement of the reference's diffusion-likelihood path -- TEST INFRASTRUCTURE ONLY:
imported by tests/ (never by the product). Pinned through oracle.decoder.estimator (itself pinned to the
reference's golden vectors); the likelihood algebra below follows the reference line by line:

* drift_fn        n_best/likelihood/likelihood.py:61-65 with SPEECHSDE.sde (sde_lib.py:278-282) and the
                  probability-flow reverse drift (sde_lib.py:93-100): drift = (0.5 beta (mu - x m)
                  - sqrt(beta)^2 s(x m) 0.5) m, s = the estimator on (x m, mask, mu, t, spk)
* div_fn          likelihood.py:27-38, 67-68: Hutchinson trace estimate through torch.autograd.grad
* euler           likelihood.py:99-107, 113-115: numpy float64 state, t_i = (i + 0.5) h
* prior_logp      sde_lib.py:293-297
"""
import numpy as np
import torch

from oracle import decoder as odec


def drift_fn(p, x, mask, mu, t, spk=None, n_spks=1, beta_min=0.05, beta_max=20.0):
    x = x * mask
    beta_t = beta_min + t * (beta_max - beta_min)
    drift = 0.5 * beta_t[:, None, None] * (mu - x)
    diffusion = torch.sqrt(beta_t)
    s = odec.estimator(p, x, mask, mu, t, spk, n_spks)
    drift = drift - diffusion[:, None, None] ** 2 * s * 0.5
    return drift * mask


def div_fn(p, x, mask, mu, t, eps, spk=None, n_spks=1, beta_min=0.05, beta_max=20.0):
    with torch.enable_grad():
        x = x.detach().requires_grad_(True)
        fn_eps = torch.sum(drift_fn(p, x, mask, mu, t, spk, n_spks, beta_min, beta_max) * eps)
        g = torch.autograd.grad(fn_eps, x)[0]
    return torch.sum(g * eps, dim=tuple(range(1, len(x.shape))))


def estimator_vjp(p, x, mask, mu, t, v, spk=None, n_spks=1):
    """(score, (d score / d x)^T v) by autograd -- the quantity gt_estimator_vjp returns."""
    with torch.enable_grad():
        x = x.detach().requires_grad_(True)
        s = odec.estimator(p, x, mask, mu, t, spk, n_spks)
        g = torch.autograd.grad(torch.sum(s * v), x)[0]
    return s.detach(), g


def prior_logp(z, mu):
    N = np.prod(z.shape[1:])
    return -N / 2. * np.log(2 * np.pi) - torch.sum((z - mu) ** 2, dim=(1, 2)) / 2.


def likelihood_euler(p, data, mask, mu, eps, n_steps, spk=None, n_spks=1, beta_min=0.05, beta_max=20.0,
                     dtype=torch.float64):
    """likelihood_fn's euler > 0 branch: returns (bpd, prior_logp, delta_logp, z). Evaluations run in `dtype`
    (fp64 for a truth reference; the reference itself evaluates in fp32)."""
    shape = data.shape
    B = shape[0]
    data = data * mask
    y = np.concatenate([data.numpy().reshape(-1).astype(np.float64), np.zeros((B,))])
    h = 1 / n_steps
    for i in range(n_steps):
        t = (i + 0.5) * h
        sample = torch.from_numpy(y[:-B].reshape(shape)).to(dtype)
        vec_t = torch.ones(B, dtype=dtype) * t
        cast = lambda a: a.to(dtype) if a is not None else None
        dr = drift_fn({k: cast(v) for k, v in p.items()}, sample, cast(mask), cast(mu), vec_t, cast(spk), n_spks,
                      beta_min, beta_max)
        dv = div_fn({k: cast(v) for k, v in p.items()}, sample, cast(mask), cast(mu), vec_t, cast(eps), cast(spk),
                    n_spks, beta_min, beta_max)
        f = np.concatenate([dr.detach().numpy().reshape(-1), dv.detach().numpy()])
        y = y + f.astype(np.float64) * h
    z = torch.from_numpy(y[:-B].reshape(shape)).float()
    delta = torch.from_numpy(y[-B:]).float()
    pl = prior_logp(z, mu)
    return -(pl + delta), pl, delta, z
