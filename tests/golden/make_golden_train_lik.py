#!/usr/bin/env python3
"""Golden fixtures for the training loss and the likelihood rescoring path (§8 f3), produced by
running the REAL reference in this container (the fixtures are data; the reference does not travel).

* loss_*.npz: ``model.diffusion.Diffusion.loss_t`` (/root/reference/model/diffusion.py:274-281, with
  ``forward_diffusion`` :244-252) in float64 and float32 with synthetic weights (seed + SHA-256 stored). The noise
  ``z`` the reference draws with ``torch.randn`` (:249-250) is a fixed draw handed to that call (``fixed_randn``),
  the same for both precisions, and stored. Reference autograd (``loss.backward()``) gives the gradient of every estimator parameter, of ``mu``
  and of ``spk``; stored as a digest per parameter tensor (sum of squares and the projection onto a fixed
  pseudo-random direction, ``grad_probe``) plus the full gradients of ``mu`` and of a few small tensors.
* lik_*.npz: ``n_best/likelihood/likelihood.get_likelihood_fn(sde, lambda x: x, euler=N)`` with the reference's
  ``sde_lib.SPEECHSDE`` on the reference estimator (fp32, as the reference evaluates), the Rademacher probe
  reproduced by seeding and stored, plus one ``drift_fn`` / ``div_fn`` evaluation (likelihood.py:61-68) through the
  reference's ``sde.reverse(...)`` and ``get_div_fn``.

Usage:  make -C oracle ref && PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train_lik.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
sys.dont_write_bytecode = True
from make_golden import REF, build_reference_decoder, import_reference, save  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402
sys.path.insert(0, REPO)
from oracle.decoder import grad_probe  # noqa: E402  (the digest direction; the test side uses the same function)

FULL_GRADS = ("mlp.0.weight", "mlp.2.bias", "final_conv.weight", "final_conv.bias", "downs.0.2.fn.g",
              "mid_attn.fn.g", "downs.0.0.mlp.1.weight", "final_block.block.1.weight")


class fixed_randn:
    """Within the block, torch.randn(shape, dtype=...) returns the fixed draw `z` cast to that dtype (the only
    random draw of Diffusion.loss_t is forward_diffusion's z, diffusion.py:249-250): the fp32 and fp64 reference
    runs see the same noise, which is stored with the fixture. Records the shapes drawn."""

    def __init__(self, z):
        self.z, self.drawn = z, []

    def __enter__(self):
        self.orig = torch.randn

        def randn(*shape, dtype=None, device=None, requires_grad=False, **kw):
            shape = tuple(shape[0]) if len(shape) == 1 and not isinstance(shape[0], int) else shape
            self.drawn.append(tuple(shape))
            assert tuple(shape) == tuple(self.z.shape)
            return self.z.to(dtype=dtype or torch.float32, device=device).clone().requires_grad_(requires_grad)

        torch.randn = randn
        return self.drawn

    def __exit__(self, *exc):
        torch.randn = self.orig
        return False


def loss_case(diffusion, name, n_spks, B, T, lengths, tvals, seed_z, seed_x=41):
    mu, x0, mask, spk = synthetic_inputs(seed_x, B, T, lengths=lengths)
    t = np.asarray(tvals, np.float32)
    z32 = torch.from_numpy(np.random.default_rng(seed_z).standard_normal(x0.shape).astype(np.float32))
    res = {}
    for dt, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        dec, sha = build_reference_decoder(diffusion, n_spks, 0, dt)
        mu_t = torch.from_numpy(mu).to(dt).requires_grad_(True)
        spk_t = torch.from_numpy(spk).to(dt).requires_grad_(True) if n_spks != 1 else None
        with fixed_randn(z32) as drawn:   # the draw of forward_diffusion (diffusion.py:249-250)
            loss, xt = dec.loss_t(torch.from_numpy(x0).to(dt), torch.from_numpy(mask).to(dt), mu_t,
                                  torch.from_numpy(t).to(dt), spk_t)
        assert drawn == [tuple(x0.shape)], drawn
        loss.backward()
        named = dict(dec.estimator.named_parameters())
        keys = list(dec.estimator.state_dict().keys())
        g = [named[k].grad for k in keys]
        res[tag] = dict(loss=float(loss.detach()), xt=xt.detach().numpy(),
                        gsq=np.array([float((gi.double() ** 2).sum()) if gi is not None else 0.0 for gi in g]),
                        gproj=np.array([float((gi.double() * torch.from_numpy(grad_probe(k, tuple(gi.shape)))).sum())
                                        if gi is not None else 0.0 for k, gi in zip(keys, g)]),
                        dmu=mu_t.grad.numpy(), dspk=spk_t.grad.numpy() if spk_t is not None else np.zeros(0),
                        full={k: named[k].grad.numpy() for k in FULL_GRADS if k in named})
    f64, f32 = res["f64"], res["f32"]
    save(name, n_spks=n_spks, seed_w=0, weights_sha256=sha, x0=x0, mu=mu, mask=mask, t=t,
         spk=spk if n_spks != 1 else np.zeros((0,), np.float32), z=z32.numpy(),
         loss=np.float64(f32["loss"]), loss_f64=np.float64(f64["loss"]), xt=f32["xt"],
         param_names=np.array(keys), gsq_f64=f64["gsq"], gproj_f64=f64["gproj"], gsq=f32["gsq"], gproj=f32["gproj"],
         dmu_f64=f64["dmu"], dspk_f64=f64["dspk"], dmu=f32["dmu"],
         **{"full_f64__" + k: v for k, v in f64["full"].items()})


def import_reference_likelihood():
    sys.path.insert(0, os.path.join(REF, "n_best"))
    from likelihood import likelihood, sde_lib   # n_best/likelihood/{likelihood,sde_lib}.py
    return likelihood, sde_lib


class RefScoreModel(torch.nn.Module):
    """The reference's ScoreModel (model/tts.py:239-250): forward(x, t) = estimator(x, y_mask, mu_y, t, spk)."""

    def __init__(self, estimator, y_mask, mu_y, spk):
        super().__init__()
        self.y_mask, self.mu_y, self.spk, self.estimator = y_mask, mu_y, spk, estimator

    def forward(self, x, t):
        return self.estimator(x=x, mask=self.y_mask, mu=self.mu_y, t=t, spk=self.spk)


def lik_case(diffusion, likelihood, sde_lib, name, n_spks, B, T, lengths, n_euler, t_eval, seed_eps, seed_x=51):
    mu, x, mask, spk = synthetic_inputs(seed_x, B, T, lengths=lengths)
    dec, sha = build_reference_decoder(diffusion, n_spks, 0, torch.float32)
    mu_t, mask_t, x_t = torch.from_numpy(mu), torch.from_numpy(mask), torch.from_numpy(x)
    spk_t = torch.from_numpy(spk) if n_spks != 1 else None
    model = RefScoreModel(dec.estimator, mask_t, mu_t, spk_t)
    sde = sde_lib.SPEECHSDE(beta_min=0.05, beta_max=20.0, N=1000, mu=mu_t, spk=spk_t, mask=mask_t)
    torch.manual_seed(seed_eps)
    eps = torch.randint_like(x_t, low=0, high=2).float() * 2 - 1.   # likelihood.py:85-86's draw
    torch.manual_seed(seed_eps)
    bpd, prior_logp, delta_logp, z = likelihood.get_likelihood_fn(sde, lambda v: v, euler=n_euler)(model, x_t)
    # one ODE evaluation (likelihood.py:61-68) at t_eval on the data
    tv = torch.full((B,), float(t_eval))
    rsde = sde.reverse(model, probability_flow=True)
    drift = (rsde.sde(x_t * mask_t, tv)[0] * mask_t).detach()
    div = likelihood.get_div_fn(lambda xx, tt: rsde.sde(xx * mask_t, tt)[0] * mask_t)(x_t.clone(), tv, eps)
    save(name, n_spks=n_spks, seed_w=0, weights_sha256=sha, x=x, mu=mu, mask=mask,
         spk=spk if n_spks != 1 else np.zeros((0,), np.float32), eps=eps.numpy(), n_euler=n_euler,
         bpd=bpd.numpy(), prior_logp=prior_logp.numpy(), delta_logp=delta_logp.numpy(), z=z.numpy(),
         t_eval=np.float32(t_eval), drift=drift.numpy(), div=div.detach().numpy())


def main():
    diffusion, _ = import_reference()
    likelihood, sde_lib = import_reference_likelihood()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    loss_case(diffusion, "loss_s1.npz", 1, 2, 32, [32, 22], [0.73, 0.21], seed_z=7)
    loss_case(diffusion, "loss_s247.npz", 247, 2, 24, [24, 17], [0.41, 0.88], seed_z=8)
    lik_case(diffusion, likelihood, sde_lib, "lik_s1_E3.npz", 1, 2, 24, [24, 15], 3, 0.37, seed_eps=9)
    lik_case(diffusion, likelihood, sde_lib, "lik_s247_E2.npz", 247, 2, 16, [16, 11], 2, 0.62, seed_eps=10)


if __name__ == "__main__":
    main()
