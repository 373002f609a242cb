"""Diffusion likelihood of a mel-spectrogram under Grad-TTS's probability-flow ODE: the n-best rescoring path
of the reference, `n_best/likelihood/likelihood.py:27-133` (`get_div_fn`,
`get_likelihood_fn`) with `sde_lib.py:256-297` (`SPEECHSDE`). Same names, arguments and return values:

* ``SPEECHSDE(beta_min, beta_max, N, mu, spk, mask)`` with VPSDE's members (``discrete_betas``, ``alphas``,
  ``alphas_cumprod``, ``marginal_prob``, ``prior_sampling``, ``discretize``, ``reverse``; sde_lib.py:111-161, 66-105);
* ``get_div_fn(fn)`` -- the Hutchinson-Skilling estimator through ``torch.autograd`` (likelihood.py:27-38). The
  estimator of this package is differentiable in ``x`` (its backward is the device VJP, gt_estimator_vjp), so the
  reference's autograd formulation runs on the MI355X unchanged;
* ``get_likelihood_fn(sde, inverse_scaler, ...)`` -> ``likelihood_fn(model, data)`` -> (bpd, prior_logp,
  delta_logp, z).

When ``model`` is this package's score model (``GradTTS.get_score_model``'s ``ScoreModel`` or the estimator) on
the SDE's own ``mu`` / ``mask``, one ODE evaluation -- the drift and its Hutchinson divergence, i.e. an estimator
forward plus a VJP -- is one library call (``gt_likelihood_drift_div``, fp32; ``get_fused_div_fn`` exposes it), and
the ``euler > 0`` branch runs the whole integration on the device (``gt_likelihood_euler``, fp64 state as the
reference's numpy state). The black-box branch hands the same evaluation to ``scipy.integrate.solve_ivp``, as the
reference does. Any other ``model`` takes the reference's own composition (``sde.reverse`` + ``get_div_fn``).
"""
import numpy as np
import torch

from ._lib import check, lib
from .diffusion import _check_binary_mask


class SPEECHSDE:
    """`SPEECHSDE(beta_min, beta_max, N, mu, spk, mask)` (sde_lib.py:256-297): the Grad-TTS forward SDE for one
    text (mean `mu` [B, 80, T]) and speaker, with the members it inherits from VPSDE (sde_lib.py:111-161)."""

    def __init__(self, beta_min, beta_max, N, mu, spk, mask):
        self.beta_0 = beta_min
        self.beta_1 = beta_max
        self.N = N
        self.discrete_betas = torch.linspace(beta_min / N, beta_max / N, N)
        self.alphas = 1. - self.discrete_betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.sqrt_alphas_cumprod = torch.sqrt(self.alphas_cumprod)
        self.sqrt_1m_alphas_cumprod = torch.sqrt(1. - self.alphas_cumprod)
        self.speaker = spk
        self.mask = mask
        self.mu = mu

    @property
    def T(self):
        return 1

    def sde(self, x, t):
        beta_t = self.beta_0 + t * (self.beta_1 - self.beta_0)
        return 0.5 * beta_t[:, None, None] * (self.mu - x), torch.sqrt(beta_t)

    def marginal_prob(self, x, t):
        log_mean_coeff = -0.25 * t ** 2 * (self.beta_1 - self.beta_0) - 0.5 * t * self.beta_0
        c = torch.exp(log_mean_coeff[:, None, None, None])
        return c * x + (1 - c) * self.mu, torch.sqrt(1. - torch.exp(2. * log_mean_coeff))

    def prior_sampling(self):
        return self.mu + torch.randn_like(self.mu)

    def prior_logp(self, z):
        N = np.prod(z.shape[1:])
        return -N / 2. * np.log(2 * np.pi) - torch.sum((z - self.mu) ** 2, dim=(1, 2)) / 2.

    def discretize(self, x, t):
        """VPSDE's DDPM discretization (sde_lib.py:154-161), inherited unchanged by SPEECHSDE."""
        timestep = (t * (self.N - 1) / self.T).long()
        beta = self.discrete_betas.to(x.device)[timestep]
        alpha = self.alphas.to(x.device)[timestep]
        return torch.sqrt(alpha)[:, None, None, None] * x - x, torch.sqrt(beta)

    def reverse(self, score_fn, probability_flow=False):
        """SDE.reverse (sde_lib.py:66-105): the reverse-time SDE / probability-flow ODE of this SDE."""
        fwd = self

        class RSDE:
            def __init__(self):
                self.N = fwd.N
                self.probability_flow = probability_flow

            @property
            def T(self):
                return fwd.T

            def sde(self, x, t):
                drift, diffusion = fwd.sde(x, t)
                score = score_fn(x, t)
                drift = drift - diffusion[:, None, None] ** 2 * score * (0.5 if self.probability_flow else 1.)
                return drift, (0. if self.probability_flow else diffusion)

            def discretize(self, x, t):
                f, G = fwd.discretize(x, t)
                rev_f = f - G[:, None, None, None] ** 2 * score_fn(x, t) * (0.5 if self.probability_flow else 1.)
                return rev_f, (torch.zeros_like(G) if self.probability_flow else G)

        return RSDE()


def get_div_fn(fn):
    """`get_div_fn(fn)` (likelihood.py:27-38): div_fn(x, t, eps) = sum(eps * d(sum(fn(x, t) * eps))/dx)."""

    def div_fn(x, t, eps):
        with torch.enable_grad():
            x.requires_grad_(True)
            fn_eps = torch.sum(fn(x, t) * eps)
            grad_fn_eps = torch.autograd.grad(fn_eps, x)[0]
        x.requires_grad_(False)
        return torch.sum(grad_fn_eps * eps, dim=tuple(range(1, len(x.shape))))

    return div_fn


def _f32(a, device):
    return a.to(device=device, dtype=torch.float32).contiguous()


def _fusable(model, sde):
    """The fused device evaluation applies when `model` is this package's estimator or a ScoreModel over it whose
    mask / mu are the SDE's (as GradTTS.get_score_model + SPEECHSDE build them, n_best_list_experiment.py:79-87)."""
    from .diffusion import GradLogPEstimator2d
    if isinstance(model, GradLogPEstimator2d):
        return True
    est = getattr(model, "estimator", None)
    if not isinstance(est, GradLogPEstimator2d):
        return False
    same = lambda a, b: a is b or (a is not None and b is not None and a.shape == b.shape and torch.equal(
        a.to(b.device, b.dtype), b))
    return same(getattr(model, "mu_y", sde.mu), sde.mu) and same(getattr(model, "y_mask", sde.mask), sde.mask)


class _Evaluator:
    """Binds an estimator and an SDE to the library's drift/divergence entry points."""

    def __init__(self, model, sde):
        est = getattr(model, "estimator", model)
        self.est = est
        self.sde = sde
        self.device = sde.mu.device
        if self.device.type != "cuda":
            raise RuntimeError("gradtts_amd.likelihood needs a HIP (MI355X) device; there is no CPU path")
        self.mu = _f32(sde.mu, self.device)
        self.mask = _f32(sde.mask, self.device)
        _check_binary_mask(self.mask)
        self.B, _, self.T = self.mu.shape
        spk = getattr(model, "spk", sde.speaker)
        self.spk = est._spk(spk, self.B, self.device)

    def handle(self):
        # the SDE's schedule; a scalar update of the shared handle (gt_decoder_set_betas), weights stay packed
        return self.est._native(self.sde.beta_0, self.sde.beta_1)

    def workspace(self, h):
        return torch.empty(lib().gt_likelihood_workspace_bytes(h, self.B, self.T), dtype=torch.uint8,
                           device=self.device)

    def drift_div(self, x, t, eps):
        from .diffusion import _stream_ptr
        with torch.cuda.device(self.device):
            h = self.handle()
            x32, t32, e32 = _f32(x, self.device), _f32(t, self.device), _f32(eps, self.device)
            drift = torch.empty_like(x32)
            div = torch.empty(self.B, dtype=torch.float32, device=self.device)
            ws = self.workspace(h)
            check(lib().gt_likelihood_drift_div(h, x32.data_ptr(), self.mask.data_ptr(), self.mu.data_ptr(),
                                                t32.data_ptr(), self.spk.data_ptr() if self.spk is not None else None,
                                                e32.data_ptr(), self.B, self.T, drift.data_ptr(), div.data_ptr(),
                                                ws.data_ptr(), ws.numel(), _stream_ptr(self.device)),
                  "gt_likelihood_drift_div")
        return drift, div

    def euler(self, data, eps, n_steps):
        from .diffusion import _stream_ptr
        with torch.cuda.device(self.device):
            h = self.handle()
            d32, e32 = _f32(data, self.device), _f32(eps, self.device)
            z = torch.empty_like(d32)
            dlogp = torch.empty(self.B, dtype=torch.float32, device=self.device)
            ws = self.workspace(h)
            check(lib().gt_likelihood_euler(h, d32.data_ptr(), self.mask.data_ptr(), self.mu.data_ptr(),
                                            self.spk.data_ptr() if self.spk is not None else None, e32.data_ptr(),
                                            self.B, self.T, int(n_steps), z.data_ptr(), dlogp.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _stream_ptr(self.device)),
                  "gt_likelihood_euler")
        return z, dlogp


def get_fused_div_fn(model, sde):
    """div_fn(x, t, eps) of the probability-flow drift of `sde` with score `model` (likelihood.py:67-68) as one
    device call: the estimator forward + VJP fused with the drift algebra (gt_likelihood_drift_div)."""
    ev = _Evaluator(model, sde)
    return lambda x, t, eps: ev.drift_div(x, t, eps)[1]


def get_likelihood_fn(sde, inverse_scaler=None, hutchinson_type='Rademacher', rtol=1e-5, atol=1e-5, method='RK45',
                      eps=1e-5, euler=0):
    """`get_likelihood_fn` (likelihood.py:41-133): returns likelihood_fn(model, data) -> (bpd, prior_logp,
    delta_logp, z). `likelihood_fn` also accepts the Hutchinson probe as `epsilon=` (drawn as the reference draws
    it otherwise)."""

    def drift_fn(model, x, t):      # likelihood.py:61-65
        rsde = sde.reverse(model, probability_flow=True)
        x = x * sde.mask
        return rsde.sde(x, t)[0] * sde.mask

    def div_fn(model, x, t, noise):   # likelihood.py:67-68
        return get_div_fn(lambda xx, tt: drift_fn(model, xx, tt))(x, t, noise)

    def likelihood_fn(model, data, epsilon=None):
        with torch.no_grad():
            shape = data.shape
            B = shape[0]
            if epsilon is None:
                if hutchinson_type == 'Gaussian':
                    epsilon = torch.randn_like(data)
                elif hutchinson_type == 'Rademacher':
                    epsilon = torch.randint_like(data, low=0, high=2).float() * 2 - 1.
                else:
                    raise NotImplementedError(f"Hutchinson type {hutchinson_type} unknown.")
            if _fusable(model, sde):
                ev = _Evaluator(model, sde)
                evaluate = lambda sample, vec_t: ev.drift_div(sample, vec_t, epsilon)
            else:
                ev = None
                evaluate = lambda sample, vec_t: (drift_fn(model, sample, vec_t), div_fn(model, sample, vec_t, epsilon))
            if euler > 0 and ev is not None:
                z, delta_logp = ev.euler(data, epsilon, euler)
            else:
                def ode_func(t, x):          # likelihood.py:92-97
                    sample = torch.from_numpy(np.ascontiguousarray(x[:-B]).reshape(shape)).to(data.device).float()
                    vec_t = torch.ones(B, device=sample.device) * t
                    drift, div = evaluate(sample, vec_t)
                    return np.concatenate([drift.detach().cpu().numpy().reshape(-1),
                                           div.detach().cpu().numpy().reshape(-1)], axis=0)

                d = (data * sde.mask).detach().cpu().numpy().reshape(-1)
                init = np.concatenate([d, np.zeros((B,))], axis=0)
                if euler > 0:                # likelihood.py:99-107, host state for a foreign model
                    y, h = init, 1 / euler
                    for i in range(euler):
                        y = y + ode_func((i + 0.5) * h, y) * h
                    zp = y
                else:
                    from scipy import integrate
                    solution = integrate.solve_ivp(ode_func, (eps, sde.T), init, rtol=rtol, atol=atol, method=method)
                    zp = solution.y[:, -1]
                z = torch.from_numpy(zp[:-B].reshape(shape)).to(data.device).float()
                delta_logp = torch.from_numpy(zp[-B:]).to(data.device).float()
            prior_logp = sde.prior_logp(z)
            bpd = -(prior_logp + delta_logp)
            return bpd, prior_logp, delta_logp, z

    return likelihood_fn
