"""Diffusion likelihood of a mel-spectrogram under Grad-TTS's probability-flow ODE: the n-best rescoring path
of the reference, `n_best/likelihood/likelihood.py:27-133` (`get_div_fn`,
`get_likelihood_fn`) with `sde_lib.py:256-297` (`SPEECHSDE`). Same names, arguments and return values.

One ODE evaluation -- the probability-flow drift and its Hutchinson divergence, i.e. an estimator forward plus a
VJP -- is one library call (`gt_likelihood_drift_div`, fp32 on the MI355X). The `euler > 0` branch runs the whole
integration on the device (`gt_likelihood_euler`, fp64 state as the reference's numpy state); the black-box
branch hands the same evaluation to `scipy.integrate.solve_ivp`, as the reference does.
"""
import numpy as np
import torch

from ._lib import check, lib


class SPEECHSDE:
    """`SPEECHSDE(beta_min, beta_max, N, mu, spk, mask)` (sde_lib.py:256-297): the Grad-TTS forward SDE for one
    text (mean `mu` [B, 80, T]) and speaker."""

    def __init__(self, beta_min, beta_max, N, mu, spk, mask):
        self.beta_0 = beta_min
        self.beta_1 = beta_max
        self.N = N
        self.speaker = spk
        self.mask = mask
        self.mu = mu

    @property
    def T(self):
        return 1

    def sde(self, x, t):
        beta_t = self.beta_0 + t * (self.beta_1 - self.beta_0)
        return 0.5 * beta_t[:, None, None] * (self.mu - x), torch.sqrt(beta_t)

    def prior_logp(self, z):
        N = np.prod(z.shape[1:])
        return -N / 2. * np.log(2 * np.pi) - torch.sum((z - self.mu) ** 2, dim=(1, 2)) / 2.


def _f32(a, device):
    return a.to(device=device, dtype=torch.float32).contiguous()


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
        self.B, _, self.T = self.mu.shape
        spk = getattr(model, "spk", sde.speaker)
        self.spk = est._spk(spk, self.B, self.device)

    def handle(self):
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


def get_div_fn(model, sde):
    """`div_fn(x, t, eps)` (likelihood.py:27-38) for the probability-flow drift of `sde` with score `model`: the
    Hutchinson estimate from the library's fused forward + VJP instead of torch.autograd."""
    ev = _Evaluator(model, sde)
    return lambda x, t, eps: ev.drift_div(x, t, eps)[1]


def get_likelihood_fn(sde, inverse_scaler=None, hutchinson_type='Rademacher', rtol=1e-5, atol=1e-5, method='RK45',
                      eps=1e-5, euler=0):
    """`get_likelihood_fn` (likelihood.py:41-133): returns likelihood_fn(model, data) -> (bpd, prior_logp,
    delta_logp, z). `model` is the reference's ScoreModel (`GradTTS.get_score_model`) or the estimator itself;
    `likelihood_fn` also accepts the Hutchinson probe as `epsilon=` (drawn as the reference draws it otherwise)."""

    def likelihood_fn(model, data, epsilon=None):
        with torch.no_grad():
            shape = data.shape
            if epsilon is None:
                if hutchinson_type == 'Gaussian':
                    epsilon = torch.randn_like(data)
                elif hutchinson_type == 'Rademacher':
                    epsilon = torch.randint_like(data, low=0, high=2).float() * 2 - 1.
                else:
                    raise NotImplementedError(f"Hutchinson type {hutchinson_type} unknown.")
            ev = _Evaluator(model, sde)
            if euler > 0:
                z, delta_logp = ev.euler(data, epsilon, euler)
            else:
                from scipy import integrate
                B = shape[0]

                def ode_func(t, x):
                    sample = torch.from_numpy(np.ascontiguousarray(x[:-B]).reshape(shape)).to(data.device)
                    vec_t = torch.ones(B, device=data.device) * t
                    drift, div = ev.drift_div(sample, vec_t, epsilon)
                    return np.concatenate([drift.cpu().numpy().reshape(-1), div.cpu().numpy()], axis=0)

                d = (data * sde.mask).detach().cpu().numpy().reshape(-1)
                init = np.concatenate([d, np.zeros((B,))], axis=0)
                solution = integrate.solve_ivp(ode_func, (eps, sde.T), init, rtol=rtol, atol=atol, method=method)
                zp = solution.y[:, -1]
                z = torch.from_numpy(zp[:-B].reshape(shape)).to(data.device).float()
                delta_logp = torch.from_numpy(zp[-B:]).to(data.device).float()
            prior_logp = sde.prior_logp(z)
            bpd = -(prior_logp + delta_logp)
            return bpd, prior_logp, delta_logp, z

    return likelihood_fn
