"""Drop-in ``Diffusion`` / ``GradLogPEstimator2d`` backed by the gfx950 HIP decoder (libgradtts.so).

Mirrors ``/root/reference/model/diffusion.py``:

* same constructor arguments (``Diffusion`` :228-242, ``GradLogPEstimator2d`` :128-172);
* same sub-module attribute names, so ``state_dict()`` keys are identical and reference checkpoints
  (``train.py:174-175`` -> ``inference.py:66``) load with ``load_state_dict`` unchanged;
* same call signatures and semantics: ``Diffusion.forward/reverse_diffusion(z, mask, mu, n_timesteps,
  stoc=False, spk=None)`` (:254-272, deterministic Euler, ``stoc`` ignored as in the reference) and
  ``GradLogPEstimator2d.forward(x, mask, mu, t, spk=None)`` (:174-216).

The sub-modules are parameter containers only: the whole U-Net (and the whole N-step sampler) runs
inside the HIP library; there is no PyTorch compute path. Compute dtype is an extension:
``compute_dtype=torch.float32`` (parity path, default), ``torch.bfloat16`` (throughput path; fp32
accumulation, fp32 sampler state), ``"bf16_w8"`` (bf16 activations, fp8 e4m3 weights for the 3x3 /
Downsample / Upsample convs with per-output-channel scales: BASELINE.json config 5) or ``"fp8"`` (as
``"bf16_w8"``, and the 3x3 convs over activations on the block-scaled fp8 MFMA: e4m3 operands with one
power-of-two scale per position and 32 channels, include/gradtts.h GT_FP8).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import GT_BF16, GT_BF16_W8, GT_F32, GT_FP8, check, lib, ops


class _ParamOnly(torch.nn.Module):
    def forward(self, *args, **kwargs):  # pragma: no cover - guard
        raise RuntimeError(f"{type(self).__name__} is a parameter container; the U-Net runs as one HIP graph "
                           "(call GradLogPEstimator2d / Diffusion instead)")


class Mish(_ParamOnly):
    pass


class SinusoidalPosEmb(_ParamOnly):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class Upsample(_ParamOnly):
    def __init__(self, dim):
        super().__init__()
        self.conv = torch.nn.ConvTranspose2d(dim, dim, 4, 2, 1)


class Downsample(_ParamOnly):
    def __init__(self, dim):
        super().__init__()
        self.conv = torch.nn.Conv2d(dim, dim, 3, 2, 1)


class Rezero(_ParamOnly):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn
        self.g = torch.nn.Parameter(torch.zeros(1))


class Residual(_ParamOnly):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn


class Block(_ParamOnly):
    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.block = torch.nn.Sequential(torch.nn.Conv2d(dim, dim_out, 3, padding=1),
                                         torch.nn.GroupNorm(groups, dim_out), Mish())


class ResnetBlock(_ParamOnly):
    def __init__(self, dim, dim_out, time_emb_dim, groups=8):
        super().__init__()
        self.mlp = torch.nn.Sequential(Mish(), torch.nn.Linear(time_emb_dim, dim_out))
        self.block1 = Block(dim, dim_out, groups=groups)
        self.block2 = Block(dim_out, dim_out, groups=groups)
        self.res_conv = torch.nn.Conv2d(dim, dim_out, 1) if dim != dim_out else torch.nn.Identity()


class LinearAttention(_ParamOnly):
    def __init__(self, dim, heads=4, dim_head=32):
        super().__init__()
        self.heads = heads
        hidden_dim = dim_head * heads
        self.to_qkv = torch.nn.Conv2d(dim, hidden_dim * 3, 1, bias=False)
        self.to_out = torch.nn.Conv2d(hidden_dim, dim, 1)


def _dtype_code(dt):
    if dt in (torch.float32, "fp32", "float32", GT_F32):
        return GT_F32
    if dt in (torch.bfloat16, "bf16", "bfloat16", GT_BF16):
        return GT_BF16
    if dt in ("bf16_w8", GT_BF16_W8):
        return GT_BF16_W8
    if dt in ("fp8", GT_FP8):
        return GT_FP8
    raise ValueError(f"compute_dtype must be float32, bfloat16, 'bf16_w8' or 'fp8', got {dt}")


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_cuda(*tensors):
    if not torch.cuda.is_available():
        raise RuntimeError("gradtts_amd needs a HIP (MI355X) device; there is no CPU path")
    dev = None
    for t in tensors:
        if t is not None and t.is_cuda:
            dev = t.device
            break
    return dev if dev is not None else torch.device("cuda", torch.cuda.current_device())


def _f32c(t, device):
    return None if t is None else t.to(device=device, dtype=torch.float32).contiguous()


def _check_binary_mask(mask):
    """Masks are 0/1 (``sequence_mask``, model/utils.py:6-10). The library computes the reference's double masking
    (``(Mish(GN(h)) * m + tb) * m``, model/diffusion.py:56-58, 74-77) as one multiply, exact only for 0/1 masks, so a
    fractional mask is rejected rather than decoded wrongly. Same rule as the torch ops (csrc/torch_ops.cpp
    check_binary_mask); skipped inside a graph capture, where the host cannot read the flag."""
    if mask.is_cuda and torch.cuda.is_current_stream_capturing():
        return
    if bool(((mask != 0) & (mask != 1)).any()):
        raise RuntimeError("gradtts: mask values must be 0 or 1 (sequence_mask); fractional masks are not supported "
                           "by the fused decoder (the reference's double masking x*m*m is computed as x*m)")


class GradLogPEstimator2d(torch.nn.Module):
    """Score network s_theta (model/diffusion.py:128-216) -- parameters here, compute in libgradtts.so."""

    def __init__(self, dim, dim_mults=(1, 2, 4), groups=8, n_spks=None, spk_emb_dim=64, n_feats=80, pe_scale=1000,
                 compute_dtype=torch.float32):
        super().__init__()
        if tuple(dim_mults) != (1, 2, 4) or groups != 8:
            raise ValueError("the HIP U-Net implements dim_mults=(1,2,4), groups=8 (the reference configuration)")
        self.dim = dim
        self.dim_mults = dim_mults
        self.groups = groups
        self.n_spks = n_spks if n_spks is not None else 1
        self.spk_emb_dim = spk_emb_dim
        self.n_feats = n_feats
        self.pe_scale = pe_scale
        self.compute_dtype = compute_dtype
        n_spks = self.n_spks
        if n_spks > 1 or n_spks == -1:
            self.spk_mlp = torch.nn.Sequential(torch.nn.Linear(spk_emb_dim, spk_emb_dim * 4), Mish(),
                                               torch.nn.Linear(spk_emb_dim * 4, n_feats))
        self.time_pos_emb = SinusoidalPosEmb(dim)
        self.mlp = torch.nn.Sequential(torch.nn.Linear(dim, dim * 4), Mish(), torch.nn.Linear(dim * 4, dim))
        dims = [2 + (1 if n_spks > 1 else 0), *map(lambda m: dim * m, dim_mults)]
        in_out = list(zip(dims[:-1], dims[1:]))
        self.downs = torch.nn.ModuleList([])
        self.ups = torch.nn.ModuleList([])
        for ind, (dim_in, dim_out) in enumerate(in_out):
            is_last = ind >= len(in_out) - 1
            self.downs.append(torch.nn.ModuleList([
                ResnetBlock(dim_in, dim_out, time_emb_dim=dim), ResnetBlock(dim_out, dim_out, time_emb_dim=dim),
                Residual(Rezero(LinearAttention(dim_out))),
                Downsample(dim_out) if not is_last else torch.nn.Identity()]))
        mid_dim = dims[-1]
        self.mid_block1 = ResnetBlock(mid_dim, mid_dim, time_emb_dim=dim)
        self.mid_attn = Residual(Rezero(LinearAttention(mid_dim)))
        self.mid_block2 = ResnetBlock(mid_dim, mid_dim, time_emb_dim=dim)
        for dim_in, dim_out in reversed(in_out[1:]):
            self.ups.append(torch.nn.ModuleList([
                ResnetBlock(dim_out * 2, dim_in, time_emb_dim=dim), ResnetBlock(dim_in, dim_in, time_emb_dim=dim),
                Residual(Rezero(LinearAttention(dim_in))), Upsample(dim_in)]))
        self.final_block = Block(dim, dim)
        self.final_conv = torch.nn.Conv2d(dim, 1, 1)
        self._handle = None
        self._synced = None

    # ------------------------------------------------------------------ native handle
    def _native(self, beta_min=0.05, beta_max=20.0):
        if self._handle is None:
            h = ctypes.c_void_p()
            check(lib().gt_decoder_create(self.n_feats, self.dim, self.n_spks, self.spk_emb_dim, float(beta_min),
                                          float(beta_max), float(self.pe_scale), ctypes.byref(h)), "gt_decoder_create")
            self._handle = h
            self._beta = (beta_min, beta_max)
        elif self._beta != (beta_min, beta_max):   # Diffusion vs SPEECHSDE schedules: a scalar change, weights stay packed
            check(lib().gt_decoder_set_betas(self._handle, float(beta_min), float(beta_max)), "gt_decoder_set_betas")
            self._beta = (beta_min, beta_max)
        sig = tuple((p.data_ptr(), p._version) for p in self.parameters())
        if sig != self._synced:
            L = lib()
            params = dict(self.named_parameters())
            names = [L.gt_decoder_param_name(self._handle, i).decode() for i in range(L.gt_decoder_num_params(self._handle))]
            if self._synced is not None and all(params[n].is_cuda for n in names):
                # after an optimizer step: one device-side copy into the library's fp32 block, no host round trip
                # (the inference images re-pack lazily from it)
                flat = torch.cat([params[n].detach().reshape(-1).to(torch.float32) for n in names])
                check(L.gt_decoder_set_params_device(self._handle, flat.data_ptr(), flat.numel(),
                                                     _stream_ptr(flat.device)), "gt_decoder_set_params_device")
            else:
                for name in names:
                    arr = np.ascontiguousarray(params[name].detach().to("cpu", torch.float32).numpy())
                    check(L.gt_decoder_set_param(self._handle, name.encode(), arr.ctypes.data, arr.size),
                          f"gt_decoder_set_param({name})")
            self._synced = sig
        return self._handle

    def _free_native(self):
        if self._handle is not None and _lib._lib is not None:
            _lib._lib.gt_decoder_destroy(self._handle)
        self._handle = None
        self._synced = None

    def __del__(self):
        try:
            self._free_native()
        except Exception:
            pass

    def _workspace(self, device, dcode, B, T, N):
        # Scratch comes from PyTorch's caching allocator on the CURRENT stream for every call: the allocator is
        # stream-ordered, so concurrent calls on different streams get disjoint scratch
        # (tests/test_decoder_gpu.py::test_concurrent_streams_match_one_stream) and nothing is kept alive between
        # calls; after the first call of a shape this is a free-list lookup.
        nbytes = lib().gt_decoder_workspace_bytes(self._handle, dcode, B, T, N)
        return torch.empty(nbytes, dtype=torch.uint8, device=device)

    def _check_shapes(self, x, mask, mu):
        if x.dim() != 3 or x.shape[1] != self.n_feats or mu.shape != x.shape or mask.shape != (x.shape[0], 1, x.shape[2]):
            raise ValueError(f"expected x, mu [B,{self.n_feats},T] and mask [B,1,T]; got {tuple(x.shape)}, "
                             f"{tuple(mu.shape)}, {tuple(mask.shape)}")
        if x.shape[2] % 4 != 0:
            raise ValueError("T must be a multiple of 4 (use fix_len_compatibility, model/utils.py:13-17)")

    def _spk(self, spk, B, device):
        if spk is None:
            if self.n_spks > 1:
                raise ValueError("n_spks > 1 needs spk [B, spk_emb_dim]")
            return None
        if not (self.n_spks > 1 or self.n_spks == -1):
            raise AttributeError("'GradLogPEstimator2d' object has no attribute 'spk_mlp' (n_spks == 1 takes no spk)")
        spk = _f32c(spk, device)
        if spk.shape != (B, self.spk_emb_dim):
            raise ValueError(f"spk must be [B,{self.spk_emb_dim}]")
        return spk

    def forward(self, x, mask, mu, t, spk=None):
        """s_theta(x_t, t) -> [B, n_feats, T]  (model/diffusion.py:174-216).

        Differentiable in ``x``: with gradients enabled and ``x.requires_grad`` the result carries a backward that
        runs the U-Net VJP on the device (gt_estimator_vjp, fp32), so the reference's autograd consumers -- the
        Hutchinson divergence ``get_div_fn(fn)`` (n_best/likelihood/likelihood.py:27-38) -- work unchanged.
        Parameter gradients come from Diffusion.loss_t (the training step); mu / spk / t are constants here."""
        if torch.is_grad_enabled() and isinstance(x, torch.Tensor) and x.requires_grad:
            return _EstimatorX.apply(x, self, mask, mu, t, spk)
        with torch.no_grad():
            return self._forward(x, mask, mu, t, spk)

    def _forward(self, x, mask, mu, t, spk=None):
        device = _require_cuda(x, mu, mask)
        self._check_shapes(x, mask, mu)
        B = x.shape[0]
        t = torch.as_tensor(t, device=device, dtype=torch.float32).reshape(-1)
        spk32 = self._spk(spk, B, device)
        dcode = _dtype_code(self.compute_dtype)
        with torch.cuda.device(device):
            h = self._native(*getattr(self, "_beta_override", (0.05, 20.0)))
            # torch.ops.gradtts.estimator (csrc/torch_ops.cpp) -> gt_estimator_forward on the current stream
            return ops().estimator(h.value, dcode, x.to(device), mask.to(device), mu.to(device), t, spk32)


class _EstimatorX(torch.autograd.Function):
    """s_theta(x) with d/dx by the device VJP: backward(v) = (ds/dx)^T v from gt_estimator_vjp (fp32 tape + U-Net
    backward without parameter gradients)."""

    @staticmethod
    def forward(ctx, x, est, mask, mu, t, spk):
        ctx.est = est
        ctx.args = (mask, mu, t, spk)
        ctx.save_for_backward(x)
        return est._forward(x.detach(), mask, mu, t, spk)

    @staticmethod
    def backward(ctx, v):
        (x,) = ctx.saved_tensors
        est = ctx.est
        mask, mu, t, spk = ctx.args
        device = x.device
        B, _, T = x.shape
        x32, m32, mu32, v32 = (_f32c(a, device) for a in (x, mask, mu, v))
        t32 = _f32c(torch.as_tensor(t, device=device).reshape(-1).expand(B), device)
        spk32 = est._spk(spk, B, device)
        score = torch.empty_like(x32)
        gx = torch.empty_like(x32)
        with torch.cuda.device(device):
            h = est._native(*getattr(est, "_beta_override", (0.05, 20.0)))
            ws = torch.empty(lib().gt_estimator_vjp_workspace_bytes(h, B, T), dtype=torch.uint8, device=device)
            check(lib().gt_estimator_vjp(h, x32.data_ptr(), m32.data_ptr(), mu32.data_ptr(), t32.data_ptr(),
                                         spk32.data_ptr() if spk32 is not None else None, v32.data_ptr(), B, T,
                                         score.data_ptr(), gx.data_ptr(), ws.data_ptr(), ws.numel(),
                                         _stream_ptr(device)), "gt_estimator_vjp")
        return gx.to(x.dtype), None, None, None, None, None


def get_noise(t, beta_init, beta_term, cumulative=False):
    """``get_noise`` (model/diffusion.py:219-224)."""
    if cumulative:
        return beta_init * t + 0.5 * (beta_term - beta_init) * (t ** 2)
    return beta_init + (beta_term - beta_init) * t


class Diffusion(torch.nn.Module):
    """Score-based decoder (model/diffusion.py:227-287); reverse_diffusion runs fully on the HIP path."""

    def __init__(self, n_feats, dim, n_spks=1, spk_emb_dim=64, beta_min=0.05, beta_max=20, pe_scale=1000,
                 compute_dtype=torch.float32):
        super().__init__()
        self.n_feats = n_feats
        self.dim = dim
        self.n_spks = n_spks
        self.spk_emb_dim = spk_emb_dim
        self.beta_min = beta_min
        self.beta_max = beta_max
        self.pe_scale = pe_scale
        self.estimator = GradLogPEstimator2d(dim, n_spks=n_spks, spk_emb_dim=spk_emb_dim, n_feats=n_feats,
                                             pe_scale=pe_scale, compute_dtype=compute_dtype)
        self.estimator._beta_override = (beta_min, beta_max)

    @property
    def compute_dtype(self):
        return self.estimator.compute_dtype

    @compute_dtype.setter
    def compute_dtype(self, dt):
        self.estimator.compute_dtype = dt

    @torch.no_grad()
    def reverse_diffusion(self, z, mask, mu, n_timesteps, stoc=False, spk=None):
        """Deterministic Euler sampler (model/diffusion.py:254-268); ``stoc`` is accepted and ignored there too."""
        est = self.estimator
        device = _require_cuda(z, mu, mask)
        est._check_shapes(z, mask, mu)
        spk32 = est._spk(spk, z.shape[0], device)
        dcode = _dtype_code(est.compute_dtype)
        with torch.cuda.device(device):
            h = est._native(self.beta_min, self.beta_max)
            # torch.ops.gradtts.reverse_diffusion (csrc/torch_ops.cpp) -> gt_reverse_diffusion on the current stream
            return ops().reverse_diffusion(h.value, dcode, z.to(device), mask.to(device), mu.to(device),
                                           int(n_timesteps), spk32)

    @torch.no_grad()
    def forward(self, z, mask, mu, n_timesteps, stoc=False, spk=None):
        return self.reverse_diffusion(z, mask, mu, n_timesteps, stoc, spk)

    # ---- training path: with gradients required, loss_t runs the fp32 training step of the
    # library (taped forward + U-Net backward, gt_diffusion_loss_grad) and the loss carries the parameter / mu / spk
    # gradients into autograd; otherwise the forward value only (gt_diffusion_loss_t, any compute dtype).
    def forward_diffusion(self, x0, mask, mu, t, z=None):
        """``Diffusion.forward_diffusion`` (model/diffusion.py:244-252) -> (xt * mask, z * mask). ``z`` defaults to
        ``torch.randn`` of x0's shape/dtype/device -- the reference's own draw (:249-250), same generator stream."""
        device = _require_cuda(x0, mu, mask)
        if z is None:
            z = torch.randn(x0.shape, dtype=x0.dtype, device=x0.device, requires_grad=False)
        x32, m32, mu32, z32 = (_f32c(a, device) for a in (x0, mask, mu, z))
        t32 = _f32c(torch.as_tensor(t).reshape(-1), device)
        B, _, T = x32.shape
        xt = torch.empty_like(x32)
        zm = torch.empty_like(x32)
        with torch.cuda.device(device):
            h = self.estimator._native(self.beta_min, self.beta_max)
            check(lib().gt_forward_diffusion(h, x32.data_ptr(), m32.data_ptr(), mu32.data_ptr(), t32.data_ptr(),
                                             z32.data_ptr(), B, T, xt.data_ptr(), zm.data_ptr(), _stream_ptr(device)),
                  "gt_forward_diffusion")
        return xt.to(x0.dtype), zm.to(x0.dtype)

    def loss_t(self, x0, mask, mu, t, spk=None, z=None):
        """``Diffusion.loss_t`` (diffusion.py:274-281) -> (loss, xt); ``z`` as in forward_diffusion."""
        est = self.estimator
        device = _require_cuda(x0, mu, mask)
        est._check_shapes(x0, mask, mu)
        if z is None:
            z = torch.randn(x0.shape, dtype=x0.dtype, device=x0.device, requires_grad=False)
        B, _, T = x0.shape
        x32, m32, mu32, z32 = (_f32c(a, device) for a in (x0, mask, mu, z))
        _check_binary_mask(m32)
        t32 = _f32c(torch.as_tensor(t).reshape(-1), device)
        spk32 = est._spk(spk, B, device)
        if torch.is_grad_enabled() and (any(p.requires_grad for p in est.parameters()) or mu.requires_grad or
                                        (spk is not None and spk.requires_grad)):
            return self._loss_t_train(x32, m32, mu32, t32, z32, spk32, mu, spk, x0.dtype)
        dcode = _dtype_code(est.compute_dtype)
        loss = torch.empty((), dtype=torch.float32, device=device)
        xt = torch.empty_like(x32)
        with torch.cuda.device(device):
            h = est._native(self.beta_min, self.beta_max)
            ws = torch.empty(lib().gt_diffusion_loss_workspace_bytes(h, dcode, B, T), dtype=torch.uint8, device=device)
            check(lib().gt_diffusion_loss_t(h, dcode, x32.data_ptr(), m32.data_ptr(), mu32.data_ptr(), t32.data_ptr(),
                                            z32.data_ptr(), spk32.data_ptr() if spk32 is not None else None, B, T,
                                            loss.data_ptr(), xt.data_ptr(), ws.data_ptr(), ws.numel(),
                                            _stream_ptr(device)), "gt_diffusion_loss_t")
        return loss.to(x0.dtype), xt.to(x0.dtype)

    def _loss_t_train(self, x32, m32, mu32, t32, z32, spk32, mu, spk, out_dtype):
        est = self.estimator
        device = x32.device
        B, _, T = x32.shape
        L = lib()
        with torch.cuda.device(device):
            h = est._native(self.beta_min, self.beta_max)
            names = [L.gt_decoder_param_name(h, i).decode() for i in range(L.gt_decoder_num_params(h))]
            flat = torch.empty(L.gt_decoder_grad_numel(h), dtype=torch.float32, device=device)
            dmu = torch.empty_like(x32)
            dspk = torch.empty((B, est.spk_emb_dim), dtype=torch.float32, device=device) if spk32 is not None else None
            loss = torch.empty(2, dtype=torch.float32, device=device)
            xt = torch.empty_like(x32)
            ws = torch.empty(L.gt_train_workspace_bytes(h, B, T), dtype=torch.uint8, device=device)
            check(L.gt_diffusion_loss_grad(h, x32.data_ptr(), m32.data_ptr(), mu32.data_ptr(), t32.data_ptr(),
                                           z32.data_ptr(), spk32.data_ptr() if spk32 is not None else None, B, T,
                                           loss.data_ptr(), xt.data_ptr(), flat.data_ptr(), dmu.data_ptr(),
                                           dspk.data_ptr() if dspk is not None else None, ws.data_ptr(), ws.numel(),
                                           _stream_ptr(device)), "gt_diffusion_loss_grad")
        params = dict(est.named_parameters())
        plist = [params[n] for n in names]
        out = _UNetLoss.apply(loss[0], flat, dmu, dspk, mu, spk, *plist)
        return out.to(out_dtype), xt.to(out_dtype)

    def compute_loss(self, x0, mask, mu, spk=None, offset=1e-5):
        """``Diffusion.compute_loss`` (diffusion.py:283-287): t ~ U(0,1) clamped to [offset, 1 - offset]."""
        t = torch.rand(x0.shape[0], dtype=x0.dtype, device=x0.device, requires_grad=False)
        t = torch.clamp(t, offset, 1.0 - offset)
        return self.loss_t(x0, mask, mu, t, spk)


class _UNetLoss(torch.autograd.Function):
    """The loss of Diffusion.loss_t with the gradients the library computed in the same call (gt_diffusion_loss_grad):
    backward scales them by the incoming gradient and hands them to the estimator parameters, mu and spk."""

    @staticmethod
    def forward(ctx, loss, flat, dmu, dspk, mu, spk, *params):
        ctx.save_for_backward(flat, dmu, dspk if dspk is not None else flat.new_empty(0))
        ctx.meta = ([p.shape for p in params], mu.dtype, spk.dtype if spk is not None else None, dspk is not None)
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        flat, dmu, dspk = ctx.saved_tensors
        shapes, mu_dtype, spk_dtype, has_spk = ctx.meta
        scaled = flat * g   # one kernel; the parameter gradients are views of it
        grads, off = [], 0
        for shp in shapes:
            n = int(np.prod(shp)) if len(shp) else 1
            grads.append(scaled[off:off + n].view(shp))
            off += n
        gmu = (dmu * g).to(mu_dtype)
        gspk = (dspk * g).to(spk_dtype) if has_spk else None
        return (None, None, None, None, gmu, gspk, *grads)
