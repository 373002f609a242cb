"""Drop-in HiFi-GAN ``Generator`` (hifi-gan/models.py:77-128, ResBlock1 :13-48, ResBlock2 :53-74): the reference's module tree and
parameter names (``bias`` / ``weight_g`` / ``weight_v`` from torch's weight_norm), so the ``generator`` entry of a
HiFi-GAN checkpoint loads unchanged (inference.py:73-76); compute in libgradtts.so (``gt_vocoder_forward``, fp32 MFMA
convs on the MI355X). ``remove_weight_norm()`` is accepted and does nothing: the library bakes g * v / ||v|| itself."""
import ctypes
import warnings

import numpy as np
import torch

from ._lib import check, lib

LRELU_SLOPE = 0.1


def _wn(m):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.nn.utils.weight_norm(m)


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)


class ResBlock1(torch.nn.Module):
    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.convs1 = torch.nn.ModuleList([_wn(torch.nn.Conv1d(channels, channels, kernel_size, 1, dilation=d,
                                                               padding=get_padding(kernel_size, d))) for d in dilation])
        self.convs2 = torch.nn.ModuleList([_wn(torch.nn.Conv1d(channels, channels, kernel_size, 1, dilation=1,
                                                               padding=get_padding(kernel_size, 1)))
                                           for _ in dilation])


class ResBlock2(torch.nn.Module):
    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3)):
        super().__init__()
        self.convs = torch.nn.ModuleList([_wn(torch.nn.Conv1d(channels, channels, kernel_size, 1, dilation=d,
                                                              padding=get_padding(kernel_size, d))) for d in dilation])


class Generator(torch.nn.Module):
    """``Generator(h, compute_dtype=torch.float32)`` with h the HiFi-GAN config (AttrDict or dict: resblock '1' / '2',
    upsample_rates, upsample_kernel_sizes, upsample_initial_channel, resblock_kernel_sizes,
    resblock_dilation_sizes). compute_dtype=torch.bfloat16 rounds the conv operands to bf16 (fp32 accumulation,
    fp32 activations in memory): the throughput mode; fp32 is the parity path."""

    def __init__(self, h, compute_dtype=torch.float32):
        super().__init__()
        if compute_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("compute_dtype must be torch.float32 (parity path) or torch.bfloat16 (throughput)")
        self.compute_dtype = compute_dtype
        g = (lambda k: h[k]) if isinstance(h, dict) else (lambda k: getattr(h, k))
        self.resblock = str(g("resblock"))
        if self.resblock not in ("1", "2"):
            raise ValueError("resblock must be '1' (ResBlock1) or '2' (ResBlock2), as models.py:84 reads it")
        self.rates = list(g("upsample_rates"))
        self.kernels = list(g("upsample_kernel_sizes"))
        self.c0 = int(g("upsample_initial_channel"))
        self.rb_k = list(g("resblock_kernel_sizes"))
        self.rb_d = [list(d) for d in g("resblock_dilation_sizes")]
        self.num_kernels = len(self.rb_k)
        self.num_upsamples = len(self.rates)
        self.n_mels = 80
        self.conv_pre = _wn(torch.nn.Conv1d(80, self.c0, 7, 1, padding=3))
        self.ups = torch.nn.ModuleList()
        for i, (u, k) in enumerate(zip(self.rates, self.kernels)):
            self.ups.append(_wn(torch.nn.ConvTranspose1d(self.c0 // (2 ** i), self.c0 // (2 ** (i + 1)), k, u,
                                                         padding=(k - u) // 2)))
        self.resblocks = torch.nn.ModuleList()
        for i in range(len(self.ups)):
            ch = self.c0 // (2 ** (i + 1))
            for k, d in zip(self.rb_k, self.rb_d):
                self.resblocks.append((ResBlock1 if self.resblock == "1" else ResBlock2)(h, ch, k, d))
        self.conv_post = _wn(torch.nn.Conv1d(ch, 1, 7, 1, padding=3))
        self._handle = None
        self._synced = None

    def remove_weight_norm(self):
        """Accepted for drop-in use (inference.py:76); the library bakes the weight norm on upload."""

    def _native(self):
        L = lib()
        if self._handle is None:
            h = ctypes.c_void_p()
            ia = lambda xs: (ctypes.c_int * len(xs))(*xs)
            nd = len(self.rb_d[0])
            if any(len(d) != nd for d in self.rb_d):
                raise ValueError("every resblock needs the same number of dilations")
            dil = [d for ds in self.rb_d for d in ds]
            check(L.gt_vocoder_create2(self.n_mels, self.c0, self.num_upsamples, ia(self.rates), ia(self.kernels),
                                       self.num_kernels, ia(self.rb_k), int(self.resblock), nd, ia(dil),
                                       ctypes.byref(h)), "gt_vocoder_create2")
            self._handle = h
        check(L.gt_vocoder_set_compute_dtype(self._handle, 1 if self.compute_dtype == torch.bfloat16 else 0),
              "gt_vocoder_set_compute_dtype")
        sig = tuple((p.data_ptr(), p._version) for p in self.parameters())
        if sig != self._synced:
            params = dict(self.named_parameters())
            for i in range(L.gt_vocoder_num_params(self._handle)):
                name = L.gt_vocoder_param_name(self._handle, i).decode()
                arr = np.ascontiguousarray(params[name].detach().to("cpu", torch.float32).numpy())
                check(L.gt_vocoder_set_param(self._handle, name.encode(), arr.ctypes.data, arr.size),
                      f"gt_vocoder_set_param({name})")
            self._synced = sig
        return self._handle

    def __del__(self):
        try:
            from . import _lib
            if self._handle is not None and _lib._lib is not None:
                _lib._lib.gt_vocoder_destroy(self._handle)
        except Exception:
            pass

    def forward(self, x):
        """mel [B, 80, T] -> audio [B, 1, T * prod(upsample_rates)] in [-1, 1] (models.py:94-110)."""
        from .diffusion import _stream_ptr
        device = self.conv_pre.bias.device
        if device.type != "cuda":
            raise RuntimeError("the HiFi-GAN generator needs a HIP (MI355X) device; there is no CPU path")
        mel = x.to(device=device, dtype=torch.float32).contiguous()
        B, _, T = mel.shape
        with torch.cuda.device(device):
            h = self._native()
            L = lib()
            audio = torch.empty(B, 1, T * L.gt_vocoder_hop(h), dtype=torch.float32, device=device)
            ws = torch.empty(L.gt_vocoder_workspace_bytes(h, B, T), dtype=torch.uint8, device=device)
            check(L.gt_vocoder_forward(h, mel.data_ptr(), B, T, audio.data_ptr(), ws.data_ptr(), ws.numel(),
                                       _stream_ptr(device)), "gt_vocoder_forward")
        return audio


HiFiGAN = Generator   # inference.py:19 imports the generator as HiFiGAN
