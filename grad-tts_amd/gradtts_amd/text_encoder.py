"""Drop-in ``TextEncoder`` (model/text_encoder.py:285-335): the reference's module tree and parameter names (so
``encoder.*`` keys of a GradTTS checkpoint load unchanged), compute in libgradtts.so (``gt_text_encoder_forward``:
fp32 MFMA convs, LayerNorms, relative-position attention on the MI355X). No PyTorch compute path."""
import ctypes
import math

import numpy as np
import torch

from ._lib import check, lib


class LayerNorm(torch.nn.Module):
    """text_encoder.py:11-29 (parameters only)."""

    def __init__(self, channels, eps=1e-4):
        super().__init__()
        self.channels = channels
        self.eps = eps
        self.gamma = torch.nn.Parameter(torch.ones(channels))
        self.beta = torch.nn.Parameter(torch.zeros(channels))


class ConvReluNorm(torch.nn.Module):
    """text_encoder.py:32-64 (parameters only)."""

    def __init__(self, in_channels, hidden_channels, out_channels, kernel_size, n_layers, p_dropout):
        super().__init__()
        self.n_layers = n_layers
        self.conv_layers = torch.nn.ModuleList()
        self.norm_layers = torch.nn.ModuleList()
        self.conv_layers.append(torch.nn.Conv1d(in_channels, hidden_channels, kernel_size, padding=kernel_size // 2))
        self.norm_layers.append(LayerNorm(hidden_channels))
        for _ in range(n_layers - 1):
            self.conv_layers.append(torch.nn.Conv1d(hidden_channels, hidden_channels, kernel_size,
                                                    padding=kernel_size // 2))
            self.norm_layers.append(LayerNorm(hidden_channels))
        self.proj = torch.nn.Conv1d(hidden_channels, out_channels, 1)
        self.proj.weight.data.zero_()
        self.proj.bias.data.zero_()


class DurationPredictor(torch.nn.Module):
    """text_encoder.py:67-93 (parameters only)."""

    def __init__(self, in_channels, filter_channels, kernel_size, p_dropout):
        super().__init__()
        self.conv_1 = torch.nn.Conv1d(in_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_1 = LayerNorm(filter_channels)
        self.conv_2 = torch.nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_2 = LayerNorm(filter_channels)
        self.proj = torch.nn.Conv1d(filter_channels, 1, 1)


class MultiHeadAttention(torch.nn.Module):
    """text_encoder.py:96-143 (parameters only; relative embeddings shared by the heads)."""

    def __init__(self, channels, out_channels, n_heads, window_size=None, heads_share=True, p_dropout=0.0,
                 proximal_bias=False, proximal_init=False):
        super().__init__()
        if window_size is None or not heads_share or proximal_bias:
            raise ValueError("the HIP encoder implements the reference configuration: shared relative embeddings "
                             "within a window, no proximal bias")
        self.n_heads = n_heads
        self.window_size = window_size
        self.k_channels = channels // n_heads
        self.conv_q = torch.nn.Conv1d(channels, channels, 1)
        self.conv_k = torch.nn.Conv1d(channels, channels, 1)
        self.conv_v = torch.nn.Conv1d(channels, channels, 1)
        rel_stddev = self.k_channels ** -0.5
        self.emb_rel_k = torch.nn.Parameter(torch.randn(1, window_size * 2 + 1, self.k_channels) * rel_stddev)
        self.emb_rel_v = torch.nn.Parameter(torch.randn(1, window_size * 2 + 1, self.k_channels) * rel_stddev)
        self.conv_o = torch.nn.Conv1d(channels, out_channels, 1)


class FFN(torch.nn.Module):
    """text_encoder.py:220-241 (parameters only)."""

    def __init__(self, in_channels, out_channels, filter_channels, kernel_size, p_dropout=0.0):
        super().__init__()
        self.conv_1 = torch.nn.Conv1d(in_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.conv_2 = torch.nn.Conv1d(filter_channels, out_channels, kernel_size, padding=kernel_size // 2)


class Encoder(torch.nn.Module):
    """text_encoder.py:244-282 (parameters only)."""

    def __init__(self, hidden_channels, filter_channels, n_heads, n_layers, kernel_size=1, p_dropout=0.0,
                 window_size=None, **kwargs):
        super().__init__()
        self.attn_layers = torch.nn.ModuleList()
        self.norm_layers_1 = torch.nn.ModuleList()
        self.ffn_layers = torch.nn.ModuleList()
        self.norm_layers_2 = torch.nn.ModuleList()
        for _ in range(n_layers):
            self.attn_layers.append(MultiHeadAttention(hidden_channels, hidden_channels, n_heads,
                                                       window_size=window_size, p_dropout=p_dropout))
            self.norm_layers_1.append(LayerNorm(hidden_channels))
            self.ffn_layers.append(FFN(hidden_channels, hidden_channels, filter_channels, kernel_size,
                                       p_dropout=p_dropout))
            self.norm_layers_2.append(LayerNorm(hidden_channels))


class TextEncoder(torch.nn.Module):
    """``TextEncoder(n_vocab, n_feats, n_channels, filter_channels, filter_channels_dp, n_heads, n_layers,
    kernel_size, p_dropout, window_size=None, spk_emb_dim=64, n_spks=1)``; ``forward(x, x_lengths, spk=None)`` ->
    (mu [B, n_feats, Tx], logw [B, 1, Tx], x_mask [B, 1, Tx]).

    With gradients enabled and parameters that require them, or in train mode with p_dropout > 0, ``forward`` is the
    training pass
    (``gt_text_encoder_forward_train`` + ``gt_text_encoder_backward`` behind an autograd Function): in train mode the
    reference's dropouts apply (``p_dropout`` at the attention probabilities, attention / FFN outputs, FFN hidden
    and duration predictor; 0.5 in the prenet), drawn from the library's counter-based generator with a seed taken
    from torch's CPU generator; in eval mode none do. Otherwise it is the inference pass (eval semantics)."""

    def __init__(self, n_vocab, n_feats, n_channels, filter_channels, filter_channels_dp, n_heads, n_layers,
                 kernel_size, p_dropout, window_size=None, spk_emb_dim=64, n_spks=1):
        super().__init__()
        if n_spks > 1:
            raise ValueError("GradTTS builds its TextEncoder speaker-agnostic (tts.py:49-51); n_spks > 1 is not "
                             "implemented")
        self.n_vocab, self.n_feats, self.n_channels = n_vocab, n_feats, n_channels
        self.filter_channels, self.filter_channels_dp = filter_channels, filter_channels_dp
        self.n_heads, self.n_layers, self.kernel_size, self.window_size = n_heads, n_layers, kernel_size, window_size
        self.p_dropout = p_dropout
        self.emb = torch.nn.Embedding(n_vocab, n_channels)
        torch.nn.init.normal_(self.emb.weight, 0.0, n_channels ** -0.5)
        self.prenet = ConvReluNorm(n_channels, n_channels, n_channels, kernel_size=5, n_layers=3, p_dropout=0.5)
        self.encoder = Encoder(n_channels, filter_channels, n_heads, n_layers, kernel_size, p_dropout,
                               window_size=window_size)
        self.proj_m = torch.nn.Conv1d(n_channels, n_feats, 1)
        self.proj_w = DurationPredictor(n_channels, filter_channels_dp, kernel_size, p_dropout)
        self._handle = None
        self._synced = None

    def _native(self):
        L = lib()
        if self._handle is None:
            h = ctypes.c_void_p()
            check(L.gt_text_encoder_create(self.n_vocab, self.n_feats, self.n_channels, self.filter_channels,
                                           self.filter_channels_dp, self.n_heads, self.n_layers, self.kernel_size,
                                           self.window_size, ctypes.byref(h)), "gt_text_encoder_create")
            self._handle = h
        sig = tuple((p.data_ptr(), p._version) for p in self.parameters())
        if sig != self._synced:
            from .diffusion import _stream_ptr
            params = dict(self.named_parameters())
            names = [L.gt_text_encoder_param_name(self._handle, i).decode()
                     for i in range(L.gt_text_encoder_num_params(self._handle))]
            if self._synced is not None and all(params[n].is_cuda for n in names):
                # after an optimizer step: device-side copy + repack, no host round trip
                flat = torch.cat([params[n].detach().reshape(-1).to(torch.float32) for n in names])
                check(L.gt_text_encoder_set_params_device(self._handle, flat.data_ptr(), flat.numel(),
                                                          _stream_ptr(flat.device)), "gt_text_encoder_set_params_device")
            else:
                for name in names:
                    arr = np.ascontiguousarray(params[name].detach().to("cpu", torch.float32).numpy())
                    check(L.gt_text_encoder_set_param(self._handle, name.encode(), arr.ctypes.data, arr.size),
                          f"gt_text_encoder_set_param({name})")
            self._synced = sig
        return self._handle

    def __del__(self):
        try:
            from . import _lib
            if self._handle is not None and _lib._lib is not None:
                _lib._lib.gt_text_encoder_destroy(self._handle)
        except Exception:
            pass

    def forward(self, x, x_lengths, spk=None):
        from .diffusion import _stream_ptr
        device = self.emb.weight.device
        if device.type != "cuda":
            raise RuntimeError("TextEncoder needs a HIP (MI355X) device; there is no CPU path")
        tokens = x.to(device=device, dtype=torch.int64).contiguous()
        lengths = x_lengths.to(device=device, dtype=torch.int64).contiguous()
        B, Tx = tokens.shape
        # the training pass: with gradients, or in train mode with dropout (torch's Dropout drops under no_grad too)
        if (torch.is_grad_enabled() and any(q.requires_grad for q in self.parameters())) or \
                (self.training and self.p_dropout > 0):
            p, ppre = (float(self.p_dropout), 0.5) if self.training else (0.0, 0.0)
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if (p > 0 or ppre > 0) else 0
            with torch.cuda.device(device):
                h = self._native()
                named = dict(self.named_parameters())
                plist = [named[lib().gt_text_encoder_param_name(h, i).decode()]
                         for i in range(lib().gt_text_encoder_num_params(h))]   # the library's inventory order
                return _TextEncoderTrain.apply(self, h, tokens, lengths, p, ppre, seed, *plist)
        with torch.cuda.device(device):
            h = self._native()
            mu = torch.empty(B, self.n_feats, Tx, dtype=torch.float32, device=device)
            logw = torch.empty(B, 1, Tx, dtype=torch.float32, device=device)
            x_mask = torch.empty(B, 1, Tx, dtype=torch.float32, device=device)
            ws = torch.empty(lib().gt_text_encoder_workspace_bytes(h, B, Tx), dtype=torch.uint8, device=device)
            check(lib().gt_text_encoder_forward(h, tokens.data_ptr(), lengths.data_ptr(), B, Tx, mu.data_ptr(),
                                                logw.data_ptr(), x_mask.data_ptr(), ws.data_ptr(), ws.numel(),
                                                _stream_ptr(device)), "gt_text_encoder_forward")
        return mu, logw, x_mask


class _TextEncoderTrain(torch.autograd.Function):
    """TextEncoder.forward with gradients: the library's training forward keeps a tape in a workspace this Function
    holds until backward, which writes every parameter's gradient into one flat buffer (views of it go to the
    parameters, passed in the library's inventory order)."""

    @staticmethod
    def forward(ctx, enc, h, tokens, lengths, p, ppre, seed, *params):
        from .diffusion import _stream_ptr
        device = tokens.device
        B, Tx = tokens.shape
        L = lib()
        mu = torch.empty(B, enc.n_feats, Tx, dtype=torch.float32, device=device)
        logw = torch.empty(B, 1, Tx, dtype=torch.float32, device=device)
        x_mask = torch.empty(B, 1, Tx, dtype=torch.float32, device=device)
        ws = torch.empty(L.gt_text_encoder_train_workspace_bytes(h, B, Tx), dtype=torch.uint8, device=device)
        check(L.gt_text_encoder_forward_train(h, tokens.data_ptr(), lengths.data_ptr(), B, Tx, p, ppre, seed,
                                              mu.data_ptr(), logw.data_ptr(), x_mask.data_ptr(), ws.data_ptr(),
                                              ws.numel(), _stream_ptr(device)), "gt_text_encoder_forward_train")
        ctx.h, ctx.ws, ctx.shape, ctx.drop = h, ws, (B, Tx), (p, ppre, seed)
        ctx.pshapes = [q.shape for q in params]
        ctx.mark_non_differentiable(x_mask)
        return mu, logw, x_mask

    @staticmethod
    def backward(ctx, dmu, dlogw, _dmask):
        from .diffusion import _stream_ptr
        B, Tx = ctx.shape
        device = ctx.ws.device
        L = lib()
        grads = torch.empty(L.gt_text_encoder_grad_numel(ctx.h), dtype=torch.float32, device=device)
        dmu = dmu.to(torch.float32).contiguous() if dmu is not None else None
        dlogw = dlogw.to(torch.float32).contiguous() if dlogw is not None else None
        with torch.cuda.device(device):
            check(L.gt_text_encoder_backward(ctx.h, dmu.data_ptr() if dmu is not None else None,
                                             dlogw.data_ptr() if dlogw is not None else None, B, Tx, *ctx.drop,
                                             grads.data_ptr(), ctx.ws.data_ptr(), ctx.ws.numel(),
                                             _stream_ptr(device)),
                  "gt_text_encoder_backward")
        out, off = [], 0
        for shp in ctx.pshapes:
            n = int(np.prod(shp)) if len(shp) else 1
            out.append(grads[off:off + n].view(shp))
            off += n
        # the tape stays in ctx.ws until autograd frees ctx: backward only writes the workspace's scratch pieces, so a
        # second backward through the same graph (retain_graph=True) differentiates the same tape again
        return (None, None, None, None, None, None, None, *out)


def fix_len_compatibility(length, num_downsamplings_in_unet=2):
    """utils.py:13-17."""
    while True:
        if length % (2 ** num_downsamplings_in_unet) == 0:
            return length
        length += 1


def align_durations(mu_x, logw, x_mask, length_scale=1.0):
    """tts.py:86-99 on the device: returns (mu_y [B, F, Ty], y_mask [B, 1, Ty], attn [B, 1, Tx, Ty], y_lengths,
    y_max_length). One host read (int(y_lengths.max())), as the reference's."""
    from .diffusion import _stream_ptr
    device = mu_x.device
    B, F, Tx = mu_x.shape
    L = lib()
    with torch.cuda.device(device):
        w_ceil = torch.empty(B, Tx, dtype=torch.float32, device=device)
        cum = torch.empty(B, Tx, dtype=torch.float32, device=device)
        y_lengths = torch.empty(B, dtype=torch.int64, device=device)
        lw, xm = logw.contiguous(), x_mask.contiguous()
        check(L.gt_durations(lw.data_ptr(), xm.data_ptr(), B, Tx, float(length_scale), w_ceil.data_ptr(),
                             cum.data_ptr(), y_lengths.data_ptr(), _stream_ptr(device)), "gt_durations")
        y_max_length = int(y_lengths.max())
        Ty = fix_len_compatibility(y_max_length)
        mu_y = torch.empty(B, F, Ty, dtype=torch.float32, device=device)
        y_mask = torch.empty(B, 1, Ty, dtype=torch.float32, device=device)
        attn = torch.empty(B, 1, Tx, Ty, dtype=torch.float32, device=device)
        mx = mu_x.contiguous()
        check(L.gt_expand(mx.data_ptr(), cum.data_ptr(), xm.data_ptr(), y_lengths.data_ptr(), B, Tx, Ty, F,
                          mu_y.data_ptr(), y_mask.data_ptr(), attn.data_ptr(), _stream_ptr(device)), "gt_expand")
    return mu_y, y_mask, attn, y_lengths, y_max_length, w_ceil
