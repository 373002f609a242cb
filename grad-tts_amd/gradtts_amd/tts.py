"""Drop-in ``GradTTS`` (model/tts.py:20-254): same constructor, same ``state_dict`` keys (a reference checkpoint
``grad_*.pt`` loads unchanged), ``forward`` = text -> encoder -> durations / alignment -> decoder entirely on the
MI355X (gradtts_amd.text_encoder + gradtts_amd.diffusion), ``compute_loss`` = the reference's training objective
(encoder training pass, log-prior + MAS, duration loss, ``out_size`` crop, ``mu_y``, diffusion loss, prior loss) with
every gradient computed by the library, ``get_score_model`` for likelihood rescoring."""
import random

import torch

from .diffusion import Diffusion
from .text_encoder import TextEncoder, align_durations


class GradTTS(torch.nn.Module):
    def __init__(self, n_vocab, n_spks, spk_emb_dim, n_enc_channels, filter_channels, filter_channels_dp, n_heads,
                 n_enc_layers, enc_kernel, enc_dropout, window_size, n_feats, dec_dim, beta_min, beta_max, pe_scale,
                 compute_dtype=torch.float32):
        super().__init__()
        self.n_vocab = n_vocab
        self.n_spks = n_spks
        self.spk_emb_dim = spk_emb_dim
        self.n_enc_channels = n_enc_channels
        self.n_feats = n_feats
        if n_spks == -1:
            self.spk_emb = None
        elif n_spks > 1:
            self.spk_emb = torch.nn.Embedding(n_spks, spk_emb_dim)
        self.encoder = TextEncoder(n_vocab, n_feats, n_enc_channels, filter_channels, filter_channels_dp, n_heads,
                                   n_enc_layers, enc_kernel, enc_dropout, window_size)
        self.decoder = Diffusion(n_feats, dec_dim, n_spks, spk_emb_dim, beta_min, beta_max, pe_scale,
                                 compute_dtype=compute_dtype)

    @torch.no_grad()
    def forward(self, x, x_lengths, n_timesteps, temperature=1.0, stoc=False, spk=None, length_scale=1.0):
        """tts.py:55-108: returns (encoder_outputs, decoder_outputs, attn), each cut to y_max_length frames."""
        device = self.encoder.emb.weight.device
        x, x_lengths = x.to(device), x_lengths.to(device)
        if self.n_spks > 1:
            spk = self.spk_emb.weight.index_select(0, spk.to(device))   # Embedding lookup (tts.py:78)
        mu_x, logw, x_mask = self.encoder(x, x_lengths, spk)
        mu_y, y_mask, attn, _, y_max_length, _ = align_durations(mu_x, logw, x_mask, length_scale)
        encoder_outputs = mu_y[:, :, :y_max_length]
        z = mu_y + torch.randn_like(mu_y, device=mu_y.device) / temperature
        decoder_outputs = self.decoder(z, y_mask, mu_y, n_timesteps, stoc, spk)
        decoder_outputs = decoder_outputs[:, :, :y_max_length]
        return encoder_outputs, decoder_outputs, attn[:, :, :y_max_length]

    @torch.no_grad()
    def get_score_model(self, x, x_lengths, y, y_lengths, spk=None):
        """tts.py:196-254: the score model of one text / mel pair for likelihood rescoring -- encoder, log-prior +
        MAS alignment (one device call, gradtts_amd.alignment) and mu_y = attn^T mu_x (gt_path_gather). Returns
        (ScoreModel(estimator, y_mask, mu_y, spk), mu_y, spk, y_mask) as the reference does."""
        from ._lib import check, lib
        from .alignment import mas_alignment
        from .diffusion import _stream_ptr
        device = self.encoder.emb.weight.device
        x, x_lengths, y, y_lengths = (a.to(device) for a in (x, x_lengths, y, y_lengths))
        if self.n_spks > 1:
            spk = self.spk_emb.weight.index_select(0, spk.to(device))
        mu_x, logw, x_mask = self.encoder(x, x_lengths, spk)
        Ty = y.shape[-1]
        y_mask = (torch.arange(Ty, device=device)[None] < y_lengths[:, None]).unsqueeze(1).to(x_mask.dtype)
        attn = mas_alignment(mu_x, y, x_mask, y_mask)
        B, F, Tx = mu_x.shape
        mu_y = torch.empty(B, F, Ty, dtype=torch.float32, device=device)
        with torch.cuda.device(device):
            check(lib().gt_path_gather(attn.contiguous().data_ptr(), mu_x.data_ptr(), B, Tx, Ty, F, mu_y.data_ptr(),
                                       _stream_ptr(device)), "gt_path_gather")
        return ScoreModel(self.decoder.estimator, y_mask, mu_y, spk), mu_y, spk, y_mask

    def compute_loss(self, x, x_lengths, y, y_lengths, spk=None, out_size=None):
        """tts.py:110-194 -> (dur_loss, prior_loss, diff_loss). The encoder runs its training pass (dropout in train
        mode, gt_text_encoder_forward_train / _backward), the alignment is one device call (log-prior + MAS,
        gradtts_amd.alignment), ``mu_y = attn^T mu_x`` and the two auxiliary losses are library kernels with their
        backward (gt_path_gather / gt_path_scatter, gt_tts_aux_losses), the diffusion loss is the decoder's
        training step (gt_diffusion_loss_grad). The crop draws its offsets with ``random.choice`` and the decoder
        draws t and z with torch.rand / torch.randn, in the reference's order, so a seeded run sees the reference's
        draws. Host reads: y_lengths for the crop, as the reference's ``.cpu()`` (:160)."""
        from .alignment import mas_alignment
        device = self.encoder.emb.weight.device
        x, x_lengths, y, y_lengths = (a.to(device) for a in (x, x_lengths, y, y_lengths))
        if self.n_spks > 1:
            spk = self.spk_emb(spk.to(device))
        mu_x, logw, x_mask = self.encoder(x, x_lengths, spk)
        y_max_length = y.shape[-1]
        y_mask = _sequence_mask(y_lengths, y_max_length).unsqueeze(1).to(x_mask)
        attn = mas_alignment(mu_x.detach(), y, x_mask, y_mask)            # [B, Tx, Ty], no gradient (:143-152)
        attn_full = attn
        if out_size is not None:                                          # :159-181
            max_offset = (y_lengths - out_size).clamp(0)
            offset_ranges = list(zip([0] * max_offset.shape[0], max_offset.cpu().numpy()))
            out_offset = [random.choice(range(start, int(end))) if end > start else 0 for start, end in offset_ranges]
            B = attn.shape[0]
            attn_cut = torch.zeros(B, attn.shape[1], out_size, dtype=attn.dtype, device=attn.device)
            y_cut = torch.zeros(B, self.n_feats, out_size, dtype=y.dtype, device=y.device)
            y_cut_lengths = []
            yl_host = y_lengths.cpu().tolist()
            for i in range(B):
                ycl = out_size + min(int(yl_host[i]) - out_size, 0)
                y_cut_lengths.append(ycl)
                lo, hi = out_offset[i], out_offset[i] + ycl
                y_cut[i, :, :ycl] = y[i, :, lo:hi]
                attn_cut[i, :, :ycl] = attn[i, :, lo:hi]
            y_mask = _sequence_mask(torch.LongTensor(y_cut_lengths)).unsqueeze(1).to(y_mask)
            attn, y = attn_cut, y_cut
        mu_y = _PathGather.apply(attn, mu_x)                              # :184-185
        diff_loss, xt = self.decoder.compute_loss(y, y_mask, mu_y, spk)   # :188
        dur_loss, prior_loss = _AuxLosses.apply(logw, mu_y, attn_full, x_mask, x_lengths, y, y_mask)   # :155-156, :191
        return dur_loss, prior_loss, diff_loss


class ScoreModel(torch.nn.Module):
    """The score model of get_score_model (tts.py:239-252): forward(x, t) = estimator(x, y_mask, mu_y, t, spk)."""

    def __init__(self, estimator, y_mask, mu_y, spk):
        super().__init__()
        self.y_mask = y_mask
        self.mu_y = mu_y
        self.spk = spk
        self.estimator = estimator

    def forward(self, x, t):
        return self.estimator(x=x, mask=self.y_mask, mu=self.mu_y, t=t, spk=self.spk)


def _sequence_mask(length, max_length=None):
    """utils.py:6-10."""
    if max_length is None:
        max_length = length.max()
    x = torch.arange(int(max_length), dtype=length.dtype, device=length.device)
    return x.unsqueeze(0) < length.unsqueeze(1)


class _PathGather(torch.autograd.Function):
    """mu_y = attn^T mu_x for a 0/1 path attn [B, Tx, Ty] (tts.py:184-185): gt_path_gather forward, gt_path_scatter
    (dmu_x = attn dmu_y) backward."""

    @staticmethod
    def forward(ctx, attn, mu_x):
        from ._lib import check, lib
        from .diffusion import _stream_ptr
        attn = attn.to(torch.float32).contiguous()
        mu = mu_x.to(torch.float32).contiguous()
        B, F, Tx = mu.shape
        Ty = attn.shape[-1]
        mu_y = torch.empty(B, F, Ty, dtype=torch.float32, device=mu.device)
        with torch.cuda.device(mu.device):
            check(lib().gt_path_gather(attn.data_ptr(), mu.data_ptr(), B, Tx, Ty, F, mu_y.data_ptr(),
                                       _stream_ptr(mu.device)), "gt_path_gather")
        ctx.save_for_backward(attn)
        ctx.dims = (B, F, Tx, Ty, mu_x.dtype)
        return mu_y.to(mu_x.dtype)

    @staticmethod
    def backward(ctx, g):
        from ._lib import check, lib
        from .diffusion import _stream_ptr
        (attn,) = ctx.saved_tensors
        B, F, Tx, Ty, dt = ctx.dims
        g = g.to(torch.float32).contiguous()
        dmu = torch.empty(B, F, Tx, dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            check(lib().gt_path_scatter(attn.data_ptr(), g.data_ptr(), B, Tx, Ty, F, dmu.data_ptr(),
                                        _stream_ptr(g.device)), "gt_path_scatter")
        return None, dmu.to(dt)


class _AuxLosses(torch.autograd.Function):
    """(dur_loss, prior_loss) of tts.py:155-156 / :191-192 in one library call (gt_tts_aux_losses), which also
    returns their gradients w.r.t. logw and mu_y for a unit upstream; backward scales them."""

    @staticmethod
    def forward(ctx, logw, mu_y, attn, x_mask, x_lengths, y, y_mask):
        from ._lib import check, lib
        from .diffusion import _stream_ptr
        dev = logw.device
        f = lambda a: a.to(device=dev, dtype=torch.float32).contiguous()
        lw, mu, at, xm, yy, ym = (f(a) for a in (logw, mu_y, attn, x_mask, y, y_mask))
        xl = x_lengths.to(device=dev, dtype=torch.int64).contiguous()
        B, Tx = lw.shape[0], lw.shape[-1]
        F, Ty = mu.shape[1], mu.shape[2]
        losses = torch.empty(4, dtype=torch.float32, device=dev)
        dlw, dmu = torch.empty_like(lw), torch.empty_like(mu)
        with torch.cuda.device(dev):
            ws = torch.empty(lib().gt_tts_aux_losses_workspace_bytes(B, Tx), dtype=torch.uint8, device=dev)
            check(lib().gt_tts_aux_losses(lw.data_ptr(), at.data_ptr(), xm.data_ptr(), xl.data_ptr(), B, Tx,
                                          at.shape[-1], yy.data_ptr(), mu.data_ptr(), ym.data_ptr(), Ty, F,
                                          losses.data_ptr(), dlw.data_ptr(), dmu.data_ptr(), ws.data_ptr(), ws.numel(),
                                          _stream_ptr(dev)), "gt_tts_aux_losses")
        ctx.save_for_backward(dlw, dmu)
        ctx.dtypes = (logw.dtype, mu_y.dtype)
        return losses[0].clone().to(logw.dtype), losses[1].clone().to(mu_y.dtype)

    @staticmethod
    def backward(ctx, gd, gp):
        dlw, dmu = ctx.saved_tensors
        tl, tm = ctx.dtypes
        return ((dlw * gd).to(tl) if gd is not None else None, (dmu * gp).to(tm) if gp is not None else None,
                None, None, None, None, None)
