"""Drop-in ``GradTTS`` (model/tts.py:20-108): same constructor, same ``state_dict`` keys (a reference checkpoint
``grad_*.pt`` loads unchanged), ``forward`` = text -> encoder -> durations / alignment -> decoder entirely on the
MI355X (gradtts_amd.text_encoder + gradtts_amd.diffusion). Training the text encoder (``compute_loss``'s encoder
gradients) is not implemented; the decoder's training step is (``Diffusion.compute_loss``)."""
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

    def compute_loss(self, *args, **kwargs):
        raise NotImplementedError("training the text encoder (GradTTS.compute_loss's encoder gradients) is not "
                                  "implemented on the HIP path; the decoder's training step is "
                                  "(gradtts_amd.diffusion.Diffusion.compute_loss)")


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
