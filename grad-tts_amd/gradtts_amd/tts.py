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

    def compute_loss(self, *args, **kwargs):
        raise NotImplementedError("training the text encoder (GradTTS.compute_loss's encoder gradients) is not "
                                  "implemented on the HIP path; the decoder's training step is "
                                  "(gradtts_amd.diffusion.Diffusion.compute_loss)")
