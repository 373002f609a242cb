import sys, numpy as np, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'grad-tts_amd'); sys.path.insert(0, '.')
from gradtts_amd.params import synthetic_state_dict, synthetic_text_encoder_state_dict
from gradtts_amd.tts import GradTTS
from gradtts_amd.text_encoder import align_durations
from oracle import decoder as odec, text_encoder as ote
m = GradTTS(149, 1, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000)
esd = synthetic_text_encoder_state_dict(2); dsd = synthetic_state_dict(seed=0, n_spks=1)
m.encoder.load_state_dict({k: torch.from_numpy(v) for k, v in esd.items()}, strict=True)
m.decoder.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in dsd.items()}, strict=True)
m = m.cuda().eval()
rng = np.random.default_rng(4)
tokens = torch.from_numpy(rng.integers(0, 149, (2, 29))); lengths = torch.tensor([29, 21])
mu_x, logw, xm = m.encoder(tokens.cuda(), lengths.cuda())
mu_y, y_mask, attn, yl, ymax, _ = align_durations(mu_x, logw, xm)
print("ours: Ty", mu_y.shape, "ylen", yl.tolist(), "ymax", ymax)
rmu, rlogw, rxm = ote.text_encoder(ote.to_torch_params(esd), tokens, lengths)
w_ceil, y_len, y_max, ry_mask, r_attn, rmu_y = ote.front_end(rmu, rlogw, rxm)
print("oracle: Ty", rmu_y.shape, "ylen", y_len.tolist(), "ymax", y_max)
print("y_mask equal", torch.equal(y_mask.cpu(), ry_mask))
torch.manual_seed(0)
z = mu_y + torch.randn_like(mu_y)
d1 = m.decoder(z, y_mask, mu_y, 5)
r = odec.reverse_diffusion(odec.to_torch_params(dsd), z.cpu(), y_mask.cpu(), mu_y.cpu(), 5)
print("decoder same inputs rel", float((d1.cpu() - r).abs().max() / r.abs().max()))
torch.manual_seed(5); a = torch.randn(3, device='cuda'); torch.manual_seed(5); b = torch.randn(3, device='cuda'); print("rng", torch.equal(a, b))
