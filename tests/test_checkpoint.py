"""Checkpoint I/O: reference-layout GradTTS checkpoints load into the drop-in decoder.

tests/golden/gradtts_layout.json holds the key order and shapes of the reference's whole ``GradTTS`` state dict
(made by make_gradtts_layout.py from /root/reference/model/tts.py with params.py's configuration). A checkpoint
with exactly that layout is written the way train.py:174-175 does (``torch.save(model.state_dict(), ...)``),
read back with the safe loader and loaded into ``gradtts_amd.diffusion.Diffusion``.
CPU part: layout and values. GPU part: the loaded decoder packs its weights once, decodes bit-identically to a
decoder given the same weights directly, and re-packs after an in-place weight change.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, gpu_available
from gradtts_amd.checkpoint import decoder_state_dict, load_decoder_checkpoint, pack_count
from gradtts_amd.diffusion import Diffusion
from gradtts_amd.params import synthetic_state_dict

with open(os.path.join(GOLDEN, "gradtts_layout.json")) as _f:
    LAYOUT = json.load(_f)


def reference_layout_checkpoint(n_spks, seed=0):
    """A GradTTS state dict with the reference's exact keys/shapes/order: decoder weights synthetic(seed), the
    text encoder and speaker table filled with noise (they are not the decoder's)."""
    dec_sd = synthetic_state_dict(seed=seed, n_spks=n_spks)
    rng = np.random.default_rng(seed + 100)
    out = {}
    for k, shape in LAYOUT[str(n_spks)]:
        if k.startswith("decoder.estimator."):
            v = dec_sd[k[len("decoder.estimator."):]]
            assert list(v.shape) == shape, k
            out[k] = torch.from_numpy(v.copy())
        else:
            out[k] = torch.from_numpy(rng.standard_normal(shape).astype(np.float32))
    return out, dec_sd


@pytest.mark.parametrize("n_spks", [1, 247, -1])
def test_decoder_keys_match_reference_gradtts_layout(n_spks):
    ref_dec = [(k[len("decoder."):], s) for k, s in LAYOUT[str(n_spks)] if k.startswith("decoder.")]
    ours = [(k, list(v.shape)) for k, v in Diffusion(80, 64, n_spks, 64, 0.05, 20, 1000).state_dict().items()]
    assert ours == ref_dec


@pytest.mark.parametrize("n_spks", [1, 247])
def test_reference_checkpoint_file_loads(tmp_path, n_spks):
    ckpt, dec_sd = reference_layout_checkpoint(n_spks)
    path = tmp_path / "grad_1.pt"
    torch.save(ckpt, path)                                     # train.py:174-175
    dec = Diffusion(80, 64, n_spks, 64, 0.05, 20, 1000)
    res = load_decoder_checkpoint(dec, str(path))              # torch.load(weights_only=True) inside
    assert not res.missing_keys and not res.unexpected_keys
    for k, v in dec.estimator.state_dict().items():
        assert np.array_equal(v.numpy(), dec_sd[k]), k
    assert pack_count(dec) == 0                                 # nothing packed before a compute call


def test_not_a_gradtts_checkpoint_is_rejected():
    with pytest.raises(KeyError):
        decoder_state_dict({"encoder.emb.weight": torch.zeros(3)})


@pytest.mark.gpu
def test_checkpoint_decoder_packs_once_and_matches():
    if not gpu_available():
        pytest.skip("no HIP device")
    from gradtts_amd.params import synthetic_inputs
    ckpt, dec_sd = reference_layout_checkpoint(247, seed=4)
    dec = Diffusion(80, 64, 247, 64, 0.05, 20, 1000, compute_dtype=torch.bfloat16)
    load_decoder_checkpoint(dec, ckpt)
    dec = dec.cuda()
    direct = Diffusion(80, 64, 247, 64, 0.05, 20, 1000, compute_dtype=torch.bfloat16)
    direct.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in dec_sd.items()})
    direct = direct.cuda()
    mu, z, mask, spk = (torch.from_numpy(a).cuda() for a in synthetic_inputs(8, 3, 128, lengths=[128, 99, 64]))
    y1 = dec(z, mask, mu, 4, False, spk)
    y2 = dec(z, mask, mu, 4, False, spk)
    assert pack_count(dec) == 1, "weights must be packed exactly once for repeated calls"
    assert torch.equal(y1, y2) and torch.equal(y1, direct(z, mask, mu, 4, False, spk))
    with torch.no_grad():                                        # an in-place update (e.g. an optimizer step)
        dec.estimator.final_conv.bias.add_(0.5)
    y3 = dec(z, mask, mu, 4, False, spk)
    assert pack_count(dec) == 2 and not torch.equal(y3, y1)
