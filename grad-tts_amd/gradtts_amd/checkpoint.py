"""Checkpoint I/O for the drop-in decoder.

The reference writes whole-model checkpoints, ``torch.save(model.state_dict(), f"{log_dir}/grad_{epoch}.pt")``
(/root/reference/train.py:174-175), and reads them with ``generator.load_state_dict(torch.load(path))``
(/root/reference/inference.py:66). Inside a ``GradTTS`` the decoder's keys are ``decoder.estimator.<...>``
(``GradTTS.decoder`` = ``Diffusion``, tts.py:52; ``Diffusion.estimator``, diffusion.py:241), next to the text
encoder's ``encoder.*`` and, for n_spks > 1, ``spk_emb.weight``.

Because the drop-in ``Diffusion`` registers the same sub-modules under the same names, a ``GradTTS`` that uses it
loads those checkpoints unchanged. These helpers do the same for a bare decoder: take the ``decoder.`` part of a
GradTTS checkpoint (file or state dict) and load it into a :class:`gradtts_amd.diffusion.Diffusion`. Files are
read with ``torch.load(..., weights_only=True)``: nothing from the file is executed.

The weights are packed into the kernels' device layouts (bf16 / fp8 images, wimage.h) once, on the first compute
call after a change -- ``gt_decoder_pack_count`` counts those packings.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

DECODER_PREFIX = "decoder."


def decoder_state_dict(sd, prefix: str = DECODER_PREFIX) -> "OrderedDict[str, torch.Tensor]":
    """The ``Diffusion`` part of a GradTTS state dict, prefix stripped (keys ``estimator.<...>``)."""
    out = OrderedDict((k[len(prefix):], v) for k, v in sd.items() if k.startswith(prefix))
    if not out:
        raise KeyError(f"no '{prefix}*' keys: not a GradTTS checkpoint (tts.py:52, train.py:174-175)")
    return out


def read_checkpoint(path_or_sd):
    """A state dict from a checkpoint path (safe loader) or an already-loaded mapping."""
    if isinstance(path_or_sd, (str, bytes)) or hasattr(path_or_sd, "__fspath__"):
        return torch.load(path_or_sd, map_location="cpu", weights_only=True)
    return path_or_sd


def load_decoder_checkpoint(diffusion, path_or_sd, strict: bool = True):
    """Load the decoder weights of a reference GradTTS checkpoint into ``diffusion`` (drop-in ``Diffusion``)."""
    return diffusion.load_state_dict(decoder_state_dict(read_checkpoint(path_or_sd)), strict=strict)


def pack_count(diffusion) -> int:
    """How many times the native decoder has packed its weights (0 before the first compute call)."""
    from ._lib import lib
    est = diffusion.estimator
    return 0 if est._handle is None else int(lib().gt_decoder_pack_count(est._handle))
