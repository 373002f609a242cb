"""Host-side extent check of the training step (GT_TRAIN_DEBUG=2: no kernel launches; every helper verifies that
the extents its kernel would touch lie inside one buffer). Usage: GT_TRAIN_DEBUG=2 python tools/train_dry.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "grad-tts_amd"))
from gpu_util import make_decoder  # noqa: E402
from gradtts_amd._lib import lib  # noqa: E402

assert os.environ.get("GT_TRAIN_DEBUG") == "2"
for n_spks, B, T in [(1, 2, 64), (247, 2, 32), (1, 1, 40), (1, 3, 128)]:
    dec, _ = make_decoder(n_spks, 0, torch.float32)
    est = dec.estimator
    h = est._native()
    L = lib()
    dev = "cuda"
    x = torch.zeros(B, 80, T, device=dev)
    mask = torch.ones(B, 1, T, device=dev)
    t = torch.full((B,), 0.5, device=dev)
    spk = torch.zeros(B, 64, device=dev) if n_spks > 1 else None
    flat = torch.empty(L.gt_decoder_grad_numel(h), device=dev)
    ws = torch.empty(L.gt_train_workspace_bytes(h, B, T), dtype=torch.uint8, device=dev)
    loss = torch.empty(2, device=dev)
    xt, dmu = torch.empty_like(x), torch.empty_like(x)
    dspk = torch.empty(B, 64, device=dev) if spk is not None else None
    rc = L.gt_diffusion_loss_grad(h, x.data_ptr(), mask.data_ptr(), x.data_ptr(), t.data_ptr(), x.data_ptr(),
                                  spk.data_ptr() if spk is not None else None, B, T, loss.data_ptr(), xt.data_ptr(),
                                  flat.data_ptr(), dmu.data_ptr(), dspk.data_ptr() if dspk is not None else None,
                                  ws.data_ptr(), ws.numel(), None)
    msg = L.gt_last_error()
    print(f"n_spks={n_spks} B={B} T={T} ws={ws.numel()} rc={rc} {msg.decode() if (rc and msg) else 'extents ok'}",
          flush=True)
