"""GPU vs the storage-emulating oracle (oracle/emulate.py): per-stage and end-to-end errors of the bf16 and fp8
estimators on the golden fixtures, and the fp8 / bf16 samplers of tests/test_fp8_gpu.py. usage: python tools/diag_emulate.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden  # noqa: E402
from gpu_util import STAGES, make_decoder, probe, rel_err  # noqa: E402
from oracle import decoder as odec, emulate  # noqa: E402


def stat(a, b):
    """max-norm relative error, rms relative error, fraction of elements not bit-identical"""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    rms = float(np.sqrt(np.mean((a.astype(np.float64) - b) ** 2) / max(np.mean(b.astype(np.float64) ** 2), 1e-30)))
    return f"{rel_err(a, b):.1e}/{rms:.1e}/{np.mean(a != b):.1e}"
from gradtts_amd.params import synthetic_inputs  # noqa: E402

torch.set_num_threads(min(16, torch.get_num_threads()))
for mode, cd in (("bf16", torch.bfloat16), ("fp8", "fp8")):
    for name in ["estimator_s1_T132.npz", "estimator_s1.npz"]:
        g = load_golden(name)
        n_spks = int(g["n_spks"])
        dec, sd = make_decoder(n_spks, int(g["seed_w"]), cd)
        p = odec.fp8_params(sd) if mode == "fp8" else odec.to_torch_params(sd)
        args = [torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")]
        spk = torch.from_numpy(g["spk"]) if n_spks != 1 else None
        taps = {}
        with torch.no_grad(), emulate.product_storage(mode):
            ref = odec.estimator(p, *args, spk, n_spks, taps=taps).numpy()
        cargs = [a.cuda() for a in args]
        y = dec.estimator(*cargs, spk.cuda() if spk is not None else None).cpu().numpy()
        line = f"{mode} {name}: estimator {stat(y, ref)} (vs fp32 golden {rel_err(y, g['out']):.2e}, emu vs golden {rel_err(ref, g['out']):.2e})"
        if name == "estimator_s1_T132.npz":
            errs = []
            for st in STAGES:
                if st not in taps:
                    continue
                r = taps[st].numpy()
                _, pr = probe(dec.estimator, cd, *cargs, spk.cuda() if spk is not None else None, st, r.shape)
                errs.append(f"{st} {stat(pr.cpu().numpy(), r)}")
            line += "\n   " + ", ".join(errs)
        print(line, flush=True)
    dec, sd = make_decoder(1, 0, cd)
    p = odec.fp8_params(sd) if mode == "fp8" else odec.to_torch_params(sd)
    for B, T, lengths in ((2, 128, [128, 97]),):
        mu, z, mask, _ = synthetic_inputs(13, B, T, lengths=lengths)
        args = (torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu))
        with torch.no_grad(), emulate.product_storage(mode):
            ref = odec.reverse_diffusion(p, *args, 10).numpy()
        y = dec(*(a.cuda() for a in args), 10).cpu().numpy()
        print(f"{mode} reverse N=10 B={B} T={T}: {rel_err(y, ref):.2e}", flush=True)
