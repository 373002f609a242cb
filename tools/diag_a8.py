"""GPU diagnostic for the GT_FP8 mode (fp8 weights + fp8 operands of the 3x3 convs over activations): errors of one
estimator call and of every U-Net stage against the oracle with the same quantization (oracle.decoder.fp8_params +
fp8_activations), next to the fp8-weight-only mode (bf16_w8) against its own oracle. Prints one line per check.

usage: python tools/diag_a8.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden  # noqa: E402
from gpu_util import STAGES, make_decoder, probe, rel_err  # noqa: E402
from oracle import decoder as odec  # noqa: E402


def cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def p999(y, ref):
    d = np.abs(y.astype(np.float64) - ref) / np.abs(ref).max()
    return float(np.quantile(d, 0.999))


def main():
    for name in ["estimator_s1.npz", "estimator_s247.npz", "estimator_sm1.npz", "estimator_s1_T132.npz",
                 "estimator_s1_T20.npz"]:
        g = load_golden(name)
        n_spks = int(g["n_spks"])
        spk = g["spk"] if n_spks != 1 else None
        args = [torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")]
        spk_t = torch.from_numpy(spk) if spk is not None else None
        for mode in ("bf16_w8", "fp8"):
            dec, sd = make_decoder(n_spks, int(g["seed_w"]), mode)
            p8 = odec.fp8_params(sd)
            with torch.no_grad():
                if mode == "fp8":
                    with odec.fp8_activations():
                        ref = odec.estimator(p8, *args, spk_t, n_spks).numpy()
                else:
                    ref = odec.estimator(p8, *args, spk_t, n_spks).numpy()
                ref32 = odec.estimator(odec.to_torch_params(sd), *args, spk_t, n_spks).numpy()
            y = dec.estimator(*(cuda(a) for a in args), cuda(spk) if spk is not None else None).cpu().numpy()
            print(f"{name} {mode:8s}: vs own oracle max {rel_err(y, ref):.3e} p99.9 {p999(y, ref):.3e} | "
                  f"own oracle vs fp32 {rel_err(ref, ref32):.3e} | gpu vs fp32 {rel_err(y, ref32):.3e}", flush=True)
    g = load_golden("estimator_s1_T132.npz")
    args = [cuda(g[k]) for k in ("x", "mask", "mu", "t")]
    for mode in ("bf16_w8", "fp8"):
        dec, sd = make_decoder(1, 0, mode)
        taps = {}
        with torch.no_grad():
            if mode == "fp8":
                with odec.fp8_activations():
                    odec.estimator(odec.fp8_params(sd), *(torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")),
                                   None, taps=taps)
            else:
                odec.estimator(odec.fp8_params(sd), *(torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")),
                               None, taps=taps)
        errs = []
        for st in STAGES:
            ref = taps[st].numpy()
            _, pr = probe(dec.estimator, mode, *args, None, st, ref.shape)
            errs.append(f"{st}={rel_err(pr.cpu().numpy(), ref):.2e}")
        print(f"stages {mode}: " + " ".join(errs), flush=True)


if __name__ == "__main__":
    main()
