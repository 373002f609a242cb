#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REAL reference.

Runs only in the build container (where /root/reference exists); the fixtures it writes are data
(inputs + expected outputs) and travel with the repo, the reference does not.

* Decoder fixtures: the reference ``model.diffusion.Diffusion`` (/root/reference/model/diffusion.py)
  with deterministic synthetic weights (``gradtts_amd.params.synthetic_state_dict``; only the seed
  and a SHA-256 of the weights are stored), run in float32 and float64.
* MAS fixtures: the reference ``model.monotonic_align.maximum_path`` (``__init__.py:8-23``) whose
  Cython core is compiled from the reference's own ``core.pyx`` by ``make -C oracle ref``
  (the shipped .so files do not import under numpy 2.x).

Usage:  make -C oracle ref && PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
import sysconfig
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("GRADTTS_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
from gradtts_amd.params import synthetic_state_dict, state_dict_sha256, synthetic_inputs  # noqa: E402

sys.dont_write_bytecode = True


def import_reference():
    """Import the unmodified reference package ``model`` without running its __init__ (which pulls in
    the text encoder), and register the locally compiled MAS core under the import path
    ``model/monotonic_align/__init__.py:5`` expects."""
    pkg = types.ModuleType("model")
    pkg.__path__ = [os.path.join(REF, "model")]
    sys.modules["model"] = pkg
    for n in ("model.monotonic_align.model", "model.monotonic_align.model.monotonic_align"):
        m = types.ModuleType(n)
        m.__path__ = []
        sys.modules[n] = m
    so = os.path.join(REPO, "oracle", "_ref", "core" + sysconfig.get_config_var("EXT_SUFFIX"))
    if not os.path.exists(so):
        raise SystemExit(f"missing {so}: run `make -C oracle ref` first")
    name = "model.monotonic_align.model.monotonic_align.core"
    spec = importlib.util.spec_from_file_location(name, so)
    core = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(core)
    sys.modules[name] = core
    import model.diffusion as diffusion  # noqa: E402
    import model.monotonic_align as monotonic_align  # noqa: E402
    return diffusion, monotonic_align


def build_reference_decoder(diffusion, n_spks, seed, dtype):
    torch.manual_seed(0)
    dec = diffusion.Diffusion(80, 64, n_spks, 64, 0.05, 20, 1000)
    sd = synthetic_state_dict(seed=seed, n_spks=n_spks)
    ref_keys = list(dec.estimator.state_dict().keys())
    assert ref_keys == list(sd.keys()), "param inventory differs from the reference registration order"
    dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    dec = dec.to(dtype).eval()
    return dec, state_dict_sha256(sd)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}  ({os.path.getsize(path)/1024:.1f} KiB)")


def estimator_case(diffusion, name, n_spks, B, T, lengths, tvals, seed_w=0, seed_x=11):
    mu, z, mask, spk = synthetic_inputs(seed_x, B, T, lengths=lengths)
    t = np.asarray(tvals, dtype=np.float32)
    outs = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        dec, sha = build_reference_decoder(diffusion, n_spks, seed_w, dt)
        spk_t = torch.from_numpy(spk).to(dt) if n_spks != 1 else None
        with torch.no_grad():
            y = dec.estimator(torch.from_numpy(z).to(dt), torch.from_numpy(mask).to(dt),
                              torch.from_numpy(mu).to(dt), torch.from_numpy(t).to(dt), spk_t)
        outs[tag] = y.numpy()
    assert np.isfinite(outs["f32"]).all()
    save(name, n_spks=n_spks, seed_w=seed_w, weights_sha256=sha, x=z, mu=mu, mask=mask, t=t,
         spk=spk if n_spks != 1 else np.zeros((0,), np.float32), out=outs["f32"], out_f64=outs["f64"])


def reverse_case(diffusion, name, n_spks, B, T, lengths, N, seed_w=0, seed_x=21, with_f64=True):
    mu, z, mask, spk = synthetic_inputs(seed_x, B, T, lengths=lengths)
    outs = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        if tag == "f64" and not with_f64:
            continue
        dec, sha = build_reference_decoder(diffusion, n_spks, seed_w, dt)
        spk_t = torch.from_numpy(spk).to(dt) if n_spks != 1 else None
        y = dec(torch.from_numpy(z).to(dt), torch.from_numpy(mask).to(dt), torch.from_numpy(mu).to(dt), N,
                False, spk_t)
        outs[tag] = y.numpy()
    assert np.isfinite(outs["f32"]).all()
    save(name, n_spks=n_spks, seed_w=seed_w, weights_sha256=sha, z=z, mu=mu, mask=mask, n_timesteps=N,
         spk=spk if n_spks != 1 else np.zeros((0,), np.float32), out=outs["f32"],
         out_f64=outs.get("f64", np.zeros((0,), np.float64)))
    return mu, z, mask, spk


def mas_case(monotonic_align, name, values, tx, ty):
    B, Txm, Tym = values.shape
    mask = np.zeros((B, Txm, Tym), np.float32)
    for b in range(B):
        mask[b, :tx[b], :ty[b]] = 1.0
    path = monotonic_align.maximum_path(torch.from_numpy(values), torch.from_numpy(mask)).numpy()
    save(name, value=values.astype(np.float32), mask=mask, path=path.astype(np.int8))


def main():
    diffusion, monotonic_align = import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))

    # ---- one estimator call (GradLogPEstimator2d.forward, diffusion.py:174-216) ----
    estimator_case(diffusion, "estimator_s1.npz", 1, 2, 64, [64, 40], [0.95, 0.3])
    estimator_case(diffusion, "estimator_s247.npz", 247, 2, 64, [64, 37], [0.5, 0.05])
    estimator_case(diffusion, "estimator_sm1.npz", -1, 2, 64, [64, 52], [0.75, 0.15])
    estimator_case(diffusion, "estimator_s1_T132.npz", 1, 1, 132, [129], [0.61])   # ragged tiles
    estimator_case(diffusion, "estimator_s1_T20.npz", 1, 2, 20, [20, 9], [0.99, 0.01])  # tiny: level-2 T=5

    # ---- full sampler (Diffusion.reverse_diffusion, diffusion.py:254-268) ----
    for N in (1, 2, 10, 50):
        reverse_case(diffusion, f"reverse_s1_N{N}.npz", 1, 2, 128, [128, 100], N)
    reverse_case(diffusion, "reverse_s247_N10.npz", 247, 2, 128, [128, 77], 10)
    # padding dependence: utterance 1 of reverse_s1_N10 run alone at T=100
    mu, z, mask, _ = synthetic_inputs(21, 2, 128, lengths=[128, 100])
    dec, sha = build_reference_decoder(diffusion, 1, 0, torch.float32)
    alone = dec(torch.from_numpy(z[1:2, :, :100].copy()), torch.from_numpy(mask[1:2, :, :100].copy()),
                torch.from_numpy(mu[1:2, :, :100].copy()), 10).numpy()
    save("reverse_s1_N10_alone_T100.npz", n_spks=1, seed_w=0, weights_sha256=sha, z=z[1:2, :, :100],
         mu=mu[1:2, :, :100], mask=mask[1:2, :, :100], n_timesteps=10, out=alone)

    # ---- monotonic alignment search (model/monotonic_align/__init__.py:8-23) ----
    rng = np.random.default_rng(5)
    tx = [17, 1, 30, 40, 8, 25]
    ty = [45, 33, 30, 97, 8, 60]
    mas_case(monotonic_align, "mas_random.npz", rng.standard_normal((6, 40, 100)).astype(np.float32), tx, ty)
    mas_case(monotonic_align, "mas_ties.npz", rng.integers(-2, 3, (6, 40, 100)).astype(np.float32), tx, ty)
    # realistic log-prior (tts.py:143-149) for ragged text/frame lengths
    B, Txm, Tym = 4, 61, 200
    txs, tys = [61, 40, 23, 55], [200, 150, 88, 199]
    mu_x = rng.standard_normal((B, 80, Txm)).astype(np.float32)
    y = rng.standard_normal((B, 80, Tym)).astype(np.float32)
    const = -0.5 * np.log(2 * np.pi) * 80
    mu_t, y_t = torch.from_numpy(mu_x), torch.from_numpy(y)
    factor = -0.5 * torch.ones(mu_t.shape, dtype=mu_t.dtype)
    y_square = torch.matmul(factor.transpose(1, 2), y_t ** 2)
    y_mu_double = torch.matmul(2.0 * (factor * mu_t).transpose(1, 2), y_t)
    mu_square = torch.sum(factor * (mu_t ** 2), 1).unsqueeze(-1)
    log_prior = (y_square - y_mu_double + mu_square + const).numpy()
    mas_case(monotonic_align, "mas_logprior.npz", log_prior.astype(np.float32), txs, tys)


if __name__ == "__main__":
    main()
