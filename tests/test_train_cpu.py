"""Training step (gt_diffusion_loss_grad) host-side checks that need no GPU: with GT_TRAIN_DEBUG=2 the library
runs only its extent check -- every forward / backward helper verifies that the index ranges its kernels would
touch lie inside one buffer (arena allocation, caller buffer, parameter block) and that the arena fits the
workspace gt_train_workspace_bytes sized. The same check runs before every live pass on the GPU."""
import ctypes

import numpy as np
import pytest

from gradtts_amd._lib import lib
from gradtts_amd.params import synthetic_state_dict


def _decoder(n_spks):
    L = lib()
    h = ctypes.c_void_p()
    assert L.gt_decoder_create(80, 64, n_spks, 64, 0.05, 20.0, 1000.0, ctypes.byref(h)) == 0
    for k, v in synthetic_state_dict(0, n_spks=n_spks).items():
        a = np.ascontiguousarray(v, np.float32)
        assert L.gt_decoder_set_param(h, k.encode(), a.ctypes.data, a.size) == 0
    return L, h


@pytest.mark.parametrize("n_spks,B,T", [(1, 2, 64), (247, 2, 32), (1, 1, 40), (1, 3, 128), (247, 1, 4)])
def test_training_step_extents(monkeypatch, n_spks, B, T):
    monkeypatch.setenv("GT_TRAIN_DEBUG", "2")
    L, h = _decoder(n_spks)
    try:
        ws = L.gt_train_workspace_bytes(h, B, T)
        assert ws > 0
        n0 = B * 80 * T
        x0, mu, z, xt, dmu = (np.zeros(n0, np.float32) for _ in range(5))
        mask, t = np.ones(B * T, np.float32), np.full(B, 0.5, np.float32)
        spk, dspk = np.zeros(B * 64, np.float32), np.zeros(B * 64, np.float32)
        grads = np.zeros(L.gt_decoder_grad_numel(h), np.float32)
        work, loss = np.zeros(ws, np.uint8), np.zeros(2, np.float32)
        p = lambda a: a.ctypes.data
        sp = p(spk) if n_spks > 1 else None
        rc = L.gt_diffusion_loss_grad(h, p(x0), p(mask), p(mu), p(t), p(z), sp, B, T, p(loss), p(xt), p(grads),
                                      p(dmu), p(dspk) if n_spks > 1 else None, p(work), ws, None)
        msg = L.gt_last_error()
        assert rc == 0, msg.decode() if msg else rc
        # a workspace one byte short is refused before anything runs
        rc = L.gt_diffusion_loss_grad(h, p(x0), p(mask), p(mu), p(t), p(z), sp, B, T, p(loss), p(xt), p(grads),
                                      p(dmu), None, p(work), ws - 1, None)
        assert rc == 5
    finally:
        L.gt_decoder_destroy(h)


def test_grad_numel_matches_state_dict():
    L, h = _decoder(247)
    try:
        n = sum(int(np.prod(v.shape)) for v in synthetic_state_dict(0, n_spks=247).values())
        assert L.gt_decoder_grad_numel(h) == n
    finally:
        L.gt_decoder_destroy(h)


@pytest.mark.parametrize("n_spks,B,T", [(1, 2, 32), (247, 3, 24)])
def test_vjp_and_likelihood_extents(monkeypatch, n_spks, B, T):
    monkeypatch.setenv("GT_TRAIN_DEBUG", "2")
    L, h = _decoder(n_spks)
    try:
        n0 = B * 80 * T
        x, mu, v, out1, out2 = (np.zeros(n0, np.float32) for _ in range(5))
        mask, t = np.ones(B * T, np.float32), np.full(B, 0.5, np.float32)
        spk, div = np.zeros(B * 64, np.float32), np.zeros(B, np.float32)
        p = lambda a: a.ctypes.data
        sp = p(spk) if n_spks > 1 else None
        ws = L.gt_estimator_vjp_workspace_bytes(h, B, T)
        work = np.zeros(ws, np.uint8)
        rc = L.gt_estimator_vjp(h, p(x), p(mask), p(mu), p(t), sp, p(v), B, T, p(out1), p(out2), p(work), ws, None)
        msg = L.gt_last_error()
        assert rc == 0, msg.decode() if msg else rc
        ws = L.gt_likelihood_workspace_bytes(h, B, T)
        work = np.zeros(ws, np.uint8)
        rc = L.gt_likelihood_drift_div(h, p(x), p(mask), p(mu), p(t), sp, p(v), B, T, p(out1), p(div), p(work), ws,
                                       None)
        msg = L.gt_last_error()
        assert rc == 0, msg.decode() if msg else rc
        rc = L.gt_likelihood_euler(h, p(x), p(mask), p(mu), sp, p(v), B, T, 4, p(out1), p(div), p(work), ws, None)
        msg = L.gt_last_error()
        assert rc == 0, msg.decode() if msg else rc
        assert L.gt_likelihood_euler(h, p(x), p(mask), p(mu), sp, p(v), B, T, 4, p(out1), p(div), p(work), ws - 1,
                                     None) == 5
    finally:
        L.gt_decoder_destroy(h)
