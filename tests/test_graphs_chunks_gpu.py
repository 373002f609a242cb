"""HIP-graph replay of the sampler and internal batch chunking (include/gradtts.h).

* Graph segments (opt-in, gt_decoder_set_graphs; gt_reverse_diffusion captures up to 100 Euler steps per graph; beyond that 50-step segments
  plus a remainder, a device-side step index selecting each step's time-bias row and beta(t)) must give results
  bit-identical to the eager launch sequence, and a repeated call with the same buffers must replay, not
  re-capture.
* Batches larger than one 32-bit-addressable chunk run chunk by chunk; because every statistic is per
  utterance, chunked results are bit-identical to unchunked ones (GT_MAX_CHUNK forces small chunks) and a real
  two-chunk fp32 batch at T = 1024 matches the same utterances decoded as small batches.
"""
import ctypes
import os
import time

import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder
from gradtts_amd import _lib
from gradtts_amd.diffusion import _dtype_code, _stream_ptr
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _inputs(seed, B, T, lengths=None):
    mu, z, mask, spk = synthetic_inputs(seed, B, T, lengths=lengths)
    return [torch.from_numpy(a).cuda() for a in (mu, z, mask, spk)]


@pytest.mark.parametrize("cdt,N", [(torch.bfloat16, 10), (torch.bfloat16, 120), (torch.float32, 57),
                                   ("bf16_w8", 130)])
def test_graph_replay_bit_exact_vs_eager(cdt, N):
    dec, _ = make_decoder(1, 0, cdt)
    mu, z, mask, _ = _inputs(7, 3, 128, lengths=[128, 100, 64])
    L = _lib.lib()
    h = dec.estimator._native()
    _lib.check(L.gt_decoder_set_graphs(h, 0), "set_graphs")
    y_eager = dec(z, mask, mu, N)
    _lib.check(L.gt_decoder_set_graphs(h, 1), "set_graphs")
    c0 = L.gt_decoder_graph_captures(h)
    y_graph = dec(z, mask, mu, N)
    torch.cuda.synchronize()
    assert L.gt_decoder_graph_captures(h) > c0
    assert torch.isfinite(y_graph).all()
    assert torch.equal(y_graph, y_eager), f"graph replay differs (max {float((y_graph - y_eager).abs().max()):.3e})"


def test_graph_reused_with_same_buffers():
    """Same shapes and buffers: the second call replays the cached graphs (no new capture)."""
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = _inputs(3, 2, 64)
    B, T, N = 2, 64, 30
    L = _lib.lib()
    h = dec.estimator._native()
    _lib.check(L.gt_decoder_set_graphs(h, 1), "set_graphs")
    dcode = _dtype_code(torch.bfloat16)
    out = torch.empty((B, 80, T), dtype=torch.float32, device="cuda")
    ws = torch.empty(L.gt_decoder_workspace_bytes(h, dcode, B, T, N), dtype=torch.uint8, device="cuda")

    def call():
        _lib.check(L.gt_reverse_diffusion(h, dcode, z.data_ptr(), mask.data_ptr(), mu.data_ptr(), None, B, T, N,
                                          out.data_ptr(), ws.data_ptr(), ws.numel(), _stream_ptr(out.device)),
                   "gt_reverse_diffusion")
        torch.cuda.synchronize()
        return out.clone()

    t0 = time.perf_counter()
    y1 = call()
    t_first = time.perf_counter() - t0
    c1 = L.gt_decoder_graph_captures(h)
    t0 = time.perf_counter()
    y2 = call()
    t_replay = time.perf_counter() - t0
    assert L.gt_decoder_graph_captures(h) == c1
    assert torch.equal(y1, y2)
    print(f"GRAPH first call (capture) {t_first * 1e3:.1f} ms, replay {t_replay * 1e3:.1f} ms")


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_forced_chunks_bit_exact(cdt, monkeypatch):
    """GT_MAX_CHUNK=2: a batch of 5 runs as chunks 2 + 2 + 1, bit-identical to one chunk."""
    mu, z, mask, _ = _inputs(11, 5, 96, lengths=[96, 80, 96, 40, 72])
    dec_full, _ = make_decoder(1, 0, cdt)
    y_full = dec_full(z, mask, mu, 4)
    est_full = dec_full.estimator(z, mask, mu, torch.full((5,), 0.37, device="cuda"))
    monkeypatch.setenv("GT_MAX_CHUNK", "2")
    dec_chunk, _ = make_decoder(1, 0, cdt)
    y_chunk = dec_chunk(z, mask, mu, 4)
    est_chunk = dec_chunk.estimator(z, mask, mu, torch.full((5,), 0.37, device="cuda"))
    assert torch.equal(y_full, y_chunk)
    assert torch.equal(est_full, est_chunk)


def test_two_chunk_fp32_batch_matches_small_batches():
    """fp32, T = 1024: at most 102 utterances fit one chunk; a batch of 104 runs as 102 + 2 and every
    utterance equals its decode in a batch of 2 (batch invariance)."""
    B, T = 104, 1024
    dec, _ = make_decoder(1, 0, torch.float32)
    mu, z, mask, _ = _inputs(5, B, T)
    t = torch.full((B,), 0.61, device="cuda")
    y = dec.estimator(z, mask, mu, t)
    torch.cuda.synchronize()
    for lo in (0, 100, 102):
        ys = dec.estimator(z[lo:lo + 2].contiguous(), mask[lo:lo + 2].contiguous(), mu[lo:lo + 2].contiguous(),
                           t[lo:lo + 2].contiguous())
        assert torch.equal(y[lo:lo + 2], ys), f"utterances {lo}..{lo + 1} differ"
    assert torch.isfinite(y).all()
