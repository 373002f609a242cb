"""attn_mf_kernel (csrc/attn.hip): the attention block's partial merge + weight fold as one launch.

It performs the same operations in the same order as attn_merge_kernel + attn_fold_kernel (four tile groups merged
online, combined in a fixed order; A_b by the same e-ordered fp32 chain; the fold on exact-fp32 MFMA), so a decoder
built with GT_ATTN_MF=1 must give bit-identical estimator outputs and samples to one built with
GT_ATTN_MF=0 -- at every level (C = 64, 128, 256), fp32 and bf16, ragged batches, several attention tile counts."""
import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder
from gradtts_amd.params import synthetic_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _run(monkeypatch, mf, dtype, n_spks, args, N):
    monkeypatch.setenv("GT_ATTN_MF", "1" if mf else "0")   # (default: off)
    # attn_mf merges in attn_merge_kernel<32>'s four tile groups; the small-batch plan (these batches) defaults to the
    # 32-group merge (GT_MERGE_DR_SMALL=4), so both runs take the four-group merge here
    monkeypatch.setenv("GT_MERGE_DR_SMALL", "32")
    dec, _ = make_decoder(n_spks, 7, dtype)
    z, mask, mu, t, spk = args
    est = dec.estimator(z, mask, mu, t, spk)
    y = dec(z, mask, mu, N, spk=spk)
    torch.cuda.synchronize()
    return est.cpu(), y.cpu()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n_spks,B,T,lengths", [(1, 3, 132, [132, 100, 44]), (247, 2, 512, [512, 300])])
def test_merge_fold_fused_bit_identical(monkeypatch, dtype, n_spks, B, T, lengths):
    mu, z, mask, spk = synthetic_inputs(17, B, T, lengths=lengths)
    t = np.linspace(0.8, 0.3, B).astype(np.float32)
    args = (_cuda(z), _cuda(mask), _cuda(mu), _cuda(t), _cuda(spk) if n_spks > 1 else None)
    e1, y1 = _run(monkeypatch, True, dtype, n_spks, args, 3)
    e0, y0 = _run(monkeypatch, False, dtype, n_spks, args, 3)
    assert torch.isfinite(e1).all() and torch.isfinite(y1).all()
    assert torch.equal(e1, e0), float((e1 - e0).abs().max())
    assert torch.equal(y1, y0), float((y1 - y0).abs().max())
