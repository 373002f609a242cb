"""torch.ops.gradtts.* (csrc/torch_ops.cpp, TORCH_LIBRARY(gradtts)) on the MI355X.

* the ops themselves against the reference's golden vectors (the drop-in modules call them too);
* torch.compile traces them through their Meta kernels (fullgraph, aot_eager backend) and gives the eager result;
* torch.cuda.graph captures a call (the C ABI sees the capturing stream and launches into the caller's graph) and
  replays it with new inputs bit-identically to eager calls.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available, load_golden
from gpu_util import make_decoder, rel_err, report
from gradtts_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")
    _lib.ops()   # registers torch.ops.gradtts (libgradtts_ops.so) for tests that name the ops directly


def _c(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_op_reverse_diffusion_matches_golden():
    g = load_golden("reverse_s1_N10.npz")
    dec, _ = make_decoder(1, int(g["seed_w"]), torch.float32)
    h = dec.estimator._native(dec.beta_min, dec.beta_max)
    y = _lib.ops().reverse_diffusion(h.value, _lib.GT_F32, _c(g["z"]), _c(g["mask"]), _c(g["mu"]),
                                     int(g["n_timesteps"]), None)
    report("op reverse_diffusion reverse_s1_N10 fp32", rel_err(y.cpu().numpy(), g["out"]), 1e-4)


def test_op_estimator_and_maximum_path_match_golden():
    g = load_golden("estimator_s247.npz")
    dec, _ = make_decoder(247, int(g["seed_w"]), torch.float32)
    h = dec.estimator._native()
    y = _lib.ops().estimator(h.value, _lib.GT_F32, _c(g["x"]), _c(g["mask"]), _c(g["mu"]), _c(g["t"]), _c(g["spk"]))
    report("op estimator estimator_s247 fp32", rel_err(y.cpu().numpy(), g["out"]), 1e-4)
    m = load_golden("mas_logprior.npz")
    p = _lib.ops().maximum_path(_c(m["value"]), _c(m["mask"]))
    assert p.dtype == torch.float32
    assert np.array_equal(p.cpu().numpy(), m["path"].astype(np.float32))


def test_torch_compile_traces_the_op():
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    h = dec.estimator._native(dec.beta_min, dec.beta_max).value
    g = load_golden("reverse_s1_N10.npz")
    z, mask, mu = _c(g["z"]), _c(g["mask"]), _c(g["mu"])

    def fn(z, mask, mu):
        return torch.ops.gradtts.reverse_diffusion(h, _lib.GT_BF16, z, mask, mu, 6, None) * mask + 1.0

    eager = fn(z, mask, mu)
    compiled = torch.compile(fn, backend="aot_eager", fullgraph=True)(z, mask, mu)
    assert torch.equal(compiled, eager)


def test_cuda_graph_capture_and_replay():
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    h = dec.estimator._native(dec.beta_min, dec.beta_max).value
    B, T, N = 2, 64, 5
    ins = [torch.randn(B, 80, T, device="cuda") for _ in range(2)]
    mask = torch.ones(B, 1, T, device="cuda")
    mask[1, :, 40:] = 0
    mu = torch.randn(B, 80, T, device="cuda")
    op = torch.ops.gradtts.reverse_diffusion
    z = ins[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        op(h, _lib.GT_BF16, z, mask, mu, N, None)        # warm-up (weights packed, code loaded) off the capture
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = op(h, _lib.GT_BF16, z, mask, mu, N, None)
    for x in ins:
        z.copy_(x)
        graph.replay()
        torch.cuda.synchronize()
        ref = op(h, _lib.GT_BF16, x, mask, mu, N, None)
        assert torch.equal(y, ref)
