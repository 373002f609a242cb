"""GPU MAS kernel: bit-exact against the reference's own outputs (golden) and the C oracle."""
import numpy as np
import pytest
import torch

from conftest import gpu_available, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _mas(value, mask):
    from gradtts_amd.monotonic_align import maximum_path
    return maximum_path(torch.from_numpy(value).cuda(), torch.from_numpy(mask).cuda()).cpu().numpy()


@pytest.mark.parametrize("name", ["mas_random.npz", "mas_ties.npz", "mas_logprior.npz"])
def test_maximum_path_bit_exact_vs_reference(name):
    g = load_golden(name)
    path = _mas(g["value"], g["mask"])
    np.testing.assert_array_equal(path.astype(np.int8), g["path"])


def test_maximum_path_dtype_device_contract():
    from gradtts_amd.monotonic_align import maximum_path
    g = load_golden("mas_random.npz")
    v = torch.from_numpy(g["value"]).double()
    out = maximum_path(v, torch.from_numpy(g["mask"]).double())   # CPU in -> CPU out, value.dtype
    assert out.device.type == "cpu" and out.dtype == torch.float64
    np.testing.assert_array_equal(out.numpy().astype(np.int8), g["path"])
    vc = torch.from_numpy(g["value"]).cuda()
    before = vc.clone()
    maximum_path(vc, torch.from_numpy(g["mask"]).cuda())
    assert torch.equal(vc, before)   # values are never mutated


@pytest.mark.parametrize("txm,tym,b", [(1, 7, 3), (64, 64, 2), (65, 300, 4), (130, 257, 3), (400, 1024, 2),
                                       (700, 1000, 2), (1030, 1100, 1)])
def test_maximum_path_random_vs_oracle(txm, tym, b, mas_oracle):
    rng = np.random.default_rng(txm * 1000 + tym)
    t_x = rng.integers(max(1, txm // 2), txm + 1, b).astype(np.int32)
    t_x[0] = txm
    t_y = np.array([rng.integers(tx, tym + 1) for tx in t_x], np.int32)
    t_y[-1] = tym
    for kind in ("normal", "ties"):
        v = (rng.standard_normal((b, txm, tym)) if kind == "normal" else rng.integers(-2, 3, (b, txm, tym))).astype(np.float32)
        mask = np.zeros_like(v)
        for i in range(b):
            mask[i, :t_x[i], :t_y[i]] = 1
        ref, _ = mas_oracle(v * mask, t_x, t_y)
        got = _mas(v, mask)
        np.testing.assert_array_equal(got.astype(np.int32), ref)


def test_maximum_path_known_answers():
    v = np.random.default_rng(0).standard_normal((2, 40, 40)).astype(np.float32)
    mask = np.zeros_like(v)
    mask[0] = 1                  # t_x == t_y -> diagonal
    mask[1, :1, :] = 1           # t_x == 1 -> row 0 all ones
    p = _mas(v, mask)
    np.testing.assert_array_equal(p[0], np.eye(40))
    assert p[1, 0].sum() == 40 and p[1, 1:].sum() == 0
    # properties: one active row per valid column, monotone, corners set
    g = load_golden("mas_logprior.npz")
    p = _mas(g["value"], g["mask"])
    for b in range(p.shape[0]):
        tx, ty = int(g["mask"][b].sum(0)[0]), int(g["mask"][b].sum(1)[0])
        rows = p[b, :, :ty].argmax(0)
        assert (p[b, :, :ty].sum(0) == 1).all() and (np.diff(rows) >= 0).all() and (np.diff(rows) <= 1).all()
        assert p[b, 0, 0] == 1 and p[b, tx - 1, ty - 1] == 1 and p[b, :, ty:].sum() == 0
