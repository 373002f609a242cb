"""CPU checks of the storage-emulating oracle (oracle/emulate.py) itself; its GPU pins are tests/test_emulate_gpu.py
and tests/test_fp8_gpu.py."""
import numpy as np
import torch

from conftest import load_golden

EST = ["estimator_s1.npz", "estimator_s247.npz", "estimator_sm1.npz", "estimator_s1_T132.npz", "estimator_s1_T20.npz"]


def test_r16_round_to_nearest_even():
    from oracle.emulate import r16
    one = 1.0
    ulp = 2.0 ** -7   # bf16 spacing in [1, 2)
    x = torch.tensor([one + ulp / 2, one + 1.5 * ulp, one + ulp / 2 + 2 ** -20, -(one + ulp / 2)], dtype=torch.float32)
    assert r16(x).tolist() == [1.0, one + 2 * ulp, one + ulp, -1.0]
    assert torch.equal(r16(r16(x)), r16(x))


def test_attn_tiles_as_decoder_cpp():
    from oracle.emulate import attn_tiles
    assert attn_tiles(80 * 128, 256) == (64, 160)    # small plan, level 0, T = 128
    assert attn_tiles(80 * 512, 16) == (2560, 16)    # throughput plan, >= 8192 positions
    assert attn_tiles(20 * 128, 32) == (128, 20)
    assert attn_tiles(50, 32) == (64, 1)


def test_emulation_is_a_small_perturbation_of_the_reference():
    """bf16 storage moves one estimator call ~1e-2 off the fp32 golden output (the library's bf16 calls measure the same
    distance), fp8 operands ~1e-1; the emulation leaves the fp32 restatement untouched outside its context."""
    from gradtts_amd.params import synthetic_state_dict
    from oracle import decoder as odec, emulate
    for name in EST:
        g = load_golden(name)
        n_spks = int(g["n_spks"])
        sd = synthetic_state_dict(seed=int(g["seed_w"]), n_spks=n_spks)
        args = [torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")]
        spk = torch.from_numpy(g["spk"]) if n_spks != 1 else None
        ref = g["out"]
        scale = np.abs(ref).max()
        with torch.no_grad():
            with emulate.product_storage("bf16"):
                e16 = odec.estimator(odec.to_torch_params(sd), *args, spk, n_spks).numpy()
            with emulate.product_storage("fp8"):
                e8 = odec.estimator(odec.fp8_params(sd), *args, spk, n_spks).numpy()
            plain = odec.estimator(odec.to_torch_params(sd), *args, spk, n_spks).numpy()
        assert 1e-3 < np.abs(e16 - ref).max() / scale < 2.5e-2, name
        assert 2e-2 < np.abs(e8 - ref).max() / scale < 2.5e-1, name
        assert np.abs(plain - ref).max() / scale <= 1e-5, name
