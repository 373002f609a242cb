"""fp8 (OCP e4m3) weight quantization of the GT_BF16_W8 mode (BASELINE.json config 5), host side.

The library quantizes the 3x3 / Downsample / Upsample weights when it packs them (gt_quantize_e4m3,
include/gradtts.h). Its rounding must be bit-identical to torch's float8_e4m3fn conversion, which the
oracle's quantize_e4m3 (oracle/decoder.py) uses to build the dequantized weights the W8 GPU path is
checked against (tests/test_decoder_gpu.py). No GPU needed: these are host functions of the library.
"""
import ctypes

import numpy as np
import torch

from gradtts_amd import _lib
from gradtts_amd.params import synthetic_state_dict
from oracle import decoder as odec


def test_e4m3_conversion_matches_torch_on_every_bf16_value():
    """Every finite bf16 bit pattern with |x| <= 448 (all e4m3 rounding ties, subnormals, signed zero)."""
    bits = np.arange(1 << 16, dtype=np.uint32) << 16
    x = bits.view(np.float32)
    x = x[np.isfinite(x) & (np.abs(x) <= 448.0)]
    want = torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    f = _lib.lib().gt_f32_to_e4m3
    got = np.fromiter((f(float(v)) for v in x), dtype=np.uint8, count=len(x))
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(float(x[i]), int(got[i]), int(want[i])) for i in bad[:8]]


def test_e4m3_saturates_instead_of_nan():
    f = _lib.lib().gt_f32_to_e4m3
    assert f(470.0) == 0x7E and f(-1e6) == 0xFE


def test_quantize_matches_oracle_per_output_channel():
    L = _lib.lib()
    sd = synthetic_state_dict(seed=3)
    keys = [k for k in sd if odec.is_fp8_key(k)]
    assert len(keys) == 29   # 24 ResnetBlock convs + final_block, 2 Downsample, 2 Upsample
    for k in keys:
        w = torch.from_numpy(sd[k])
        ax = odec.fp8_axis(k)
        q_ref, s_ref = odec.quantize_e4m3(w, ax)
        wm = w.movedim(ax, 0).contiguous()            # rows = output channels
        rows, cols = wm.shape[0], wm[0].numel()
        q = np.zeros(rows * cols, np.uint8)
        s = np.zeros(rows, np.float32)
        rc = L.gt_quantize_e4m3(wm.numpy().ctypes.data_as(ctypes.c_void_p), rows, cols, cols, 1,
                                q.ctypes.data_as(ctypes.c_void_p), s.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0
        np.testing.assert_array_equal(s, s_ref.numpy(), err_msg=k)
        np.testing.assert_array_equal(q.reshape(wm.shape), q_ref.movedim(ax, 0).numpy(), err_msg=k)


def test_fp8_params_error_envelope():
    """Dequantized weights are within half an e4m3 step (2^-4 relative) of the originals, and the
    zero channel case keeps scale 1."""
    sd = synthetic_state_dict(seed=0)
    p8 = odec.fp8_params(sd)
    for k, v in sd.items():
        if not odec.is_fp8_key(k):
            assert torch.equal(p8[k], torch.from_numpy(v))
            continue
        w = torch.from_numpy(v)
        ax = odec.fp8_axis(k)
        red = tuple(d for d in range(w.dim()) if d != ax)
        amax = w.abs().amax(dim=red, keepdim=True)
        # normal range: relative error <= 2^-4; subnormal range: absolute error <= 2^-10 * amax/448
        err = (p8[k] - w).abs()
        bound = torch.maximum(w.abs() * 2.0 ** -4, amax / 448.0 * 2.0 ** -10) * (1 + 1e-6)
        assert bool((err <= bound).all()), k
    q, s = odec.quantize_e4m3(torch.zeros(2, 3, 3, 3), 0)
    assert torch.equal(s, torch.ones(2)) and int(q.sum()) == 0


def test_activation_quantizer_of_the_fp8_operand_mode():
    """oracle.decoder.quantize_act_e4m3 (GT_FP8's conv-operand quantization, csrc/conv.hip store_item_a8): one
    power-of-two scale 2^k per (utterance, position, 32 channels) with k the least integer keeping max|x| / 2^k <= 448;
    values already on that grid are unchanged, an all-zero block stays zero, the error is at most half an e4m3 step."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 3, 7, generator=g) * torch.logspace(-6, 6, 7)      # a wide range of magnitudes per column
    x[0, 32:, 1, 2] = 0
    q = odec.quantize_act_e4m3(x)
    blocks = x.reshape(2, 2, 32, 3, 7)
    amax = blocks.abs().amax(2, keepdim=True)
    k = torch.ceil(torch.log2(amax / 448.0)).clamp(min=-126)
    s = torch.exp2(k)
    assert bool(((amax / s) <= 448).all()) and bool(((amax / s)[amax > 0] > 224).all())   # the least such k
    err = (q - x).reshape(blocks.shape).abs()
    assert bool((err <= torch.maximum(blocks.abs() * 2.0 ** -4, s * 2.0 ** -10) * (1 + 1e-6)).all())
    assert bool((q[0, 32:, 1, 2] == 0).all())
    on_grid = torch.tensor([448.0, -1.75, 0.5, 2.0 ** -6] + [0.0] * 28).reshape(1, 32, 1, 1) * 2.0 ** 10
    assert torch.equal(odec.quantize_act_e4m3(on_grid), on_grid)
    with odec.fp8_activations():   # the context only switches the Block-conv hook on, and restores it
        assert odec._ACT_Q is odec.quantize_act_e4m3
    assert odec._ACT_Q is None
