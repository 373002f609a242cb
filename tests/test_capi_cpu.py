"""CPU-only checks of the C ABI and the host mirror (no GPU compute is issued here).

* libgradtts.so loads and exports every function declared in include/gradtts.h;
* the library's parameter inventory == params.py inventory == the module's state_dict keys
  (== the reference registration order, pinned by make_golden.py against the real reference);
* argument validation happens before any HIP call.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from gradtts_amd import _lib
from gradtts_amd.diffusion import Diffusion, GradLogPEstimator2d
from gradtts_amd.params import estimator_param_shapes, synthetic_state_dict


def header_functions():
    txt = open(os.path.join(REPO, "include", "gradtts.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gt_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), f"{n} declared in gradtts.h but not exported"
    assert {s[0] for s in _lib.SIGNATURES} == set(names), "ctypes table out of sync with the header"
    assert b"gfx950" in L.gt_version()


@pytest.mark.parametrize("n_spks", [1, 247, -1])
def test_inventory_matches_params_and_module(n_spks):
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.gt_decoder_create(80, 64, n_spks, 64, 0.05, 20.0, 1000.0, ctypes.byref(h)), "create")
    try:
        names = [L.gt_decoder_param_name(h, i).decode() for i in range(L.gt_decoder_num_params(h))]
        numels = [L.gt_decoder_param_numel(h, i) for i in range(L.gt_decoder_num_params(h))]
        shapes = estimator_param_shapes(64, n_spks)
        assert names == list(shapes.keys())
        assert numels == [int(np.prod(s)) for s in shapes.values()]
        est = GradLogPEstimator2d(64, n_spks=n_spks)
        sd = est.state_dict()
        assert list(sd.keys()) == names
        assert [tuple(v.shape) for v in sd.values()] == [tuple(s) for s in shapes.values()]
    finally:
        L.gt_decoder_destroy(h)


def test_reference_state_dict_loads_into_module():
    dec = Diffusion(80, 64, 1, 64, 0.05, 20, 1000)
    sd = synthetic_state_dict(seed=3)
    missing, unexpected = dec.load_state_dict({"estimator." + k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    assert not missing and not unexpected
    assert torch.equal(dec.estimator.downs[1][2].fn.fn.to_qkv.weight, torch.from_numpy(sd["downs.1.2.fn.fn.to_qkv.weight"]))


def test_argument_validation_before_any_hip_call():
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.gt_decoder_create(80, 32, 1, 64, 0.05, 20.0, 1000.0, ctypes.byref(h)) == _lib.GT_ERR_UNSUPPORTED
    assert L.gt_decoder_create(80, 64, 1, 64, 0.05, 20.0, 1000.0, ctypes.byref(h)) == _lib.GT_OK
    try:
        x = np.zeros(4, np.float32)
        assert L.gt_decoder_set_param(h, b"nope.weight", x.ctypes.data, 4) == _lib.GT_ERR_PARAM
        assert L.gt_decoder_set_param(h, b"final_conv.bias", x.ctypes.data, 4) == _lib.GT_ERR_PARAM  # numel 1
        assert L.gt_decoder_set_param(h, b"final_conv.bias", x.ctypes.data, 1) == _lib.GT_OK
        ws = L.gt_decoder_workspace_bytes(h, _lib.GT_BF16, 32, 512, 50)
        assert ws > 0 and L.gt_decoder_workspace_bytes(h, _lib.GT_F32, 32, 512, 50) > ws
        fake = ctypes.c_void_p(16)
        # T not a multiple of 4 -> GT_ERR_ARG (fix_len_compatibility contract), no device access
        rc = L.gt_reverse_diffusion(h, _lib.GT_F32, fake, fake, fake, None, 2, 30, 10, fake, fake, 1 << 40, None)
        assert rc == _lib.GT_ERR_ARG and b"multiple of 4" in L.gt_last_error()
        rc = L.gt_reverse_diffusion(h, _lib.GT_F32, fake, fake, fake, None, 2, 32, 10, fake, fake, 16, None)
        assert rc == _lib.GT_ERR_WORKSPACE
        rc = L.gt_reverse_diffusion(h, 7, fake, fake, fake, None, 2, 32, 10, fake, fake, 1 << 40, None)
        assert rc == _lib.GT_ERR_ARG
        # every parameter must be set before compute -> GT_ERR_PARAM from the lazy packer
        rc = L.gt_reverse_diffusion(h, _lib.GT_F32, fake, fake, fake, None, 2, 32, 10, fake, fake, 1 << 40, None)
        assert rc == _lib.GT_ERR_PARAM and b"never set" in L.gt_last_error()
    finally:
        L.gt_decoder_destroy(h)
    assert L.gt_maximum_path(None, None, None, None, 2, 3, 4, -1e9, None, 0, None) == _lib.GT_ERR_ARG
    assert L.gt_maximum_path_workspace_bytes(2, 30, 100) >= 2 * 100 * 4


def test_product_path_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    dec = Diffusion(80, 64)
    z = torch.zeros(1, 80, 8)
    with pytest.raises(RuntimeError, match="HIP"):
        dec(z, torch.ones(1, 1, 8), z, 2)
    from gradtts_amd.monotonic_align import maximum_path
    with pytest.raises(RuntimeError, match="HIP"):
        maximum_path(torch.zeros(1, 3, 4), torch.ones(1, 3, 4))


def test_torch_ops_registered_with_meta_kernels():
    """torch.ops.gradtts.* (csrc/torch_ops.cpp) load and bind on a CPU-only host; their Meta kernels give
    torch.compile's fake tensors the reference shapes and dtypes, and bad shapes raise like the C ABI."""
    import torch
    from gradtts_amd import _lib
    ops = _lib.ops()
    for name, schema in [
        ("reverse_diffusion", "gradtts::reverse_diffusion(int decoder, int dtype, Tensor z, Tensor mask, Tensor mu, "
                              "int n_timesteps, Tensor? spk) -> Tensor"),
        ("estimator", "gradtts::estimator(int decoder, int dtype, Tensor x, Tensor mask, Tensor mu, Tensor t, "
                      "Tensor? spk) -> Tensor"),
        ("maximum_path", "gradtts::maximum_path(Tensor value, Tensor mask) -> Tensor"),
    ]:
        assert str(getattr(ops, name).default._schema) == schema
    z = torch.empty(3, 80, 64, device="meta", dtype=torch.bfloat16)
    m = torch.empty(3, 1, 64, device="meta")
    y = ops.reverse_diffusion(0, _lib.GT_BF16, z, m, z, 10, None)
    assert y.shape == (3, 80, 64) and y.dtype == torch.bfloat16 and y.device.type == "meta"
    assert ops.estimator(0, _lib.GT_F32, z, m, z, torch.empty(3, device="meta"), None).shape == (3, 80, 64)
    v = torch.empty(2, 7, 30, device="meta")
    assert ops.maximum_path(v, v).shape == (2, 7, 30)
    with pytest.raises(RuntimeError, match="multiple of 4"):
        ops.reverse_diffusion(0, 0, torch.empty(1, 80, 30, device="meta"), torch.empty(1, 1, 30, device="meta"),
                              torch.empty(1, 80, 30, device="meta"), 1, None)


def test_text_encoder_and_vocoder_registries_match_reference_layouts():
    """The C-ABI parameter registries of the text encoder and the HiFi-GAN generator list exactly the reference
    modules' state_dict keys and sizes (tests/golden/gradtts_layout.json, hifigan_layout.json, recorded from the
    real modules); unknown names and wrong sizes are rejected (no GPU needed)."""
    import json
    from gradtts_amd.params import HIFIGAN_V1
    L = _lib.lib()
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    enc_ref = [(k[len("encoder."):], int(np.prod(s))) for k, s in json.load(open(os.path.join(gold, "gradtts_layout.json")))["1"]
               if k.startswith("encoder.")]
    h = ctypes.c_void_p()
    assert L.gt_text_encoder_create(149, 80, 192, 768, 256, 2, 6, 3, 4, ctypes.byref(h)) == 0
    try:
        got = [(L.gt_text_encoder_param_name(h, i).decode(), L.gt_text_encoder_param_numel(h, i))
               for i in range(L.gt_text_encoder_num_params(h))]
        assert got == enc_ref
        x = np.zeros(4, np.float32)
        assert L.gt_text_encoder_set_param(h, b"no.such.param", x.ctypes.data, 4) == 3
        assert L.gt_text_encoder_set_param(h, b"proj_w.proj.bias", x.ctypes.data, 4) == 3
        assert L.gt_text_encoder_set_param(h, b"proj_w.proj.bias", x.ctypes.data, 1) == 0
        assert L.gt_text_encoder_workspace_bytes(h, 2, 10) > 0
    finally:
        L.gt_text_encoder_destroy(h)
    voc_ref = [(k, int(np.prod(s))) for k, s in json.load(open(os.path.join(gold, "hifigan_layout.json")))]
    ia = lambda xs: (ctypes.c_int * len(xs))(*xs)
    v = ctypes.c_void_p()
    dil = [d for ds in HIFIGAN_V1["resblock_dilation_sizes"] for d in ds]
    assert L.gt_vocoder_create(80, 512, 4, ia([8, 8, 2, 2]), ia([16, 16, 4, 4]), 3, ia([3, 7, 11]), ia(dil),
                               ctypes.byref(v)) == 0
    try:
        got = [(L.gt_vocoder_param_name(v, i).decode(), L.gt_vocoder_param_numel(v, i))
               for i in range(L.gt_vocoder_num_params(v))]
        assert got == voc_ref
        assert L.gt_vocoder_hop(v) == 256
        assert L.gt_vocoder_set_compute_dtype(v, 1) == 0 and L.gt_vocoder_set_compute_dtype(v, 2) == 1
        assert L.gt_vocoder_workspace_bytes(v, 1, 10) > 0
    finally:
        L.gt_vocoder_destroy(v)
    # an unsupported configuration (upsampling kernel != 2 x rate) is refused at creation
    assert L.gt_vocoder_create(80, 512, 1, ia([8]), ia([15]), 3, ia([3, 7, 11]), ia(dil), ctypes.byref(v)) == 4
    # HiFi-GAN V3 (ResBlock2, 2 dilations per resblock): the reference Generator's layout
    from gradtts_amd.params import HIFIGAN_V3, vocoder_param_shapes
    dil3 = [d for ds in HIFIGAN_V3["resblock_dilation_sizes"] for d in ds]
    assert L.gt_vocoder_create2(80, 256, 3, ia([8, 8, 4]), ia([16, 16, 8]), 3, ia([3, 5, 7]), 2, 2, ia(dil3),
                                ctypes.byref(v)) == 0
    try:
        got = [(L.gt_vocoder_param_name(v, i).decode(), L.gt_vocoder_param_numel(v, i))
               for i in range(L.gt_vocoder_num_params(v))]
        assert got == [(k, int(np.prod(s))) for k, s in vocoder_param_shapes(HIFIGAN_V3).items()]
        assert L.gt_vocoder_hop(v) == 256
    finally:
        L.gt_vocoder_destroy(v)
    assert L.gt_vocoder_create2(80, 256, 3, ia([8, 8, 4]), ia([16, 16, 8]), 3, ia([3, 5, 7]), 3, 2, ia(dil3),
                                ctypes.byref(v)) == 1   # resblock must be 1 or 2
