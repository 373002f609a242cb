"""Drop-in ``maximum_path`` (model/monotonic_align/__init__.py:8-23) on the gfx950 MAS kernel.

Same signature and result: ``maximum_path(value [b,t_x,t_y], mask [b,t_x,t_y]) -> path`` of
``value.dtype`` on ``value.device``, bit-identical to the Cython core. Differences by design: no
device->host->device round trip (the reference copies to numpy, __init__.py:16-23), and ``value``
is never mutated. CPU inputs are moved to the current HIP device and the result moved back; there
is no CPU compute path.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib, ops


def maximum_path_c(paths, values, t_xs, t_ys, max_neg_val=-1e9):
    """C-level entry (core.pyx:38-45) on device tensors: int32 paths [b,tx,ty] (written),
    fp32 values [b,tx,ty] (read only), int32 t_xs/t_ys [b]."""
    b, tx, ty = values.shape
    nbytes = lib().gt_maximum_path_workspace_bytes(b, tx, ty)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=values.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(values.device).cuda_stream)
    check(lib().gt_maximum_path(paths.data_ptr(), values.data_ptr(), t_xs.data_ptr(), t_ys.data_ptr(), b, tx, ty,
                                float(max_neg_val), ws.data_ptr(), ws.numel(), stream), "gt_maximum_path")


@torch.no_grad()
def maximum_path(value, mask):
    """value: [b, t_x, t_y]; mask: [b, t_x, t_y]  ->  monotonic alignment path (0/1) as value.dtype."""
    if not torch.cuda.is_available():
        raise RuntimeError("gradtts_amd.maximum_path needs a HIP (MI355X) device; there is no CPU path")
    out_device, out_dtype = value.device, value.dtype
    device = value.device if value.is_cuda else torch.device("cuda", torch.cuda.current_device())
    with torch.cuda.device(device):
        # torch.ops.gradtts.maximum_path (csrc/torch_ops.cpp): value * mask (__init__.py:13), t_x / t_y from the
        # mask (:20-21), the DP on device (:22), path as value.dtype (:23)
        path = ops().maximum_path(value.to(device), mask.to(device))
    return path.to(device=out_device, dtype=out_dtype)
