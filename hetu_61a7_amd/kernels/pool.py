"""Pooling (channels-last) bindings (``pool.hip``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I32

CL = torch.channels_last


def _out_hw(H, W, kh, kw, sh, sw, ph, pw):
    return (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1


def maxpool2d(x, kh, kw, sh, sw, ph, pw):
    """x logical NCHW (any layout); returns (y channels-last, argmax-tap bytes)."""
    N, C, H, W = x.shape
    Ho, Wo = _out_hw(H, W, kh, kw, sh, sw, ph, pw)
    if native(x) and supported_float(x):
        x = x.contiguous(memory_format=CL)
        y = _NA.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=CL)
        idx = _NA.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        f = fn('hetu_maxpool_fwd', [P, P, P] + [I32] * 13 + [P])
        check(f(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw,
                ph, pw, is_bf16(x), stream_ptr()), 'maxpool')
        return y, idx
    from . import cpu_native
    if cpu_native.active(x):
        return cpu_native.maxpool2d(x, kh, kw, sh, sw, ph, pw)
    y, ind = F.max_pool2d(x.float(), (kh, kw), (sh, sw), (ph, pw), return_indices=True)
    return y.to(x.dtype), ind


def maxpool2d_backward(dy, idx, x_shape, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x_shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    if native(dy) and supported_float(dy) and idx.dtype == torch.uint8:
        dy = dy.contiguous(memory_format=CL)
        dx = _NA.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=CL)
        f = fn('hetu_maxpool_bwd', [P, P, P] + [I32] * 13 + [P])
        check(f(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw,
                ph, pw, is_bf16(dy), stream_ptr()), 'maxpool_bwd')
        return dx
    from . import cpu_native
    if cpu_native.active(dy) and idx.dtype == torch.int32:
        return cpu_native.maxpool2d_backward(dy, idx, x_shape)
    return F.max_unpool2d(dy.float(), idx, (kh, kw), (sh, sw), (ph, pw),
                          output_size=(H, W)).to(dy.dtype)


def avgpool2d(x, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x.shape
    Ho, Wo = _out_hw(H, W, kh, kw, sh, sw, ph, pw)
    if native(x) and supported_float(x):
        x = x.contiguous(memory_format=CL)
        y = _NA.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=CL)
        f = fn('hetu_avgpool_fwd', [P, P] + [I32] * 13 + [P])
        check(f(x.data_ptr(), y.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                is_bf16(x), stream_ptr()), 'avgpool')
        return y
    from . import cpu_native
    if cpu_native.active(x):
        return cpu_native.avgpool2d(x, kh, kw, sh, sw, ph, pw)
    return F.avg_pool2d(x.float(), (kh, kw), (sh, sw), (ph, pw)).to(x.dtype)


def avgpool2d_backward(dy, x_shape, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x_shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    if native(dy) and supported_float(dy):
        dy = dy.contiguous(memory_format=CL)
        dx = _NA.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=CL)
        f = fn('hetu_avgpool_bwd', [P, P] + [I32] * 13 + [P])
        check(f(dy.data_ptr(), dx.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                is_bf16(dy), stream_ptr()), 'avgpool_bwd')
        return dx
    from . import cpu_native
    if cpu_native.active(dy):
        return cpu_native.avgpool2d_backward(dy, x_shape, kh, kw, sh, sw, ph, pw)
    xs = _NA.zeros(x_shape, dtype=torch.float32, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = F.avg_pool2d(xs, (kh, kw), (sh, sw), (ph, pw))
        (g,) = torch.autograd.grad(y, xs, dy.float())
    return g.to(dy.dtype)
