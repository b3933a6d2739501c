"""2-D convolution (logical NCHW, physical channels-last on the GPU).

The forward/backward-data/backward-filter entry points dispatch per shape to
the hand-written implicit-GEMM MFMA kernel (``gemm.hip`` via ``conv_igemm``)
or to the vendor convolution (MIOpen through torch).  ``HETU_CONV=auto``
(default) selects per shape by measurement (``autotune.choose``), so the
hand-written kernel runs exactly where it is at least as fast; ``hip`` /
``vendor`` force one side.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import native

CL = torch.channels_last
MODE = os.environ.get('HETU_CONV', 'auto')  # hip | vendor | auto (per-shape measured choice)


def _pick(key, hip, vendor):
    if MODE == 'hip':
        r = hip()
        return r if r is not None else vendor()
    if MODE == 'vendor':
        return vendor()
    from .autotune import choose
    c = choose(key, {'hip': hip, 'vendor': vendor})
    if c == 'hip':
        r = hip()
        if r is not None:
            return r
    return vendor()


def _match(x, w):
    if x.dtype != w.dtype:
        if w.dtype == torch.bfloat16 or x.dtype == torch.bfloat16:
            x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
        else:
            w = w.to(x.dtype)
    return x, w


def conv2d(x, w, b, stride, padding):
    x, w = _match(x, w)
    if x.is_cuda:
        x = x.contiguous(memory_format=CL)
        w = w.contiguous(memory_format=CL)
        from . import conv_igemm
        y = _pick(('fwd', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(padding)),
                  lambda: conv_igemm.try_forward(x, w, stride, padding),
                  lambda: F.conv2d(x, w, None, stride, padding))
        if b is not None:
            from .elementwise import binary
            n, c, h, ww = y.shape
            y = binary('add', y.permute(0, 2, 3, 1), b.to(y.dtype).contiguous()).permute(0, 3, 1, 2)
        return y
    y = F.conv2d(x, w, b.to(x.dtype) if b is not None else None, stride, padding)
    return y


def conv2d_backward_data(g, w, x_shape, stride, padding, acc=None):
    """dx (+ acc when given: a gradient joined at the conv input, fused into the
    epilogue on the HIP path)."""
    g, w = _match(g, w)
    if g.is_cuda:
        g = g.contiguous(memory_format=CL)
        w = w.contiguous(memory_format=CL)
        if acc is not None:
            acc = acc.contiguous(memory_format=CL)
        from . import conv_igemm
        return _pick(('dgrad', tuple(g.shape), tuple(w.shape), tuple(stride), tuple(padding), acc is not None),
                     lambda: conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc),
                     lambda: _vendor_dgrad(g, w, x_shape, stride, padding, acc))
    return _vendor_dgrad(g, w, x_shape, stride, padding, acc)


def _vendor_dgrad(g, w, x_shape, stride, padding, acc=None):
    dx = _vendor_dgrad0(g, w, x_shape, stride, padding)
    if acc is not None:
        dx = dx + acc.to(dx.dtype)
    return dx


def _vendor_dgrad0(g, w, x_shape, stride, padding):
    xs = torch.empty(x_shape, dtype=g.dtype, device=g.device)
    if g.is_cuda:
        xs = xs.contiguous(memory_format=CL)
    dx, _, _ = torch.ops.aten.convolution_backward(
        g, xs, w, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [True, False, False])
    return dx


def conv2d_backward_filter(g, x, w_shape, stride, padding, out=None):
    """Weight gradient.  ``out`` (an fp32 channels-last view, e.g. the
    optimizer's flat gradient slot) receives the result in place."""
    g, x = _match(g, x)
    if out is not None and (out.dtype != torch.float32 or tuple(out.shape) != tuple(w_shape) or
                            not out.is_contiguous(memory_format=CL)):
        out = None
    if g.is_cuda:
        g = g.contiguous(memory_format=CL)
        x = x.contiguous(memory_format=CL)
        from . import conv_igemm

        def vendor():
            dw = _vendor_wgrad(g, x, w_shape, stride, padding)
            if out is None:
                return dw
            out.copy_(dw)
            return out
        return _pick(('wgrad', tuple(g.shape), tuple(x.shape), tuple(w_shape), tuple(stride), tuple(padding)),
                     lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                            accumulate=False),
                     vendor)
    dw = _vendor_wgrad(g, x, w_shape, stride, padding)
    if out is not None:
        out.copy_(dw)
        return out
    return dw


def _vendor_wgrad(g, x, w_shape, stride, padding):
    ws = torch.empty(w_shape, dtype=g.dtype, device=g.device)
    if g.is_cuda:
        ws = ws.contiguous(memory_format=CL)
    _, dw, _ = torch.ops.aten.convolution_backward(
        g, x, ws, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [False, True, False])
    return dw
