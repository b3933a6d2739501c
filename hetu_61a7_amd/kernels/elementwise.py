"""Unary / binary / scalar elementwise ops (HIP ``elementwise.hip``)."""
from __future__ import annotations

import math

import ctypes

import torch
import torch.nn.functional as F
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32, F32

U = dict(relu=0, sigmoid=1, tanh=2, exp=3, log=4, sqrt=5, rsqrt=6, abs=7, neg=8, gelu=9,
         leaky_relu=10, floor=11, sin=12, cos=13, add_c=14, mul_c=15, rsub_c=16, rdiv_c=17,
         pow_c=18, cpow=19, clamp=20, sign=21, gt_c=22, recip=23, square=24, gelu_tanh=25)
B = dict(add=0, sub=1, mul=2, div=3, max=4, min=5, relu_grad=6, gelu_grad=7, tanh_grad=8,
         sigmoid_grad=9, leaky_relu_grad=10, abs_grad=11, pow=12, add_relu=13, log_grad=14,
         sqrt_grad=15, gelu_tanh_grad=16, relu_grad_c=17)


def _ref_unary(op, x, c, c2):
    if op == 'relu':
        return torch.relu(x)
    if op == 'sigmoid':
        return torch.sigmoid(x)
    if op == 'tanh':
        return torch.tanh(x)
    if op == 'exp':
        return torch.exp(x)
    if op == 'log':
        return torch.log(x)
    if op == 'sqrt':
        return torch.sqrt(x)
    if op == 'rsqrt':
        return torch.rsqrt(x)
    if op == 'abs':
        return torch.abs(x)
    if op == 'neg':
        return -x
    if op == 'gelu':
        return F.gelu(x)
    if op == 'gelu_tanh':
        return F.gelu(x, approximate='tanh')
    if op == 'leaky_relu':
        return F.leaky_relu(x, c)
    if op == 'floor':
        return torch.floor(x)
    if op == 'sin':
        return torch.sin(x)
    if op == 'cos':
        return torch.cos(x)
    if op == 'add_c':
        return x + c
    if op == 'mul_c':
        return x * c
    if op == 'rsub_c':
        return c - x
    if op == 'rdiv_c':
        return c / x
    if op == 'pow_c':
        return torch.pow(x, c)
    if op == 'cpow':
        return torch.pow(torch.tensor(c, dtype=x.dtype, device=x.device), x)
    if op == 'clamp':
        return torch.clamp(x, c, c2)
    if op == 'sign':
        return torch.sign(x)
    if op == 'gt_c':
        return (x > c).to(x.dtype)
    if op == 'recip':
        return torch.reciprocal(x)
    if op == 'square':
        return x * x
    raise KeyError(op)


def unary(op: str, x: torch.Tensor, c: float = 0.0, c2: float = 0.0, out=None) -> torch.Tensor:
    if native(x) and supported_float(x) and x.is_contiguous():
        y = out if out is not None else _NA.empty_like(x)
        f = fn('hetu_unary', [I32, P, P, I64, I32, F32, F32, P])
        check(f(U[op], x.data_ptr(), y.data_ptr(), x.numel(), is_bf16(x), float(c), float(c2),
                stream_ptr()), 'unary:' + op)
        return y
    from . import cpu_native
    if cpu_native.active(x, out):
        return cpu_native.unary_code(U[op], x, c, c2, out)
    cpu_native.record_fallback('unary:' + op, x)
    r = _ref_unary(op, x, c, c2)
    if out is not None:
        out.copy_(r)
        return out
    return r


def _ref_binary(op, a, b, c):
    if op == 'add':
        return a + b
    if op == 'sub':
        return a - b
    if op == 'mul':
        return a * b
    if op == 'div':
        return a / b
    if op == 'max':
        return torch.maximum(a, b.to(a.dtype))
    if op == 'min':
        return torch.minimum(a, b.to(a.dtype))
    if op == 'relu_grad':
        return torch.where(a > 0, b, _NA.zeros_like(b))
    if op == 'gelu_grad':
        cdf = 0.5 * (1.0 + torch.erf(a / math.sqrt(2.0)))
        pdf = torch.exp(-0.5 * a * a) / math.sqrt(2 * math.pi)
        return b * (cdf + a * pdf)
    if op == 'relu_grad_c':
        return torch.where(a > 0, b * c, torch.zeros_like(b))
    if op == 'gelu_tanh_grad':
        k = math.sqrt(2 / math.pi)
        u = k * (a + 0.044715 * a ** 3)
        t = torch.tanh(u)
        return b * (0.5 * (1 + t) + 0.5 * a * (1 - t * t) * k * (1 + 3 * 0.044715 * a * a))
    if op == 'tanh_grad':
        return b * (1 - a * a)
    if op == 'sigmoid_grad':
        return b * a * (1 - a)
    if op == 'leaky_relu_grad':
        return torch.where(a > 0, b, c * b)
    if op == 'abs_grad':
        return torch.sign(a) * b
    if op == 'pow':
        return torch.pow(a, b)
    if op == 'add_relu':
        return torch.relu(a + b)
    if op == 'log_grad':
        return b / a
    if op == 'sqrt_grad':
        return b * 0.5 / a
    raise KeyError(op)


def binary(op: str, a: torch.Tensor, b: torch.Tensor, c: float = 0.0, out=None) -> torch.Tensor:
    """``a`` sets the output shape/dtype; ``b`` is same-shape, a trailing-row
    broadcast (``b.numel()`` == ``a.shape[-k:]`` product) or a scalar tensor."""
    if native(a, b) and supported_float(a) and supported_float(b) and a.is_contiguous() \
            and b.is_contiguous() and b.device == a.device:
        if b.shape == a.shape:
            mode, inner = 0, a.numel()
        elif b.numel() == 1:
            mode, inner = 2, 1
        elif a.dim() >= b.dim() and tuple(a.shape[a.dim() - b.dim():]) == tuple(b.shape):
            mode, inner = 1, b.numel()
        else:
            mode, inner = -1, 1
        bnum = 1
        if mode < 0:
            m3 = _periodic(a, b)
            if m3 is not None:
                mode, (inner, bnum) = 3, m3
        if mode >= 0:
            y = out if out is not None else _NA.empty_like(a)
            f = fn('hetu_binary3', [I32, P, P, P, I64, I32, I32, I32, I64, I64, F32, P])
            check(f(B[op], a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), is_bf16(a),
                    is_bf16(b), mode, inner, bnum, float(c), stream_ptr()), 'binary:' + op)
            return y
        r = _binary_nd(op, a, b, c, out)
        if r is not None:
            return r
    elif native(a, b) and supported_float(a) and supported_float(b) and b.device == a.device:
        r = _binary_nd(op, a, b, c, out)
        if r is not None:
            return r
    if native(a, b):
        from . import record_fallback
        record_fallback('binary:' + op, 'dtype %s/%s' % (a.dtype, b.dtype))
    if b.dtype != a.dtype and b.numel() <= a.numel():
        b = b.to(a.dtype)
    from . import cpu_native
    if cpu_native.active(a, b, out):
        try:
            shape = torch.broadcast_shapes(a.shape, b.shape)
        except RuntimeError:
            shape = None
        if shape is not None and (out is None or tuple(out.shape) == tuple(shape)):
            r = cpu_native.binary_code(B[op], a, b, c, out)
            if r is not None:
                return r
    cpu_native.record_fallback('binary:' + op, a, b)
    r = _ref_binary(op, a, b, c)
    if r.dtype != a.dtype and a.dtype.is_floating_point:
        r = r.to(a.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def _periodic(a, b):
    """(inner, bnum) when contiguous ``b`` broadcast to ``a`` equals b[(i // inner) % bnum]
    for flat index i -- b spans one contiguous block of a's dims ([T,1] vs [T,d],
    [1,C,1,1] vs [N,C,H,W]); else None"""
    nd = a.dim()
    if b.dim() > nd:
        return None
    bs = [1] * (nd - b.dim()) + list(b.shape)
    full = [i for i in range(nd) if bs[i] != 1]
    if not full:
        return None
    j, k = full[0], full[-1] + 1
    if any(bs[i] != a.shape[i] for i in range(j, k)):
        return None
    inner = 1
    for d in a.shape[k:]:
        inner *= int(d)
    return inner, b.numel()


def _collapse(shape, sa, sb):
    """drop unit dims and merge neighbours that are contiguous in all three of the
    output (row-major ``shape``), a and b"""
    dims = [(int(n), int(x), int(y)) for n, x, y in zip(shape, sa, sb) if n != 1]
    out = []
    for n, x, y in dims:
        if out and out[-1][1] == n * x and out[-1][2] == n * y:
            n0 = out[-1][0]
            out[-1] = (n0 * n, x, y)
        else:
            out.append((n, x, y))
    if not out:
        out = [(1, 0, 0)]
    return [d[0] for d in out], [d[1] for d in out], [d[2] for d in out]


def _binary_nd(op, a, b, c, out):
    """General broadcast / strided form (``hetu_binary_nd``): the output takes the
    broadcast shape of a and b in a's dtype; None when it needs more than 8 dims."""
    try:
        shape = torch.broadcast_shapes(a.shape, b.shape)
    except RuntimeError:
        return None
    if len(shape) > 8:
        return None
    if len(shape) == 0:
        shape = (1,)
        a, b = a.reshape(1), b.reshape(1)
    ae, be = a.expand(shape), b.expand(shape)
    if out is not None and (tuple(out.shape) != tuple(shape) or not out.is_contiguous() or out.dtype != a.dtype):
        return None
    y = out if out is not None else _NA.empty(shape, dtype=a.dtype, device=a.device)
    cs, ca, cb = _collapse(shape, ae.stride(), be.stride())
    nd = len(cs)
    arr = ctypes.c_int64 * nd
    f = fn('hetu_binary_nd', [I32, P, P, P, I32, P, P, P, I32, I32, F32, P])
    check(f(B[op], a.data_ptr(), b.data_ptr(), y.data_ptr(), nd, arr(*cs), arr(*ca), arr(*cb),
            is_bf16(a), is_bf16(b), float(c), stream_ptr()), 'binary_nd:' + op)
    return y


def cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if x.dtype == dtype:
        return x
    if native(x) and x.is_contiguous() and {x.dtype, dtype} == {torch.float32, torch.bfloat16}:
        y = _NA.empty(x.shape, dtype=dtype, device=x.device)
        f = fn('hetu_cast', [P, I32, P, I32, I64, P])
        check(f(x.data_ptr(), is_bf16(x), y.data_ptr(), 1 if dtype == torch.bfloat16 else 0,
                x.numel(), stream_ptr()), 'cast')
        return y
    return x.to(dtype)
