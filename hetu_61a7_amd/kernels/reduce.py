"""Axis reductions (``pool.hip`` reduce_mid / reduce_last / bcast_mid)."""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32, F32


def reduce_mid(x3: torch.Tensor, scale: float = 1.0, out_dtype=None, out=None) -> torch.Tensor:
    """x3 [B, R, C] contiguous -> [B, C] = scale * sum over R (into ``out`` if given)."""
    B, R, C = x3.shape
    if out is not None:
        out_dtype = out.dtype
    out_dtype = out_dtype or x3.dtype
    if native(x3) and supported_float(x3) and out_dtype in (torch.float32, torch.bfloat16):
        x3 = x3.contiguous()
        wsf = fn('hetu_reduce_mid_ws', [I64, I64, I64], restype=I64)
        ws = _NA.empty(wsf(B, R, C), dtype=torch.float32, device=x3.device)
        y = out if out is not None else _NA.empty((B, C), dtype=out_dtype, device=x3.device)
        f = fn('hetu_reduce_mid', [P, P, I64, I64, I64, F32, I32, I32, P, P])
        check(f(x3.data_ptr(), y.data_ptr(), B, R, C, float(scale), is_bf16(x3),
                1 if out_dtype == torch.bfloat16 else 0, ws.data_ptr(), stream_ptr()), 'reduce_mid')
        return y
    from . import cpu_native
    if out_dtype == torch.float32 and cpu_native.active(x3, out):
        if C == 1:
            y = cpu_native.reduce_lastdim(x3.reshape(B, R), scale).reshape(B, 1)
        elif B == 1:
            y = cpu_native.reduce_axis0(x3.reshape(R, C), scale).reshape(1, C)
        else:
            y = torch.stack([cpu_native.reduce_axis0(x3[b], scale) for b in range(B)]) if B <= 16 else None
            if y is None:   # many short reductions: sum over R of each [C] row block via a permute
                xt = _NA.empty((R, B, C), dtype=torch.float32)
                cpu_native.copy_nd(x3.permute(1, 0, 2), xt)
                y = cpu_native.reduce_axis0(xt.reshape(R, B * C), scale).reshape(B, C)
        if out is not None:
            cpu_native.copy_nd(y.reshape(out.shape), out)
            return out
        return y
    cpu_native.record_fallback('reduce_mid', x3)
    r = (x3.float().sum(1) * scale).to(out_dtype)
    if out is not None:
        out.copy_(r.reshape(out.shape))
        return out
    return r


def reduce_last(x2: torch.Tensor, scale: float = 1.0, out_dtype=None) -> torch.Tensor:
    R, C = x2.shape
    out_dtype = out_dtype or x2.dtype
    if native(x2) and supported_float(x2) and out_dtype in (torch.float32, torch.bfloat16):
        x2 = x2.contiguous()
        y = _NA.empty((R,), dtype=out_dtype, device=x2.device)
        f = fn('hetu_reduce_last', [P, P, I64, I64, F32, I32, I32, P])
        check(f(x2.data_ptr(), y.data_ptr(), R, C, float(scale), is_bf16(x2),
                1 if out_dtype == torch.bfloat16 else 0, stream_ptr()), 'reduce_last')
        return y
    from . import cpu_native
    if out_dtype == torch.float32 and cpu_native.active(x2):
        return cpu_native.reduce_lastdim(x2, scale)
    cpu_native.record_fallback('reduce_last', x2)
    return (x2.float().sum(1) * scale).to(out_dtype)


def reduce_sum(x: torch.Tensor, dims, keepdim: bool = False) -> torch.Tensor:
    """Sum over ``dims`` (any set) with the native middle-axis reduction, one pass per
    reduced dim (fp32 result)."""
    dims = sorted({d % x.dim() for d in dims}, reverse=True)
    y = x.contiguous()
    shape = list(x.shape)
    for d in dims:
        outer = 1
        for s_ in shape[:d]:
            outer *= s_
        inner = 1
        for s_ in shape[d + 1:]:
            inner *= s_
        y = reduce_mid(y.reshape(outer, shape[d], inner), out_dtype=torch.float32)
        shape[d] = 1
        y = y.reshape(shape)
    if not keepdim:
        y = y.reshape([s_ for i, s_ in enumerate(shape) if i not in dims])
    return y


def sum_to_shape(g: torch.Tensor, shape) -> torch.Tensor:
    """Reduce a broadcast gradient back to ``shape`` (numpy broadcasting rules)."""
    shape = tuple(shape)
    if tuple(g.shape) == shape:
        return g
    nd = g.dim()
    full = (1,) * (nd - len(shape)) + shape
    # fast path: leading-dims reduction (bias / row-broadcast) -> reduce_mid
    k = 0
    while k < nd and full[k] == 1 and g.shape[k] != 1:
        k += 1
    if all(full[i] == g.shape[i] for i in range(k, nd)) and g.is_contiguous():
        lead = 1
        for i in range(k):
            lead *= g.shape[i]
        inner = g.numel() // max(lead, 1)
        return reduce_mid(g.reshape(1, lead, inner)).reshape(shape)
    dims = [i for i in range(nd) if full[i] == 1 and g.shape[i] != 1]
    from . import cpu_native
    if cpu_native.active(g) and dims:
        return reduce_sum(g, dims, keepdim=True).reshape(shape)
    r = g.float().sum(dim=dims, keepdim=True) if dims else g.float()
    return r.reshape(shape).to(g.dtype)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """x logical NCHW -> [N, C] mean over H*W (channels-last fast path)."""
    N, C, H, W = x.shape
    if native(x) and supported_float(x):
        xc = x.contiguous(memory_format=torch.channels_last)
        return reduce_mid(xc.permute(0, 2, 3, 1).reshape(N, H * W, C), 1.0 / (H * W))
    from . import cpu_native
    if cpu_native.active(x):
        return reduce_last(x.contiguous().reshape(N * C, H * W), 1.0 / (H * W)).reshape(N, C)
    return x.float().mean((2, 3)).to(x.dtype)


def global_avg_pool_backward(dy: torch.Tensor, x_shape) -> torch.Tensor:
    N, C, H, W = x_shape
    if native(dy) and supported_float(dy):
        dy = dy.contiguous()
        dx = _NA.empty((N, C, H, W), dtype=dy.dtype, device=dy.device,
                         memory_format=torch.channels_last)
        f = fn('hetu_bcast_mid', [P, P, I64, I64, I64, F32, I32, P])
        check(f(dy.data_ptr(), dx.data_ptr(), N, H * W, C, 1.0 / (H * W), is_bf16(dy),
                stream_ptr()), 'bcast_mid')
        return dx
    from . import cpu_native
    if cpu_native.active(dy):
        dx = _NA.empty((N, C, H, W), dtype=torch.float32)
        cpu_native.copy_nd(dy.reshape(N, C, 1, 1).expand(N, C, H, W), dx)
        return cpu_native.unary_code(15, dx, 1.0 / (H * W), out=dx)
    return (dy.reshape(N, C, 1, 1).float() / (H * W)).expand(N, C, H, W).to(dy.dtype).contiguous()
