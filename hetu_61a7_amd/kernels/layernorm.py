"""Row LayerNorm forward/backward (``layernorm.hip``): one wave per row, fp32
statistics, fused dx/dgamma/dbeta (two-stage column reduction for the
parameter gradients).  Replaces LayerNorm.cu (fwd block-per-row with
E[x^2]-E[x]^2 variance, bwd = 3 elementwise kernels + 4 cuDNN reductions)."""
from __future__ import annotations

import torch

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32, F32


def layer_norm(x, gamma, beta, eps):
    N = x.shape[-1]
    R = x.numel() // N
    if native(x) and supported_float(x):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        mean = torch.empty(R, dtype=torch.float32, device=x.device)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        f = fn('hetu_layernorm_fwd', [P, P, P, P, P, P, I64, I32, F32, I32, P])
        check(f(xc.data_ptr(), gamma.float().contiguous().data_ptr(), beta.float().contiguous().data_ptr(),
                y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), R, N, float(eps), is_bf16(x),
                stream_ptr()), 'layernorm')
        return y, mean, rstd
    xf = x.float().reshape(R, N)
    mean = xf.mean(1)
    var = xf.var(1, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()
    return y.reshape(x.shape).to(x.dtype), mean, rstd


def layer_norm_backward(dy, x, gamma, mean, rstd):
    N = x.shape[-1]
    R = x.numel() // N
    if native(x) and supported_float(x) and dy.dtype == x.dtype:
        xc, dyc = x.contiguous(), dy.contiguous()
        dx = torch.empty_like(xc)
        ws_rows = min(R, 1024)
        ws = torch.empty(2 * ws_rows * N, dtype=torch.float32, device=x.device)
        dg = torch.empty(N, dtype=torch.float32, device=x.device)
        db = torch.empty(N, dtype=torch.float32, device=x.device)
        f = fn('hetu_layernorm_bwd', [P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, P])
        check(f(dyc.data_ptr(), xc.data_ptr(), gamma.float().contiguous().data_ptr(), mean.data_ptr(),
                rstd.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), ws.data_ptr(), R, N,
                ws_rows, is_bf16(x), stream_ptr()), 'layernorm_bwd')
        return dx, dg, db
    xf = x.float().reshape(R, N)
    g = dy.float().reshape(R, N)
    xhat = (xf - mean[:, None]) * rstd[:, None]
    dg = (g * xhat).sum(0)
    db = g.sum(0)
    gg = g * gamma.float()
    dx = rstd[:, None] * (gg - gg.mean(1, keepdim=True) - xhat * (gg * xhat).mean(1, keepdim=True))
    return dx.reshape(x.shape).to(x.dtype), dg, db
