"""BatchNorm (channels-last, fused ReLU / residual) bindings (``batchnorm.hip``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, P, I64, I32, F32


_TUNED = [False]


def _tune_once():
    """HETU_BN_TUNE=chunks,apply_blocks,min_passes (0 keeps a default): the BatchNorm
    kernels' launch shapes (hetu_bn_tune; scripts/bench_bn.py sweeps them)"""
    if _TUNED[0]:
        return
    _TUNED[0] = True
    import os
    v = os.environ.get('HETU_BN_TUNE')
    if v:
        a = [int(t) for t in v.split(',')] + [0, 0, 0]
        fn('hetu_bn_tune', [I32, I32, I32], restype=None)(a[0], a[1], a[2])


def _as_rows(x):
    """View x as [M, C] channels-last rows; returns (rows, restore_fn) or None."""
    if x.dim() == 2:
        if x.is_contiguous():
            return x, x.shape
        return None
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = x.shape
        return x.permute(0, 2, 3, 1).reshape(n * h * w, c), x.shape
    return None


def _like_rows(x):
    if x.dim() == 4:
        return _NA.empty_like(x, memory_format=torch.channels_last)
    return _NA.empty_like(x)


def _ws(M, C, bf, device):
    _tune_once()
    f = fn('hetu_bn_workspace_floats', [I64, I32, I32], restype=I64)
    n = f(M, C, bf)
    return _NA.empty(n, dtype=torch.float32, device=device)


def col_sums(x):
    """[2, C] fp32: per-channel sum and sum of squares of a channels-last activation
    (the BatchNorm statistics inputs), or None where the native path does not apply."""
    rows = _as_rows(x) if native(x) and x.dtype in (torch.float32, torch.bfloat16) else None
    C = x.shape[1]
    if rows is None or C % (8 if x.dtype == torch.bfloat16 else 4):
        return None
    xr, _ = rows
    M = xr.shape[0]
    sums = _NA.empty(2 * C, dtype=torch.float32, device=x.device)
    ws = _ws(M, C, is_bf16(x), x.device)
    f = fn('hetu_col_sums', [P, I64, I32, I32, P, P, P])
    check(f(xr.data_ptr(), M, C, is_bf16(x), ws.data_ptr(), sums.data_ptr(), stream_ptr()), 'col_sums')
    return sums


def relu_mask_bytes(x):
    """Size of the ReLU keep-bit mask ``bn_forward(mask=...)`` writes: one byte per
    16-byte vector of x (8 bf16 / 4 fp32 channels)."""
    return x.numel() // (8 if x.dtype == torch.bfloat16 else 4)


def bn_forward(x, scale, bias, running_mean, running_var, factor, eps, training,
               relu=False, residual=None, sums=None, mask=None):
    """Returns (y, save_mean, save_invstd).  ``factor`` = weight of the new batch
    statistics in the running average.  ``sums`` ([2C] fp32 per-channel sum and sum
    of squares of x, e.g. from the convolution epilogue that produced x) skips the
    statistics pass.  ``mask`` (uint8 [relu_mask_bytes(x)], ReLU only): receives the
    ReLU keep-bits, which ``bn_backward(mask=...)`` reads instead of y."""
    C = x.shape[1]
    if native(x) and x.dtype in (torch.float32, torch.bfloat16):
        if x.dim() == 4 and not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        if residual is not None and residual.dim() == 4:
            residual = residual.contiguous(memory_format=torch.channels_last)
        rows = _as_rows(x)
        vec = 8 if x.dtype == torch.bfloat16 else 4
        if rows is not None and C % vec == 0:
            xr, _ = rows
            M = xr.shape[0]
            y = _like_rows(x)
            save_mean = _NA.empty(C, dtype=torch.float32, device=x.device)
            save_invstd = _NA.empty(C, dtype=torch.float32, device=x.device)
            ws = _ws(M, C, is_bf16(x), x.device)
            if mask is not None:
                assert relu and mask.dtype == torch.uint8 and mask.numel() == relu_mask_bytes(x) and mask.is_cuda
            f = fn('hetu_bn_fwd', [P, P, P, I64, I32, I32, P, P, P, P, F32, F32, P, P, P, I32, I32, P, P, I32, P])
            check(f(x.data_ptr(), residual.data_ptr() if residual is not None else None, y.data_ptr(),
                    M, C, is_bf16(x), scale.data_ptr(), bias.data_ptr(),
                    running_mean.data_ptr() if running_mean is not None else None,
                    running_var.data_ptr() if running_var is not None else None,
                    float(factor), float(eps), save_mean.data_ptr(), save_invstd.data_ptr(),
                    ws.data_ptr(), int(relu), int(training),
                    sums.data_ptr() if (sums is not None and training) else None,
                    mask.data_ptr() if mask is not None else None,
                    sums.numel() // (2 * C) if sums is not None else 1, stream_ptr()), 'bn_fwd')
            return y, save_mean, save_invstd
    if sums is not None:
        sums.zero_()     # not consumed here: leave the (persistent) totals ready for next time
    from . import cpu_native
    if (x.dim() == 4 and cpu_native.active(x, scale, bias, running_mean, running_var)
            and (training or running_mean is not None)):
        y, mean, invstd = cpu_native.batchnorm(x, scale, bias, running_mean, running_var, factor, eps, training)
        if residual is not None:
            y = y + residual.float()
        if relu:
            y = cpu_native.unary('relu', y)
        return y, mean, invstd
    # torch reference (CPU backend / unsupported layouts)
    xf = x.float()
    dims = [0] + list(range(2, x.dim()))
    shape = [1, C] + [1] * (x.dim() - 2)
    if training:
        mean = xf.mean(dims)
        var = xf.var(dims, unbiased=False)
        if running_mean is not None:
            n = x.numel() // C
            unb = var * n / max(n - 1, 1)
            running_mean.mul_(1 - factor).add_(factor * mean)
            running_var.mul_(1 - factor).add_(factor * unb)
    else:
        mean, var = running_mean, running_var
    invstd = torch.rsqrt(var + eps)
    y = (xf - mean.view(shape)) * (invstd * scale.float()).view(shape) + bias.float().view(shape)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    return y, mean.float(), invstd.float()


def bn_bwd_sums(dy, x, mask, sums):
    """sums[:C] += sum(dy'), sums[C:] += sum(dy' * x) per channel (dy' = dy masked by the
    ReLU keep-bits ``mask``, or dy): the reduction a data-gradient epilogue fuses, as a
    pass of its own.  bf16 channels-last dy / x."""
    rows = _as_rows(x)
    C = x.shape[1]
    M = x.numel() // C
    dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
    ws = _ws(M, C, 1, x.device)
    f = fn('hetu_bn_bwd_sums', [P, P, P, I64, I32, P, P, P])
    check(f(dy.data_ptr(), rows[0].data_ptr(), mask.data_ptr() if mask is not None else None, M, C,
            ws.data_ptr(), sums.data_ptr(), stream_ptr()), 'bn_bwd_sums')
    return sums


def bn_backward(dy, y, x, scale, save_mean, save_invstd, relu=False, want_dres=False, bias=None,
                dscale_out=None, dbias_out=None, mask=None, bsums=None, bsums_next=None):
    """Returns (dx, dscale, dbias, dres).  ``mask``: the forward's ReLU keep-bits
    (native path only; y is then not read).  ``bsums``: [2C] totals sum(dy') and
    sum(dy' * x) already accumulated (the producing data-gradient epilogue), or [R * 2C]
    replicas of them folded here; the reduction pass is skipped and the totals are zeroed
    for their next use.
    ``bsums_next``: the other half of double-buffered totals -- the apply kernel folds the
    coefficients itself (no finalize launch) and zeroes ``bsums_next`` instead."""
    C = x.shape[1]
    if native(x) and x.dtype in (torch.float32, torch.bfloat16):
        cl = torch.channels_last
        if x.dim() == 4:
            x = x.contiguous(memory_format=cl)
            dy = dy.contiguous(memory_format=cl)
            if relu and mask is None:
                y = y.contiguous(memory_format=cl)
        else:
            dy = dy.contiguous()
        vec = 8 if x.dtype == torch.bfloat16 else 4
        if C % vec == 0 and dy.dtype == x.dtype:
            M = x.numel() // C
            dx = _like_rows(x)
            dres = _like_rows(x) if want_dres else None
            dscale = dscale_out if dscale_out is not None else _NA.empty(C, dtype=torch.float32, device=x.device)
            dbias = dbias_out if dbias_out is not None else _NA.empty(C, dtype=torch.float32, device=x.device)
            ws = _ws(M, C, is_bf16(x), x.device)
            if mask is not None:
                assert relu and mask.dtype == torch.uint8 and mask.numel() == relu_mask_bytes(x)
            f = fn('hetu_bn_bwd', [P, P, P, P, P, I64, I32, I32, P, P, P, P, P, P, P, I32, P, P, P, I32, P])
            check(f(dy.data_ptr(), y.data_ptr() if (relu and mask is None) else None, x.data_ptr(),
                    dx.data_ptr(), dres.data_ptr() if dres is not None else None, M, C, is_bf16(x),
                    scale.data_ptr(), bias.float().contiguous().data_ptr() if bias is not None else None,
                    save_mean.data_ptr(), save_invstd.data_ptr(),
                    dscale.data_ptr(), dbias.data_ptr(), ws.data_ptr(), int(relu),
                    mask.data_ptr() if mask is not None else None,
                    bsums.data_ptr() if bsums is not None else None,
                    bsums_next.data_ptr() if (bsums is not None and bsums_next is not None) else None,
                    bsums.numel() // (2 * C) if bsums is not None else 1,
                    stream_ptr()),
                  'bn_bwd')
            return dx, dscale, dbias, dres
    if bsums is not None:
        bsums.zero_()
        if bsums_next is not None:
            bsums_next.zero_()
    from . import cpu_native
    if x.dim() == 4 and cpu_native.active(dy, x, scale, save_mean, save_invstd) and (not relu or y is not None):
        g = cpu_native.relu_grad(y.float().contiguous(), dy.float().contiguous()) if relu else dy.float()
        dx, dscale, dbias = cpu_native.batchnorm_backward(g, x, scale, save_mean, save_invstd)
        return dx, dscale, dbias, (g.clone() if want_dres else None)
    dims = [0] + list(range(2, x.dim()))
    shape = [1, C] + [1] * (x.dim() - 2)
    g = dy.float()
    if relu:
        g = torch.where(y > 0, g, _NA.zeros_like(g))
    xhat = (x.float() - save_mean.view(shape)) * save_invstd.view(shape)
    M = x.numel() // C
    dbias = g.sum(dims)
    dscale = (g * xhat).sum(dims)
    dx = (scale.float() * save_invstd).view(shape) * (g - dbias.view(shape) / M - xhat * dscale.view(shape) / M)
    dres = g.to(x.dtype, copy=True) if want_dres else None   # never an alias of dy
    dx = dx.to(x.dtype)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        dx = dx.contiguous(memory_format=torch.channels_last)
        if dres is not None:
            dres = dres.contiguous(memory_format=torch.channels_last)
    return dx, dscale, dbias, dres


def layer_norm_ref(x, gamma, beta, eps):
    return F.layer_norm(x.float(), x.shape[-1:], gamma.float() if gamma is not None else None,
                        beta.float() if beta is not None else None, eps).to(x.dtype)
