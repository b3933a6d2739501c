"""Row LayerNorm forward/backward (``layernorm.hip``): one wave per row, fp32
statistics, fused dx/dgamma/dbeta (two-stage column reduction for the
parameter gradients).  Replaces LayerNorm.cu (fwd block-per-row with
E[x^2]-E[x]^2 variance, bwd = 3 elementwise kernels + 4 cuDNN reductions)."""
from __future__ import annotations

import os

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32, F32



# LayerNorm backward blocks (4 waves, a wave per row): more blocks keep more rows in
# flight, fewer write fewer dgamma / dbeta partial rows (HETU_LN_BWD_BLOCKS)
_LN_BWD_BLOCKS = int(os.environ.get('HETU_LN_BWD_BLOCKS', '512'))
# waves (rows in flight) per LayerNorm-backward block (HETU_LN_BWD_WAVES, 4 or 8): 8 waves
# measured slower in the BERT step (29.3 vs 24.3 us per call at 8192 x 768, profiles/
# bert_steady_r5d.txt vs bert_steady_r5.txt), so 4 stays the default
_LN_BWD_WAVES = int(os.environ.get('HETU_LN_BWD_WAVES', '4'))

def layer_norm(x, gamma, beta, eps):
    N = x.shape[-1]
    R = x.numel() // N
    if _fused_ok(x):
        y, _, mean, rstd = layer_norm_fused(x, None, gamma, beta, eps)
        return y, mean, rstd
    if native(x) and supported_float(x):
        xc = x.contiguous()
        y = _NA.empty_like(xc)
        mean = _NA.empty(R, dtype=torch.float32, device=x.device)
        rstd = _NA.empty(R, dtype=torch.float32, device=x.device)
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


def _dest(out, N, dev):
    """fp32 [N] result buffer: the caller's (e.g. the optimizer's flat gradient slot) or new"""
    if out is not None and out.dtype == torch.float32 and out.is_contiguous() and out.numel() == N:
        return out
    return _NA.empty(N, dtype=torch.float32, device=dev)


def layer_norm_backward(dy, x, gamma, mean, rstd, dg_out=None, db_out=None):
    """(dx, dgamma, dbeta); ``dg_out`` / ``db_out``: fp32 buffers that receive
    dgamma / dbeta (the optimizer's flat gradient slots)."""
    N = x.shape[-1]
    R = x.numel() // N
    if _fused_ok(x) and dy.dtype == x.dtype:
        ds, _, dg, db = layer_norm_fused_backward(dy, x, gamma, mean, rstd, need_dx=False,
                                                  dg_out=dg_out, db_out=db_out)
        return ds, dg, db
    if native(x) and supported_float(x) and dy.dtype == x.dtype:
        xc, dyc = x.contiguous(), dy.contiguous()
        dx = _NA.empty_like(xc)
        ws_rows = min(R, 1024)
        ws = _NA.empty(2 * ws_rows * N, dtype=torch.float32, device=x.device)
        dg, db = _dest(dg_out, N, x.device), _dest(db_out, N, x.device)
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


def _fused_ok(x):
    N = x.shape[-1]
    return native(x) and supported_float(x) and N % 4 == 0 and N <= 2048


def layer_norm_fused(x, residual, gamma, beta, eps, keep=1.0, seed=0):
    """y = LN(dropout(x; keep, seed) + residual) in one pass (``residual`` may be
    None, ``keep`` 1 disables dropout).  Returns (y, s, mean, rstd) where ``s``
    is the normalised input (needed by the backward; ``x`` itself when there is
    neither residual nor dropout)."""
    N = x.shape[-1]
    R = x.numel() // N
    plain = residual is None and keep >= 1.0
    if _fused_ok(x) and (residual is None or residual.dtype == x.dtype):
        xc = x.contiguous()
        rc = residual.contiguous() if residual is not None else None
        y = _NA.empty_like(xc)
        s = xc if plain else _NA.empty_like(xc)
        mean = _NA.empty(R, dtype=torch.float32, device=x.device)
        rstd = _NA.empty(R, dtype=torch.float32, device=x.device)
        f = fn('hetu_ln_fused_fwd', [P, P, P, P, P, P, P, P, I64, I32, F32, F32, I64, I32, P])
        check(f(xc.data_ptr(), rc.data_ptr() if rc is not None else None, gamma.float().contiguous().data_ptr(),
                beta.float().contiguous().data_ptr(), y.data_ptr(), None if plain else s.data_ptr(),
                mean.data_ptr(), rstd.data_ptr(), R, N, float(eps), float(keep), int(seed), is_bf16(x),
                stream_ptr()), 'ln_fused_fwd')
        return y, s, mean, rstd
    from . import dropout as KD
    s = x if keep >= 1.0 else KD.dropout(x, keep, seed)
    if residual is not None:
        s = (s.float() + residual.float()).to(x.dtype)
    y, mean, rstd = layer_norm(s, gamma, beta, eps)
    return y, s, mean, rstd


def layer_norm_fused_backward(dy, s, gamma, mean, rstd, keep=1.0, seed=0, need_ds=True, need_dx=True,
                              dg_out=None, db_out=None, want_dlin=False, dlin_out=None):
    """Backward of ``layer_norm_fused``: (ds, dx, dgamma, dbeta) with ds the grad
    of the normalised input (= grad of the residual) and dx = dropout-mask(ds)
    the grad of ``x`` (None when not requested).  ``want_dlin`` appends the
    column sums of dx over all rows -- the bias gradient of the linear layer that
    produced x -- computed in the same row pass (into ``dlin_out`` when given)."""
    N = s.shape[-1]
    R = s.numel() // N
    if _fused_ok(s) and dy.dtype == s.dtype:
        dyc, sc = dy.contiguous(), s.contiguous()
        ds = _NA.empty_like(sc) if need_ds else None
        dx = _NA.empty_like(sc) if (need_dx and keep < 1.0) else None
        if need_dx and keep >= 1.0 and not need_ds:
            ds = _NA.empty_like(sc)
        nblk = max(1, min(_LN_BWD_BLOCKS, (R + 7) // 8))
        ws = _NA.empty((3 if want_dlin else 2) * nblk * N, dtype=torch.float32, device=s.device)
        dg, db = _dest(dg_out, N, s.device), _dest(db_out, N, s.device)
        dlin = _dest(dlin_out, N, s.device) if want_dlin else None
        from . import deterministic
        f = fn('hetu_ln_fused_bwd3', [P, P, P, P, P, P, P, P, P, P, P, I64, I32, I32, F32, I64, I32, I32, I32, P])
        check(f(dyc.data_ptr(), sc.data_ptr(), gamma.float().contiguous().data_ptr(), mean.data_ptr(),
                rstd.data_ptr(), ds.data_ptr() if ds is not None else None,
                dx.data_ptr() if dx is not None else None, dg.data_ptr(), db.data_ptr(),
                dlin.data_ptr() if dlin is not None else None, ws.data_ptr(), R, N, nblk,
                float(keep), int(seed), is_bf16(s), int(deterministic()), _LN_BWD_WAVES, stream_ptr()), 'ln_fused_bwd')
        if need_dx and keep >= 1.0:
            dx = ds
        return (ds, dx, dg, db, dlin) if want_dlin else (ds, dx, dg, db)
    ds, dg, db = layer_norm_backward(dy, s, gamma, mean, rstd)
    dx = None
    if need_dx or want_dlin:
        from . import dropout as KD
        dx = ds if keep >= 1.0 else KD.dropout(ds, keep, seed)
    if want_dlin:
        dlin = dx.reshape(-1, N).float().sum(0)
        if dlin_out is not None:
            dlin_out.view(-1).copy_(dlin)
            dlin = dlin_out
        return ds, dx, dg, db, dlin
    return ds, dx, dg, db


def gelu_grad_colsum(pre, dy, out=None):
    """(g, colsum) with g = dy * gelu'(pre) (erf form) and colsum = g summed over
    rows -- the transformer FFN1 bias gradient -- from one pass over pre and dy
    (``hetu_gelu_grad_colsum``).  ``out``: fp32 [N] destination (e.g. the
    optimizer's flat gradient slot).  2-D inputs; other layouts take the generic
    elementwise kernel + reduction."""
    N = pre.shape[-1]
    dt = pre.dtype
    V = 8 if dt == torch.bfloat16 else 4
    if not (pre.is_cuda and pre.dim() == 2 and dy.dtype == dt and dt in (torch.bfloat16, torch.float32)
            and N % V == 0):
        from .elementwise import binary
        from . import reduce as KR
        g = binary('gelu_grad', pre.contiguous(), dy.contiguous())
        cs = KR.reduce_mid(g.reshape(1, g.shape[0], -1)).reshape(g.shape[1:])
        if out is not None and out.numel() == cs.numel():
            out.view(cs.shape).copy_(cs)
            cs = out.view(cs.shape)
        return g, cs
    pre, dy = pre.contiguous(), dy.contiguous()
    R = pre.shape[0]
    g = _NA.empty_like(pre)
    cv = N // V
    W = min(cv, 64)
    RP = 256 // W
    tiles = -(-cv // W)
    chunks = max(1, min(max(1, 2048 // tiles), R // (RP * 4)))   # ~2048 blocks: 8 waves per CU
    ws = _NA.empty(chunks * N, dtype=torch.float32, device=pre.device)
    cs = _dest(out, N, pre.device)
    from . import deterministic
    f = fn('hetu_gelu_grad_colsum', [P, P, P, P, P, I64, I32, I32, I32, I32, P])
    check(f(pre.data_ptr(), dy.data_ptr(), g.data_ptr(), cs.data_ptr(), ws.data_ptr(), R, N, chunks,
            is_bf16(pre), int(deterministic()), stream_ptr()), 'gelu_grad_colsum')
    return g, cs
