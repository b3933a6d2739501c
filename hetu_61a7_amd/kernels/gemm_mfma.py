"""Bindings of the hand-written bf16 MFMA GEMM (``csrc/kernels/gemm.hip``).

Every transpose mode is handled in-kernel (K-contiguous operands are read
row-wise from LDS, MN-contiguous ones through the hardware transpose read), so
a transposed view never costs a copy.  Shapes whose contiguous extent or
leading dimension is not a multiple of 8 elements return ``None`` and the
caller uses the library GEMM.
"""
from __future__ import annotations

import os

import torch
from .. import native_array as _NA

from . import fn, stream_ptr, check, record_native, P, I64, I32, F32

_ACT = {None: 0, 'relu': 1, 'gelu': 2}
_ARGS = [P, P, P, P, P, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I64, I64, I64, I64,
         F32, F32, I32, I32, I32, I32, I32, I32, P, I32, P]
# tile configurations of the kernel (gemm.hip launch): 0 = 128x128 tile, 4 waves;
# 1 = 256x256 tile, 8 waves, phase-interleaved K loop (one block per CU)
TILES = (0, 1, 2, 3, 5, 6, 7)   # 128x128, 256x256, 128x64, 128x128 single-stage (4 blocks / CU), 128x96,
#                               and 128x128 / 128x96 with the two-ahead K loop (plain GEMMs)


def _operand(t, rows_dim_last, q=8):
    """Describe a 2-D (or batched 3-D) operand view.  ``t`` is viewed as
    [..., R, K] (rows first) -> returns (kmaj, ld, batch_stride) or None.
    ``q``: elements per 16-byte staging chunk (8 bf16, 4 fp32) -- the contiguous
    extent and the leading dimension must be multiples of it."""
    sr, sk = t.stride(-2), t.stride(-1)
    R, K = t.shape[-2], t.shape[-1]
    bs = t.stride(0) if t.dim() == 3 else 0
    if sk == 1 or K == 1:
        ld = sr if R > 1 else max(K, q)
        if K % q or ld % q:
            return None
        return True, ld, bs
    if sr == 1 or R == 1:
        ld = sk if K > 1 else max(R, q)
        if R % q or ld % q:
            return None
        return False, ld, bs
    return None


def _dense_f32(t):
    """t as a contiguous fp32 tensor (native cast / strided copy on the GPU; no copy if already)"""
    if t.dtype == torch.float32 and t.is_contiguous():
        return t
    if not t.is_cuda:
        return t.float().contiguous()
    from .tensor import copy_into
    return copy_into(_NA.empty(tuple(t.shape), dtype=torch.float32, device=t.device), t)


def _aligned(*ts):
    return all(t.data_ptr() % 16 == 0 for t in ts)


_F32_ARGS = [P, P, P, P, P, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I64, I64, I64, I64,
             F32, F32, I32, I32, I32, P]


def gemm_f32(a, b, out=None, bias=None, act=None, alpha=1.0, beta=0.0, cin=None, accumulate=False,
             bias_on_m=False):
    """fp32 product on the exact-fp32 MFMA kernel (``gemm_f32.hip``, 16x16x4 f32):
    the parity-mode GEMM.  Same view rules as :func:`gemm` with 4-element chunks."""
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() != b.dim() or a.dim() not in (2, 3):
        return None
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if b.shape[-2] != K:
        raise ValueError('gemm shape mismatch %s @ %s' % (tuple(a.shape), tuple(b.shape)))
    batch = a.shape[0] if a.dim() == 3 else 1
    if a.dim() == 3 and b.shape[0] != batch:
        return None
    da = _operand(a, False, 4)
    db = _operand(b.transpose(-1, -2), False, 4)
    if da is None or db is None or not _aligned(a, b):
        return None
    if out is None:
        shape = (batch, M, N) if a.dim() == 3 else (M, N)
        if accumulate:
            from .tensor import zeros
            out = zeros(shape, torch.float32, a.device)
        else:
            out = _NA.empty(shape, dtype=torch.float32, device=a.device)
    if out.dtype != torch.float32 or out.stride(-1) != 1 or (out.dim() == 3 and out.dim() != a.dim()):
        return None
    ldc = out.stride(-2) if M > 1 else N
    sC = out.stride(0) if out.dim() == 3 else 0
    cin_t, ldcin, sCin = None, 0, 0
    if cin is not None and beta != 0.0:
        cin_t = cin.expand_as(out) if cin.shape != out.shape else cin
        if cin_t.dtype != torch.float32 or cin_t.stride(-1) != 1:
            cin_t = _dense_f32(cin_t)
        ldcin = cin_t.stride(-2)
        sCin = cin_t.stride(0) if cin_t.dim() == 3 else 0
    bias_t = _dense_f32(bias) if bias is not None else None
    f = fn('hetu_gemm_f32', _F32_ARGS)
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), cin_t.data_ptr() if cin_t is not None else None,
            bias_t.data_ptr() if bias_t is not None else None, M, N, K, da[1], db[1], ldc, ldcin,
            int(da[0]), int(db[0]), batch, da[2], db[2], sC, sCin, float(alpha), float(beta), _ACT[act],
            int(bias_on_m), int(accumulate), stream_ptr()), 'gemm_f32')
    record_native('gemm_f32')
    return out


_DEBUG = os.environ.get('HETU_GEMM_DEBUG') == '1'


def _reject(where, a, b, out):
    """None (unsupported operands); HETU_GEMM_DEBUG=1 names the check that refused them"""
    if _DEBUG:
        import sys
        print('gemm_mfma.gemm: refused at check %d: a %s %s %s ptr%%16=%d, b %s %s %s ptr%%16=%d, out %s' % (
            where, tuple(a.shape), tuple(a.stride()), a.dtype, a.data_ptr() % 16, tuple(b.shape), tuple(b.stride()),
            b.dtype, b.data_ptr() % 16, None if out is None else (tuple(out.shape), tuple(out.stride()), out.dtype)),
            file=sys.stderr)
    return None


def gemm(a, b, out=None, bias=None, act=None, alpha=1.0, beta=0.0, cin=None, out_dtype=None,
         accumulate=False, splitk=1, bias_on_m=False, tile=0, pre_out=None, drop=None):
    """out[M,N] = alpha * a[M,K] @ b[K,N] (+beta*cin) (+bias) -> act, a/b arbitrary
    strided views (batched 3-D allowed).  Returns None if unsupported.
    ``pre_out``: also store the pre-activation (bias added) there -- bf16, out's shape and
    layout -- from the same epilogue (a training GELU layer's saved input)."""
    if pre_out is not None or drop is not None:
        keep, seed = drop if drop is not None else (1.0, 0)
        if pre_out is not None and keep < 1.0:
            return None          # one epilogue extension per kernel build (gemm_core.h EX)
        return _gemm_ex(a, b, pre_out, bias, act, tile, out, keep, seed)
    if a.dtype == torch.float32 and b.dtype == torch.float32 and (out is None or out.dtype == torch.float32) \
            and splitk == 1:
        return gemm_f32(a, b, out=out, bias=bias, act=act, alpha=alpha, beta=beta, cin=cin,
                        accumulate=accumulate, bias_on_m=bias_on_m)
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return _reject(1, a, b, out)
    if a.dim() != b.dim() or a.dim() not in (2, 3):
        return _reject(2, a, b, out)
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if b.shape[-2] != K:
        raise ValueError('gemm shape mismatch %s @ %s' % (tuple(a.shape), tuple(b.shape)))
    batch = a.shape[0] if a.dim() == 3 else 1
    if a.dim() == 3 and b.shape[0] != batch:
        return _reject(3, a, b, out)
    da = _operand(a, False)
    db = _operand(b.transpose(-1, -2), False)  # view as [N, K]
    if da is None or db is None or not _aligned(a, b):
        return _reject(4, a, b, out)
    odt = out_dtype or (out.dtype if out is not None else torch.bfloat16)
    if out is None:
        shape = (batch, M, N) if a.dim() == 3 else (M, N)
        if accumulate:
            from .tensor import zeros
            out = zeros(shape, odt, a.device)
        else:
            out = _NA.empty(shape, dtype=odt, device=a.device)
    if out.stride(-1) != 1 or (out.dim() == 3 and out.dim() != a.dim()):
        return _reject(5, a, b, out)
    if accumulate and splitk == 1 and out.dtype != torch.float32:
        return _reject(6, a, b, out)
    ldc = out.stride(-2) if M > 1 else N
    sC = out.stride(0) if out.dim() == 3 else 0
    cin_t, ldcin, sCin = None, 0, 0
    if cin is not None and beta != 0.0:
        cin_t = cin.expand_as(out) if cin.shape != out.shape else cin
        if cin_t.stride(-1) != 1:
            cin_t = cin_t.contiguous()
        ldcin = cin_t.stride(-2)
        sCin = cin_t.stride(0) if cin_t.dim() == 3 else 0
    bias_t = _dense_f32(bias) if bias is not None else None
    ws = None
    if splitk > 1:
        if bias is not None or act is not None or cin_t is not None:
            return _reject(7, a, b, out)
        ws = _NA.empty(splitk * batch * M * N, dtype=torch.float32, device=a.device)
        if batch > 1:
            return _reject(8, a, b, out)
    f = fn('hetu_gemm_bf16', _ARGS)
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), cin_t.data_ptr() if cin_t is not None else None,
            bias_t.data_ptr() if bias_t is not None else None, M, N, K, da[1], db[1], ldc, ldcin,
            int(da[0]), int(db[0]), batch, da[2], db[2], sC, sCin, float(alpha), float(beta),
            _ACT[act], int(out.dtype == torch.float32),
            int(cin_t is not None and cin_t.dtype == torch.float32), int(bias_on_m), int(splitk),
            int(accumulate), ws.data_ptr() if ws is not None else None, int(tile), stream_ptr()),
          'gemm_bf16')
    record_native('gemm_bf16')
    return out


def _gemm_ex(a, b, pre, bias, act, tile, out, keep=1.0, seed=0):
    """bf16 out = dropout(act(a @ b + bias)) and (``pre``, nullable) pre = a @ b + bias in one
    epilogue (2-D / batched; dropout: 2-D, N % 8 == 0, the standalone dropout's counters)"""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != b.dim() or a.dim() not in (2, 3):
        return _reject(11, a, b, out)
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    batch = a.shape[0] if a.dim() == 3 else 1
    da = _operand(a, False)
    db = _operand(b.transpose(-1, -2), False)
    if da is None or db is None or not _aligned(a, b):
        return _reject(12, a, b, out)
    shape = (batch, M, N) if a.dim() == 3 else (M, N)
    if out is None:
        out = _NA.empty(shape, dtype=torch.bfloat16, device=a.device)
    if out.dtype != torch.bfloat16 or tuple(out.shape) != shape or out.stride(-1) != 1:
        return _reject(13, a, b, out)
    if pre is not None and (pre.dtype != torch.bfloat16 or tuple(pre.shape) != shape or out.stride() != pre.stride()):
        return _reject(14, a, b, out)
    if keep < 1.0 and (batch != 1 or N % 8):
        return _reject(15, a, b, out)
    ldc = out.stride(-2) if M > 1 else N
    sC = out.stride(0) if out.dim() == 3 else 0
    bias_t = _dense_f32(bias) if bias is not None else None
    f = fn('hetu_gemm_bf16_ex', [P, P, P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, I32, I64, I64, I64,
                                 I32, I32, F32, I64, P])
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), pre.data_ptr() if pre is not None else None,
            bias_t.data_ptr() if bias_t is not None else None, M, N, K, da[1], db[1], ldc, int(da[0]), int(db[0]),
            batch, da[2], db[2], sC, _ACT[act], int(tile), float(keep), int(seed), stream_ptr()), 'gemm_bf16_ex')
    record_native('gemm_bf16')
    return out


def gemm_gmask(a, b, g, scale, tile=0, out=None):
    """bf16 out = (a @ b) * scale where g > 0, else 0 (2-D; g bf16 of the output's shape,
    contiguous): the data gradient of a ReLU (+ dropout) output g computed and masked in one
    GEMM epilogue.  None when unsupported."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        return _reject(21, a, b, out)
    M, K = a.shape
    N = b.shape[1]
    da = _operand(a, False)
    db = _operand(b.t(), False)
    if da is None or db is None or not _aligned(a, b):
        return _reject(22, a, b, out)
    if g.dtype != torch.bfloat16 or tuple(g.shape) != (M, N) or not g.is_contiguous() or g.data_ptr() % 16:
        return _reject(23, a, b, out)
    if out is None:
        out = _NA.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if out.dtype != torch.bfloat16 or tuple(out.shape) != (M, N) or not out.is_contiguous():
        return _reject(24, a, b, out)
    f = fn('hetu_gemm_bf16_gmask', [P, P, P, P, F32, I64, I64, I64, I64, I64, I64, I32, I32, I32, P])
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), g.data_ptr(), float(scale), M, N, K, da[1], db[1], N,
            int(da[0]), int(db[0]), int(tile), stream_ptr()), 'gemm_bf16_gmask')
    record_native('gemm_bf16')
    return out


def gemm_drop_bits(a, b, act, keep, seed, tile=0):
    """(out, bits): bf16 out = dropout(act(a @ b)) as ``_gemm_ex`` (2-D, N % 8 == 0) and the
    keep bits of out (uint8, one byte per 8 elements of a row, bit t set where out > 0) from
    the same epilogue -- the mask ``gemm_gbits`` reads in the backward.  None when unsupported."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2 or not keep < 1.0:
        return _reject(25, a, b, None)
    M, K = a.shape
    N = b.shape[1]
    da = _operand(a, False)
    db = _operand(b.t(), False)
    if da is None or db is None or not _aligned(a, b) or N % 8:
        return _reject(26, a, b, None)
    out = _NA.empty((M, N), dtype=torch.bfloat16, device=a.device)
    bits = _NA.empty((M * N // 8,), dtype=torch.uint8, device=a.device)
    f = fn('hetu_gemm_bf16_drop_bits', [P, P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32, F32, I64, P])
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), bits.data_ptr(), M, N, K, da[1], db[1], N, int(da[0]),
            int(db[0]), _ACT[act], int(tile), float(keep), int(seed), stream_ptr()), 'gemm_bf16_drop_bits')
    record_native('gemm_bf16')
    return out, bits


def gemm_gbits(a, b, bits, scale, tile=0):
    """bf16 out = (a @ b) * scale where the keep bit is set, else 0 (2-D; ``bits`` from
    ``gemm_drop_bits`` over an output of this shape): ``gemm_gmask`` reading 1/16 of the
    bytes.  None when unsupported."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        return _reject(27, a, b, None)
    M, K = a.shape
    N = b.shape[1]
    da = _operand(a, False)
    db = _operand(b.t(), False)
    if da is None or db is None or not _aligned(a, b):
        return _reject(28, a, b, None)
    if N % 8 or bits.dtype != torch.uint8 or bits.numel() != M * N // 8 or not bits.is_contiguous():
        return _reject(29, a, b, None)
    out = _NA.empty((M, N), dtype=torch.bfloat16, device=a.device)
    f = fn('hetu_gemm_bf16_gbits', [P, P, P, P, F32, I64, I64, I64, I64, I64, I64, I32, I32, I32, P])
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), bits.data_ptr(), float(scale), M, N, K, da[1], db[1], N,
            int(da[0]), int(db[0]), int(tile), stream_ptr()), 'gemm_bf16_gbits')
    record_native('gemm_bf16')
    return out


SMALL_MAX_OUT = 1 << 16


def wgrad_longk(a_pm, b_pm, out, accumulate=False, splits=None):
    """out[M,N] (fp32, row stride multiple of 4) (+)= a_pm^T @ b_pm for pixel-major bf16
    operands a_pm [P, M], b_pm [P, N] (rows contiguous, M and N multiples of 64): the
    64x64-tile split-K kernel for small outputs over very long reductions
    (``wgrad_longk.hip``).  None when unsupported."""
    if a_pm.dtype != torch.bfloat16 or b_pm.dtype != torch.bfloat16 or a_pm.dim() != 2 or b_pm.dim() != 2:
        return None
    P_, M = a_pm.shape
    N = b_pm.shape[1]
    if b_pm.shape[0] != P_ or M % 64 or N % 64 or a_pm.stride(1) != 1 or b_pm.stride(1) != 1:
        return None
    lda, ldb = (a_pm.stride(0) if P_ > 1 else M), (b_pm.stride(0) if P_ > 1 else N)
    if lda % 8 or ldb % 8 or not _aligned(a_pm, b_pm) or out.dtype != torch.float32 or out.stride(-1) != 1 \
            or tuple(out.shape) != (M, N) or out.data_ptr() % 16 or (M > 1 and out.stride(0) % 4):
        return None
    tiles = (M // 64) * (N // 64)
    if splits is None:
        splits = max(1, min(2048 // tiles, -(-P_ // 512)))
    ws = _NA.empty(int(fn('hetu_wgrad_longk_ws', [I32, I32, I32], restype=I64)(M, N, splits)),
                     dtype=torch.float32, device=a_pm.device)
    f = fn('hetu_wgrad_longk', [P, P, P, P, I64, I32, I32, I32, I32, I64, I32, I32, P])
    check(f(a_pm.data_ptr(), b_pm.data_ptr(), out.data_ptr(), ws.data_ptr(), P_, M, N, lda, ldb,
            out.stride(0) if M > 1 else N, int(splits), int(bool(accumulate)), stream_ptr()), 'wgrad_longk')
    record_native('wgrad_longk')
    return out


def gemm_small(a, b, out=None, bias=None, act=None, alpha=1.0, beta=0.0, cin=None, out_dtype=None, bias_on_m=False):
    """out[M,N] = act(alpha * a @ b + beta * cin + bias) for 2-D fp32 / bf16 views of any
    strides, one wave per output (``gemm_small.hip``): the small / ragged products the
    MFMA tiles cannot take (N = 2 classifier heads, 64-row poolers).  None when unsupported."""
    if a.dim() != 2 or b.dim() != 2 or a.dtype not in (torch.float32, torch.bfloat16) or \
            b.dtype not in (torch.float32, torch.bfloat16) or not a.is_cuda:
        return None
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K or M * N > SMALL_MAX_OUT:
        return None
    odt = out_dtype or (out.dtype if out is not None else a.dtype)
    if out is None:
        out = _NA.empty((M, N), dtype=odt, device=a.device)
    if out.dim() != 2 or out.stride(-1) != 1 or out.dtype not in (torch.float32, torch.bfloat16):
        return None
    cin_t = None
    if cin is not None and beta != 0.0:
        cin_t = cin.expand(M, N) if tuple(cin.shape) != (M, N) else cin
        if cin_t.stride(-1) != 1 or cin_t.dtype not in (torch.float32, torch.bfloat16):
            cin_t = _dense_f32(cin_t)
    bias_t = _dense_f32(bias) if bias is not None else None
    f = fn('hetu_gemm_small', [P, P, P, P, P, I64, I64, I64, I64, I64, I64, I64, I64, I64, I32, I32, F32, F32, I32,
                               I32, I32, I32, P])
    check(f(a.data_ptr(), b.data_ptr(), out.data_ptr(), cin_t.data_ptr() if cin_t is not None else None,
            bias_t.data_ptr() if bias_t is not None else None, M, N, K, a.stride(0), a.stride(1), b.stride(0),
            b.stride(1), out.stride(0) if M > 1 else N, (cin_t.stride(0) if M > 1 else N) if cin_t is not None else 0,
            int(a.dtype == torch.float32), int(b.dtype == torch.float32), float(alpha), float(beta), _ACT[act],
            int(out.dtype == torch.float32), int(cin_t is not None and cin_t.dtype == torch.float32), int(bias_on_m),
            stream_ptr()), 'gemm_small')
    record_native('gemm_small')
    return out


def padded(a, b, out=None, bias=None, act=None, cin=None, beta=0.0):
    """Hand-written product of operands no MFMA tile takes as they are (a contiguous extent
    or leading dimension not a multiple of 16 bytes, a misaligned base, a few output
    columns): zero-padded aligned copies [.., M, Kp] @ [.., Kp, Np] (natively filled and
    copied) on the MFMA tile, the [.., M, N] corner copied into ``out`` (or a new dense
    tensor).  2-D or batched 3-D, bf16 or fp32; ``cin`` (beta = 1) is padded the same way."""
    from .tensor import zeros, copy_into
    if a.dim() != b.dim() or a.dim() not in (2, 3) or a.dtype != b.dtype or \
            a.dtype not in (torch.bfloat16, torch.float32) or not a.is_cuda:
        return None
    q = 8 if a.dtype == torch.bfloat16 else 4
    lead = tuple(a.shape[:-2])
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    Kp, Np = -(-K // q) * q, -(-N // q) * q
    if Kp == K and _operand(a, False, q) is not None and a.data_ptr() % 16 == 0:
        ap = a                      # A already fits a tile: only B / the output are padded
    else:
        ap = zeros(lead + (M, Kp), a.dtype, a.device)
        copy_into(ap[..., :K], a)
    bp = zeros(lead + (Kp, Np), b.dtype, b.device)
    copy_into(bp[..., :K, :N], b)
    bias_p = None
    if bias is not None:
        bias_p = zeros((Np,), torch.float32, a.device)
        copy_into(bias_p[:N], bias.reshape(-1))
    cin_p = None
    if cin is not None and beta != 0.0:
        c = cin.expand(lead + (M, N)) if tuple(cin.shape) != lead + (M, N) else cin
        cin_p = zeros(lead + (M, Np), c.dtype, a.device)
        copy_into(cin_p[..., :N], c)
    odt = out.dtype if out is not None else a.dtype
    op = _NA.empty(lead + (M, Np), dtype=odt, device=a.device)
    if gemm(ap, bp, out=op, bias=bias_p, act=act, cin=cin_p, beta=beta if cin_p is not None else 0.0) is None:
        return None
    if out is None:
        if Np == N:
            return op
        out = _NA.empty(lead + (M, N), dtype=odt, device=a.device)
    copy_into(out, op[..., :N])
    return out


def try_gemm(a, b, ta, tb, bias=None, activation=None):
    A = a.transpose(-1, -2) if ta else a
    B = b.transpose(-1, -2) if tb else b
    return gemm(A, B, bias=bias, act=activation)


def try_bmm(a, b, ta, tb):
    A = a.transpose(-1, -2) if ta else a
    B = b.transpose(-1, -2) if tb else b
    lead = A.shape[:-2]
    if B.shape[:-2] != lead or len(lead) == 0:
        return None
    if len(lead) > 1:
        try:
            A = A.view(-1, *A.shape[-2:])
            B = B.view(-1, *B.shape[-2:])
        except RuntimeError:
            return None
    y = gemm(A, B)
    if y is None:
        return None
    return y.view(*lead, *y.shape[-2:])
