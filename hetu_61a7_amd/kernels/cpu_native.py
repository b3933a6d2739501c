"""Native C++/OpenMP CPU backend (``csrc/cpu/*.cc`` -> ``libhetu_cpu.so``), the
counterpart of the reference's DNNL/OpenMP CPU ops (``src/dnnl_ops``,
``cpu_links/dnnl_op.py``; the reference probes DNNL and uses it whenever it is
available, ``_base.py:15-63``).  It is the default for fp32 CPU tensors;
``HETU_CPU_BACKEND=aten`` selects torch's ATen instead (the test oracle), and
``use(True/False)`` switches it at run time.

An fp32 CPU op that still takes an ATen path while the backend is on is counted in
``FALLBACKS`` (``HETU_STRICT_NATIVE=1`` turns it into an error), so tests can assert
that a CPU step stays native.
"""
from __future__ import annotations

import ctypes
import os

import torch
from .. import native_array as _NA

from .._base import _LIB_DIR

_PATH = os.path.join(_LIB_DIR, 'libhetu_cpu.so')
_lib = None
_enabled = os.environ.get('HETU_CPU_BACKEND', 'native') != 'aten'
P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
FALLBACKS = {}
_STRICT = os.environ.get('HETU_STRICT_NATIVE', '0') == '1'
_ARR = ctypes.c_int64 * 8
UNARY = {'relu': 0, 'sigmoid': 1, 'tanh': 2, 'gelu': 3, 'exp': 4, 'sqrt': 5}
OPT = dict(sgd=0, momentum=1, nesterov=2, adagrad=3, adam=4, adamw=5)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            raise RuntimeError('libhetu_cpu.so not built (%s); run make -C csrc' % _PATH)
        # the library's OpenMP runtime (libgomp) is separate from torch's bundled one; with
        # the default wait policy the two thread pools spin against each other and a
        # logreg step took 125 ms instead of 2.5 ms on 8 cores.  Read at libgomp's load.
        os.environ.setdefault('OMP_WAIT_POLICY', 'PASSIVE')
        L = ctypes.CDLL(_PATH)
        sig = {'hetu_cpu_gemm': [P, P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, F32, F32],
               'hetu_cpu_softmax_ce': [P, P, P, P, I64, I64],
               'hetu_cpu_softmax_ce_bwd': [P, P, P, P, P, I64, I64, I32],
               'hetu_cpu_unary': [I32, P, P, I64], 'hetu_cpu_relu_grad': [P, P, P, I64],
               'hetu_cpu_reduce_rows': [P, P, I64, I64, F32], 'hetu_cpu_gather_rows': [P, P, P, I64, I64, I64],
               'hetu_cpu_optimizer': [I32, P, P, P, P, I64] + [F32] * 10,
               'hetu_cpu_conv2d': [P, P, P, P] + [I64] * 11,
               'hetu_cpu_conv2d_bwd_data': [P, P, P] + [I64] * 11,
               'hetu_cpu_conv2d_bwd_filter': [P, P, P, P] + [I64] * 11,
               'hetu_cpu_maxpool2d': [P, P, P] + [I64] * 11,
               'hetu_cpu_maxpool2d_bwd': [P, P, P] + [I64] * 5,
               'hetu_cpu_avgpool2d': [P, P] + [I64] * 11,
               'hetu_cpu_avgpool2d_bwd': [P, P] + [I64] * 11,
               'hetu_cpu_batchnorm': [P] * 8 + [I64] * 3 + [F32, F32, I32],
               'hetu_cpu_batchnorm_bwd': [P] * 8 + [I64] * 3,
               'hetu_cpu_fill': [P, I64, F32],
               'hetu_cpu_softmax': [P, P, I64, I64, I32], 'hetu_cpu_softmax_bwd': [P, P, P, I64, I64],
               'hetu_cpu_dropout': [P, P, I64, F32, I64],
               'hetu_cpu_random_init': [P, I64, I32, F32, F32, I64],
               'hetu_cpu_reduce_axis0': [P, P, I64, I64, F32], 'hetu_cpu_reduce_lastdim': [P, P, I64, I64, F32],
               'hetu_cpu_softmax_ce_sparse': [P, P, P, P, I64, I64, I64],
               'hetu_cpu_softmax_ce_sparse_bwd': [P, P, P, I32, P, P, I64, I64, I64]}
        for k, v in sig.items():
            getattr(L, k).argtypes = v
            getattr(L, k).restype = None
        for k, v in {'hetu_cpu_unary_ext': [I32, P, P, I64, F32, F32],
                     'hetu_cpu_binary_nd': [I32, P, P, P, I32, P, P, P, F32],
                     'hetu_cpu_copy_nd': [P, P, I32, I32, P, P, P]}.items():
            getattr(L, k).argtypes = v
            getattr(L, k).restype = I32
        _lib = L
    return _lib


def use(flag=True):
    global _enabled
    _enabled = bool(flag)


def enabled() -> bool:
    return _enabled


def active(*ts) -> bool:
    if not _enabled:
        return False
    for t in ts:
        if t is not None and (t.is_cuda or t.dtype != torch.float32):
            return False
    return True


def record_fallback(name, *ts):
    """an op on fp32 CPU tensors that took the ATen path although the native backend
    is on (callers pass the tensors; nothing is recorded for other dtypes / devices)"""
    if _enabled and all(t is None or (isinstance(t, torch.Tensor) and not t.is_cuda and t.dtype == torch.float32)
                        for t in ts):
        FALLBACKS[name] = FALLBACKS.get(name, 0) + 1
        if _STRICT:
            raise RuntimeError('HETU_STRICT_NATIVE: CPU op %s took the ATen path' % name)


def reset_fallbacks():
    FALLBACKS.clear()


def _arr(v):
    a = _ARR()
    for i, x in enumerate(v):
        a[i] = int(x)
    return a


def _chk(r, name):
    if r != 0:
        raise RuntimeError('native CPU op %s failed (%d)' % (name, r))


def _p(t):
    return t.data_ptr() if t is not None else None


def _operand(t):
    """(ptr, ld, trans) for a 2-D fp32 view that is row- or column-contiguous."""
    if t.stride(1) == 1:
        return t, t.stride(0) if t.shape[0] > 1 else t.shape[1], 0
    if t.stride(0) == 1:
        return t, t.stride(1) if t.shape[1] > 1 else t.shape[0], 1
    t = t.contiguous()
    return t, t.shape[1], 0


def gemm(a, b, bias=None):
    """op(a)[M,K] @ op(b)[K,N] (+bias) for 2-D fp32 views (transposes taken from strides)."""
    M, K = a.shape
    N = b.shape[1]
    A, lda, ta = _operand(a)
    B, ldb, tb = _operand(b)
    out = _NA.empty((M, N), dtype=torch.float32)
    bias = bias.contiguous() if bias is not None else None
    lib().hetu_cpu_gemm(_p(A), _p(B), _p(out), _p(bias), M, N, K, lda, ldb, N, ta, tb, 1.0, 0.0)
    return out


def softmax_ce(logits, labels):
    R, C = logits.shape
    x, y = logits.contiguous(), labels.float().contiguous()
    loss = _NA.empty(R, dtype=torch.float32)
    lse = _NA.empty(R, dtype=torch.float32)
    lib().hetu_cpu_softmax_ce(_p(x), _p(y), _p(loss), _p(lse), R, C)
    return loss, lse


def softmax_ce_backward(logits, labels, grad, lse):
    R, C = logits.shape
    x, y = logits.contiguous(), labels.float().contiguous()
    g = grad.float().contiguous().reshape(-1)
    dx = _NA.empty((R, C), dtype=torch.float32)
    lib().hetu_cpu_softmax_ce_bwd(_p(x), _p(y), _p(g), _p(lse.contiguous()), _p(dx), R, C, int(g.numel() == 1))
    return dx


def unary(op, x):
    xc = x.contiguous()
    y = _NA.empty_like(xc)
    lib().hetu_cpu_unary(UNARY[op], _p(xc), _p(y), xc.numel())
    return y


def relu_grad(x, g):
    xc, gc = x.contiguous(), g.contiguous()
    y = _NA.empty_like(xc)
    lib().hetu_cpu_relu_grad(_p(xc), _p(gc), _p(y), xc.numel())
    return y


def reduce_rows(x2, scale=1.0):
    R, C = x2.shape
    xc = x2.contiguous()
    y = _NA.empty(C, dtype=torch.float32)
    lib().hetu_cpu_reduce_rows(_p(xc), _p(y), R, C, float(scale))
    return y


def gather_rows(table, ids):
    dim = table.shape[-1]
    idx = ids.reshape(-1).long().contiguous()
    out = _NA.empty((idx.numel(), dim), dtype=torch.float32)
    lib().hetu_cpu_gather_rows(_p(table.contiguous()), _p(idx), _p(out), idx.numel(), dim, table.shape[0])
    return out.reshape(tuple(ids.shape) + (dim,))


def optimizer(mode, p, g, s1, s2, lr, l2, mu, b1, b2, b1t, b2t, eps, wd, gscale):
    lib().hetu_cpu_optimizer(OPT[mode], _p(p), _p(g), _p(s1), _p(s2), p.numel(), lr, l2, mu, b1, b2, b1t, b2t, eps,
                             wd, gscale)


# ---- convolution / pooling / batch norm (NCHW fp32; reference src/dnnl_ops) ----------
def _nchw(t):
    return t.float().contiguous()


def _conv_out(H, W, KH, KW, stride, padding):
    return (H + 2 * padding[0] - KH) // stride[0] + 1, (W + 2 * padding[1] - KW) // stride[1] + 1


def conv2d(x, w, b, stride, padding):
    x, w = _nchw(x), _nchw(w)
    N, C, H, W = x.shape
    K, _, KH, KW = w.shape
    OH, OW = _conv_out(H, W, KH, KW, stride, padding)
    y = _NA.empty((N, K, OH, OW), dtype=torch.float32)
    lib().hetu_cpu_conv2d(_p(x), _p(w), _p(b.float().contiguous() if b is not None else None), _p(y),
                          N, C, H, W, K, KH, KW, stride[0], stride[1], padding[0], padding[1])
    return y


def conv2d_backward_data(dy, w, x_shape, stride, padding):
    dy, w = _nchw(dy), _nchw(w)
    N, C, H, W = x_shape
    K, _, KH, KW = w.shape
    dx = _NA.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_conv2d_bwd_data(_p(dy), _p(w), _p(dx), N, C, H, W, K, KH, KW, stride[0], stride[1],
                                   padding[0], padding[1])
    return dx


def conv2d_backward_filter(dy, x, w_shape, stride, padding, want_bias=False):
    dy, x = _nchw(dy), _nchw(x)
    N, C, H, W = x.shape
    K, _, KH, KW = w_shape
    dw = _NA.empty(tuple(w_shape), dtype=torch.float32)
    db = _NA.empty(K, dtype=torch.float32) if want_bias else None
    lib().hetu_cpu_conv2d_bwd_filter(_p(dy), _p(x), _p(dw), _p(db), N, C, H, W, K, KH, KW, stride[0], stride[1],
                                     padding[0], padding[1])
    return (dw, db) if want_bias else dw


def maxpool2d(x, kh, kw, sh, sw, ph, pw):
    """(y, idx int32 [N, C, OH, OW] = argmax offset inside the H*W plane)"""
    x = _nchw(x)
    N, C, H, W = x.shape
    OH, OW = _conv_out(H, W, kh, kw, (sh, sw), (ph, pw))
    y = _NA.empty((N, C, OH, OW), dtype=torch.float32)
    idx = _NA.empty((N, C, OH, OW), dtype=torch.int32)
    lib().hetu_cpu_maxpool2d(_p(x), _p(y), _p(idx), N * C, H, W, kh, kw, sh, sw, ph, pw, OH, OW)
    return y, idx


def maxpool2d_backward(dy, idx, x_shape):
    dy = _nchw(dy)
    N, C, H, W = x_shape
    dx = _NA.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_maxpool2d_bwd(_p(dy), _p(idx.contiguous()), _p(dx), N * C, H, W, dy.shape[2], dy.shape[3])
    return dx


def avgpool2d(x, kh, kw, sh, sw, ph, pw):
    x = _nchw(x)
    N, C, H, W = x.shape
    OH, OW = _conv_out(H, W, kh, kw, (sh, sw), (ph, pw))
    y = _NA.empty((N, C, OH, OW), dtype=torch.float32)
    lib().hetu_cpu_avgpool2d(_p(x), _p(y), N * C, H, W, kh, kw, sh, sw, ph, pw, OH, OW)
    return y


def avgpool2d_backward(dy, x_shape, kh, kw, sh, sw, ph, pw):
    dy = _nchw(dy)
    N, C, H, W = x_shape
    dx = _NA.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_avgpool2d_bwd(_p(dy), _p(dx), N * C, H, W, kh, kw, sh, sw, ph, pw, dy.shape[2], dy.shape[3])
    return dx


def batchnorm(x, scale, bias, running_mean, running_var, factor, eps, training):
    """(y, save_mean, save_invstd); running stats updated in place when training"""
    x = _nchw(x)
    N, C = x.shape[0], x.shape[1]
    HW = x.numel() // max(N * C, 1)
    y = _NA.empty_like(x)
    sm = _NA.empty(C, dtype=torch.float32)
    sr = _NA.empty(C, dtype=torch.float32)
    lib().hetu_cpu_batchnorm(_p(x), _p(scale.float().contiguous()), _p(bias.float().contiguous()), _p(y),
                             _p(running_mean), _p(running_var), _p(sm), _p(sr), N, C, HW, float(factor), float(eps),
                             int(bool(training)))
    return y, sm, sr


def batchnorm_backward(dy, x, scale, save_mean, save_invstd):
    dy, x = _nchw(dy), _nchw(x)
    N, C = x.shape[0], x.shape[1]
    HW = x.numel() // max(N * C, 1)
    dx = _NA.empty_like(x)
    ds = _NA.empty(C, dtype=torch.float32)
    db = _NA.empty(C, dtype=torch.float32)
    lib().hetu_cpu_batchnorm_bwd(_p(dy), _p(x), _p(scale.float().contiguous()), _p(save_mean.contiguous()),
                                 _p(save_invstd.contiguous()), _p(dx), _p(ds), _p(db), N, C, HW)
    return dx, ds, db


# ---- elementwise / layout / softmax / dropout / init (csrc/cpu/cpu_tensor_ops.cc) --------
def unary_code(code, x, c=0.0, c2=0.0, out=None):
    """y = unary op ``code`` (elementwise.hip's U table) of fp32 ``x``."""
    xc = x.contiguous()
    y = out if out is not None and out.is_contiguous() else _NA.empty_like(xc)
    _chk(lib().hetu_cpu_unary_ext(int(code), _p(xc), _p(y), xc.numel(), float(c), float(c2)), 'unary')
    if out is not None and y is not out:
        copy_nd(y, out)
        return out
    return y


def _collapse(shape, sa, sb):
    dims = [(int(n), int(x), int(y)) for n, x, y in zip(shape, sa, sb) if n != 1]
    out = []
    for n, x, y in dims:
        if out and out[-1][1] == n * x and out[-1][2] == n * y:
            out[-1] = (out[-1][0] * n, x, y)
        else:
            out.append((n, x, y))
    if not out:
        out = [(1, 0, 0)]
    return [d[0] for d in out], [d[1] for d in out], [d[2] for d in out]


def binary_code(code, a, b, c=0.0, out=None):
    """y (broadcast shape, contiguous) = binary op ``code`` (elementwise.hip's B table);
    None when the broadcast needs more than 8 dims."""
    shape = torch.broadcast_shapes(a.shape, b.shape)
    if len(shape) == 0:
        shape = (1,)
    ae, be = a.reshape(a.shape or (1,)).expand(shape), b.reshape(b.shape or (1,)).expand(shape)
    cs, ca, cb = _collapse(shape, ae.stride(), be.stride())
    if len(cs) > 8:
        return None
    y = out if (out is not None and out.is_contiguous() and tuple(out.shape) == tuple(shape)) else \
        _NA.empty(shape, dtype=torch.float32)
    _chk(lib().hetu_cpu_binary_nd(int(code), _p(a), _p(b), _p(y), len(cs), _arr(cs), _arr(ca), _arr(cb), float(c)),
         'binary')
    if out is not None and y is not out:
        copy_nd(y.reshape(out.shape), out)
        return out
    return y if (a.dim() or b.dim()) else y.reshape(())


_ESIZE = {torch.float32: 4, torch.int32: 4, torch.int64: 8, torch.float64: 8, torch.bfloat16: 2,
          torch.float16: 2, torch.int16: 2, torch.uint8: 1, torch.int8: 1, torch.bool: 1}


def copy_nd(src, dst):
    """dst[...] = src (same dtype, same shape, any strides; up to 8 collapsed dims)"""
    if src.dtype != dst.dtype or tuple(src.shape) != tuple(dst.shape):
        raise ValueError('copy_nd: %s %s -> %s %s' % (src.dtype, tuple(src.shape), dst.dtype, tuple(dst.shape)))
    if dst.numel() == 0:
        return dst
    cs, cd, css = _collapse(dst.shape or (1,), dst.stride() or (1,), src.stride() or (1,))
    if len(cs) > 8:
        dst.copy_(src)
        return dst
    _chk(lib().hetu_cpu_copy_nd(_p(src), _p(dst), _ESIZE[dst.dtype], len(cs), _arr(cs), _arr(css), _arr(cd)),
         'copy_nd')
    return dst


def fill(t, v):
    assert t.is_contiguous() and t.dtype == torch.float32
    lib().hetu_cpu_fill(_p(t), t.numel(), float(v))
    return t


def softmax(x, log=False):
    xc = x.contiguous()
    y = _NA.empty_like(xc)
    C = x.shape[-1] if x.dim() else 1
    lib().hetu_cpu_softmax(_p(xc), _p(y), xc.numel() // max(C, 1), C, int(bool(log)))
    return y


def softmax_backward(y, dy):
    yc, gc = y.contiguous(), dy.contiguous()
    dx = _NA.empty_like(yc)
    C = y.shape[-1]
    lib().hetu_cpu_softmax_bwd(_p(yc), _p(gc), _p(dx), yc.numel() // C, C)
    return dx


def softmax_ce_sparse(logits, labels, ignored):
    C = logits.shape[-1]
    x = logits.contiguous()
    lab = labels.reshape(-1).long().contiguous()
    R = x.numel() // C
    loss = _NA.empty(R, dtype=torch.float32)
    lse = _NA.empty(R, dtype=torch.float32)
    lib().hetu_cpu_softmax_ce_sparse(_p(x), _p(lab), _p(loss), _p(lse), R, C, int(ignored))
    return loss.reshape(logits.shape[:-1]), lse.reshape(logits.shape[:-1])


def softmax_ce_sparse_backward(logits, labels, g, scalar, lse, ignored):
    C = logits.shape[-1]
    x = logits.contiguous()
    lab = labels.reshape(-1).long().contiguous()
    R = x.numel() // C
    dx = _NA.empty_like(x)
    lib().hetu_cpu_softmax_ce_sparse_bwd(_p(x), _p(lab), _p(g), int(scalar), _p(lse.contiguous()), _p(dx), R, C,
                                         int(ignored))
    return dx


def dropout(x, keep, seed):
    """Philox mask at counter = flat index / 4: the GPU kernel's mask for the same seed"""
    xc = x.contiguous()
    y = _NA.empty_like(xc)
    lib().hetu_cpu_dropout(_p(xc), _p(y), xc.numel(), float(keep), int(seed))
    return y


INIT = {'uniform': 0, 'normal': 1, 'truncated_normal': 2}


def random_init(t, kind, a, b, seed):
    """fill contiguous fp32 ``t``: uniform [a, b), normal(a, b), truncated normal(a, b)"""
    assert t.is_contiguous() and t.dtype == torch.float32 and not t.is_cuda
    lib().hetu_cpu_random_init(_p(t), t.numel(), INIT[kind], float(a), float(b), int(seed) & ((1 << 63) - 1))
    return t


def reduce_axis0(x2, scale=1.0):
    R, C = x2.shape
    xc = x2.contiguous()
    y = _NA.empty(C, dtype=torch.float32)
    lib().hetu_cpu_reduce_axis0(_p(xc), _p(y), R, C, float(scale))
    return y


def reduce_lastdim(x2, scale=1.0):
    R, C = x2.shape
    xc = x2.contiguous()
    y = _NA.empty(R, dtype=torch.float32)
    lib().hetu_cpu_reduce_lastdim(_p(xc), _p(y), R, C, float(scale))
    return y
