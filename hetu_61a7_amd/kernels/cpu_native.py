"""Native C++/OpenMP CPU backend (``csrc/cpu/cpu_ops.cc`` -> ``libhetu_cpu.so``),
the counterpart of the reference's DNNL/OpenMP CPU ops (``src/dnnl_ops``,
``cpu_links/dnnl_op.py``).  Active for fp32 CPU tensors when
``HETU_CPU_BACKEND=native`` (otherwise the CPU path is torch's ATen);
``use(True/False)`` switches it at run time.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .._base import _LIB_DIR

_PATH = os.path.join(_LIB_DIR, 'libhetu_cpu.so')
_lib = None
_enabled = os.environ.get('HETU_CPU_BACKEND', '') == 'native'
P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
UNARY = {'relu': 0, 'sigmoid': 1, 'tanh': 2, 'gelu': 3, 'exp': 4, 'sqrt': 5}
OPT = dict(sgd=0, momentum=1, nesterov=2, adagrad=3, adam=4, adamw=5)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            raise RuntimeError('libhetu_cpu.so not built (%s); run make -C csrc' % _PATH)
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
               'hetu_cpu_batchnorm_bwd': [P] * 8 + [I64] * 3}
        for k, v in sig.items():
            getattr(L, k).argtypes = v
            getattr(L, k).restype = None
        _lib = L
    return _lib


def use(flag=True):
    global _enabled
    _enabled = bool(flag)


def active(*ts) -> bool:
    if not _enabled:
        return False
    for t in ts:
        if t is not None and (t.is_cuda or t.dtype != torch.float32):
            return False
    return True


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
    out = torch.empty((M, N), dtype=torch.float32)
    bias = bias.contiguous() if bias is not None else None
    lib().hetu_cpu_gemm(_p(A), _p(B), _p(out), _p(bias), M, N, K, lda, ldb, N, ta, tb, 1.0, 0.0)
    return out


def softmax_ce(logits, labels):
    R, C = logits.shape
    x, y = logits.contiguous(), labels.float().contiguous()
    loss = torch.empty(R, dtype=torch.float32)
    lse = torch.empty(R, dtype=torch.float32)
    lib().hetu_cpu_softmax_ce(_p(x), _p(y), _p(loss), _p(lse), R, C)
    return loss, lse


def softmax_ce_backward(logits, labels, grad, lse):
    R, C = logits.shape
    x, y = logits.contiguous(), labels.float().contiguous()
    g = grad.float().contiguous().reshape(-1)
    dx = torch.empty((R, C), dtype=torch.float32)
    lib().hetu_cpu_softmax_ce_bwd(_p(x), _p(y), _p(g), _p(lse.contiguous()), _p(dx), R, C, int(g.numel() == 1))
    return dx


def unary(op, x):
    xc = x.contiguous()
    y = torch.empty_like(xc)
    lib().hetu_cpu_unary(UNARY[op], _p(xc), _p(y), xc.numel())
    return y


def relu_grad(x, g):
    xc, gc = x.contiguous(), g.contiguous()
    y = torch.empty_like(xc)
    lib().hetu_cpu_relu_grad(_p(xc), _p(gc), _p(y), xc.numel())
    return y


def reduce_rows(x2, scale=1.0):
    R, C = x2.shape
    xc = x2.contiguous()
    y = torch.empty(C, dtype=torch.float32)
    lib().hetu_cpu_reduce_rows(_p(xc), _p(y), R, C, float(scale))
    return y


def gather_rows(table, ids):
    dim = table.shape[-1]
    idx = ids.reshape(-1).long().contiguous()
    out = torch.empty((idx.numel(), dim), dtype=torch.float32)
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
    y = torch.empty((N, K, OH, OW), dtype=torch.float32)
    lib().hetu_cpu_conv2d(_p(x), _p(w), _p(b.float().contiguous() if b is not None else None), _p(y),
                          N, C, H, W, K, KH, KW, stride[0], stride[1], padding[0], padding[1])
    return y


def conv2d_backward_data(dy, w, x_shape, stride, padding):
    dy, w = _nchw(dy), _nchw(w)
    N, C, H, W = x_shape
    K, _, KH, KW = w.shape
    dx = torch.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_conv2d_bwd_data(_p(dy), _p(w), _p(dx), N, C, H, W, K, KH, KW, stride[0], stride[1],
                                   padding[0], padding[1])
    return dx


def conv2d_backward_filter(dy, x, w_shape, stride, padding, want_bias=False):
    dy, x = _nchw(dy), _nchw(x)
    N, C, H, W = x.shape
    K, _, KH, KW = w_shape
    dw = torch.empty(tuple(w_shape), dtype=torch.float32)
    db = torch.empty(K, dtype=torch.float32) if want_bias else None
    lib().hetu_cpu_conv2d_bwd_filter(_p(dy), _p(x), _p(dw), _p(db), N, C, H, W, K, KH, KW, stride[0], stride[1],
                                     padding[0], padding[1])
    return (dw, db) if want_bias else dw


def maxpool2d(x, kh, kw, sh, sw, ph, pw):
    """(y, idx int32 [N, C, OH, OW] = argmax offset inside the H*W plane)"""
    x = _nchw(x)
    N, C, H, W = x.shape
    OH, OW = _conv_out(H, W, kh, kw, (sh, sw), (ph, pw))
    y = torch.empty((N, C, OH, OW), dtype=torch.float32)
    idx = torch.empty((N, C, OH, OW), dtype=torch.int32)
    lib().hetu_cpu_maxpool2d(_p(x), _p(y), _p(idx), N * C, H, W, kh, kw, sh, sw, ph, pw, OH, OW)
    return y, idx


def maxpool2d_backward(dy, idx, x_shape):
    dy = _nchw(dy)
    N, C, H, W = x_shape
    dx = torch.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_maxpool2d_bwd(_p(dy), _p(idx.contiguous()), _p(dx), N * C, H, W, dy.shape[2], dy.shape[3])
    return dx


def avgpool2d(x, kh, kw, sh, sw, ph, pw):
    x = _nchw(x)
    N, C, H, W = x.shape
    OH, OW = _conv_out(H, W, kh, kw, (sh, sw), (ph, pw))
    y = torch.empty((N, C, OH, OW), dtype=torch.float32)
    lib().hetu_cpu_avgpool2d(_p(x), _p(y), N * C, H, W, kh, kw, sh, sw, ph, pw, OH, OW)
    return y


def avgpool2d_backward(dy, x_shape, kh, kw, sh, sw, ph, pw):
    dy = _nchw(dy)
    N, C, H, W = x_shape
    dx = torch.empty((N, C, H, W), dtype=torch.float32)
    lib().hetu_cpu_avgpool2d_bwd(_p(dy), _p(dx), N * C, H, W, kh, kw, sh, sw, ph, pw, dy.shape[2], dy.shape[3])
    return dx


def batchnorm(x, scale, bias, running_mean, running_var, factor, eps, training):
    """(y, save_mean, save_invstd); running stats updated in place when training"""
    x = _nchw(x)
    N, C = x.shape[0], x.shape[1]
    HW = x.numel() // max(N * C, 1)
    y = torch.empty_like(x)
    sm = torch.empty(C, dtype=torch.float32)
    sr = torch.empty(C, dtype=torch.float32)
    lib().hetu_cpu_batchnorm(_p(x), _p(scale.float().contiguous()), _p(bias.float().contiguous()), _p(y),
                             _p(running_mean), _p(running_var), _p(sm), _p(sr), N, C, HW, float(factor), float(eps),
                             int(bool(training)))
    return y, sm, sr


def batchnorm_backward(dy, x, scale, save_mean, save_invstd):
    dy, x = _nchw(dy), _nchw(x)
    N, C = x.shape[0], x.shape[1]
    HW = x.numel() // max(N * C, 1)
    dx = torch.empty_like(x)
    ds = torch.empty(C, dtype=torch.float32)
    db = torch.empty(C, dtype=torch.float32)
    lib().hetu_cpu_batchnorm_bwd(_p(dy), _p(x), _p(scale.float().contiguous()), _p(save_mean.contiguous()),
                                 _p(save_invstd.contiguous()), _p(dx), _p(ds), _p(db), N, C, HW)
    return dx, ds, db
