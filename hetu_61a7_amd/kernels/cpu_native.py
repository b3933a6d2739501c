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
               'hetu_cpu_optimizer': [I32, P, P, P, P, I64] + [F32] * 10}
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
