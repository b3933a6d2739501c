"""Bindings of ``csrc/kernels/tensor_ops.hip`` and ``losses.hip``: the layout,
indexing, scan, sort and loss kernels of the op long tail (concat / pad / roll /
repeat / gather / scatter-add / cumsum / argmax / argsort / p-norm / CE / BCE / NLL).

Each function takes torch tensors on the GPU and runs on the current HIP stream;
the op modules call them for GPU tensors (``kernels.native``) and keep their torch
reference path for the CPU backend.
"""
from __future__ import annotations

import ctypes

import torch
from .. import native_array as _NA

from . import fn, check, stream_ptr, P, I32, I64, F32, record_native

_ELEM = {torch.float32: 4, torch.bfloat16: 2, torch.float16: 2, torch.int64: 8, torch.int32: 4, torch.uint8: 1,
         torch.int8: 1, torch.bool: 1, torch.float64: 8, torch.int16: 2}
_ARR = ctypes.c_int64 * 8


def _arr(v):
    a = _ARR()
    for i, x in enumerate(v):
        a[i] = int(x)
    return a


def _bf(t):
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError('kernel takes fp32 / bf16, got %s' % t.dtype)


def _dims(shape, dim):
    dim = dim % len(shape) if len(shape) else 0
    outer = 1
    for s in shape[:dim]:
        outer *= int(s)
    inner = 1
    for s in shape[dim + 1:]:
        inner *= int(s)
    return outer, int(shape[dim]) if len(shape) else 1, inner


# ---- strided copies --------------------------------------------------------------------
def nd_copy(src, dst, shift=None, imod=None):
    """dst[c] = src[(c + shift) % imod] elementwise over dst's shape (both strided views
    of the same dtype; src's shape may differ where imod wraps)."""
    assert src.dtype == dst.dtype
    if not dst.is_cuda:
        from . import cpu_native
        if shift is None and imod is None and cpu_native.enabled():
            return cpu_native.copy_nd(src, dst)
        cpu_native.record_fallback('nd_copy', src, dst)
        if shift is None and imod is None:
            return dst.copy_(src)
        idx = [torch.remainder(torch.arange(n) + (sh or 0), m or n) for n, sh, m in zip(dst.shape, shift, imod)]
        dst.copy_(src[torch.meshgrid(*idx, indexing='ij')] if idx else src)
        return dst
    nd = dst.dim()
    if nd == 0:
        dst.copy_(src)
        return dst
    if nd > 8:
        raise ValueError('nd_copy: at most 8 dims')
    f = fn('hetu_nd_copy', [P, P, I32, I32, P, P, P, P, P, P])
    check(f(src.data_ptr(), dst.data_ptr(), _ELEM[dst.dtype], nd, _arr(dst.shape), _arr(dst.stride()),
            _arr(src.stride()), _arr(shift) if shift is not None else None,
            _arr(imod) if imod is not None else None, stream_ptr()), 'nd_copy')
    record_native('nd_copy')
    return dst


def fill_(t, value):
    """t (contiguous) = value."""
    assert t.is_contiguous()
    if not t.is_cuda:
        from . import cpu_native
        if t.dtype == torch.float32 and cpu_native.enabled():
            return cpu_native.fill(t, value)
        return t.fill_(value)
    bits = torch.tensor([value], dtype=t.dtype).view({1: torch.uint8, 2: torch.int16, 4: torch.int32,
                                                      8: torch.int64}[_ELEM[t.dtype]]).item()
    f = fn('hetu_fill', [P, I32, I64, ctypes.c_uint64, P])
    check(f(t.data_ptr(), _ELEM[t.dtype], t.numel(), bits & ((1 << (8 * _ELEM[t.dtype])) - 1), stream_ptr()), 'fill')
    return t


def zeros(shape, dtype=torch.float32, device='cuda'):
    """zero-filled device tensor by the native fill kernel (no torch fill launch)"""
    t = _NA.empty(shape, dtype=dtype, device=device)
    if t.is_cuda and t.numel():
        f = fn('hetu_fill', [P, I32, I64, ctypes.c_uint64, P])
        check(f(t.data_ptr(), _ELEM[t.dtype], t.numel(), 0, stream_ptr()), 'fill')
    elif t.numel():
        fill_(t, 0)
    return t


def one_hot(idx, C):
    """fp32 one-hot rows of int64 / int32 / fp32 class ids (out-of-range ids: zero rows)"""
    kind = {torch.int64: 0, torch.int32: 1, torch.float32: 2}[idx.dtype]
    idx = idx.contiguous()
    y = _NA.empty(tuple(idx.shape) + (C,), dtype=torch.float32, device=idx.device)
    f = fn('hetu_one_hot', [P, I32, P, I64, I32, P])
    check(f(idx.data_ptr(), kind, y.data_ptr(), idx.numel(), C, stream_ptr()), 'one_hot')
    record_native('one_hot')
    return y


def _dense(t):
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def copy_into(dst, src):
    """dst[...] = src on the native kernels: same dtype -> strided copy (nd_copy);
    fp32 <-> bf16 over identical dense layouts -> the cast kernel on the flat storage."""
    if not (dst.is_cuda or src.is_cuda) and tuple(dst.shape) == tuple(src.shape) and dst.dtype == src.dtype:
        return nd_copy(src, dst)
    if not (dst.is_cuda and src.is_cuda) or tuple(dst.shape) != tuple(src.shape):
        return dst.copy_(src)
    if dst.dtype == src.dtype:
        return nd_copy(src, dst)
    if {dst.dtype, src.dtype} == {torch.float32, torch.bfloat16} and dst.stride() == src.stride() and _dense(dst):
        f = fn('hetu_cast', [P, I32, P, I32, I64, P])
        check(f(src.data_ptr(), int(src.dtype == torch.bfloat16), dst.data_ptr(), int(dst.dtype == torch.bfloat16),
                dst.numel(), stream_ptr()), 'cast')
        record_native('cast')
        return dst
    if {dst.dtype, src.dtype} == {torch.float32, torch.bfloat16} and _dense(src):
        tmp = _NA.empty_like(src, dtype=dst.dtype)       # src's dense layout
        copy_into(tmp, src)
        return nd_copy(tmp, dst)
    from . import record_fallback
    record_fallback('copy_into', '%s %s -> %s %s' % (src.dtype, tuple(src.stride()), dst.dtype, tuple(dst.stride())))
    return dst.copy_(src)


def concat(tensors, axis):
    dt = tensors[0].dtype
    shape = list(tensors[0].shape)
    axis = axis % len(shape)
    shape[axis] = sum(int(t.shape[axis]) for t in tensors)
    out = _NA.empty(shape, dtype=dt, device=tensors[0].device)
    off = 0
    for t in tensors:
        n = int(t.shape[axis])
        if n:
            nd_copy(t.to(dt), out.narrow(axis, off, n))
        off += n
    return out


def pad_constant(x, pads, value):
    """pads: [(before, after)] per dim (all dims)."""
    shape = [int(s) + a + b for s, (a, b) in zip(x.shape, pads)]
    out = _NA.empty(shape, dtype=x.dtype, device=x.device)
    fill_(out, value)
    view = out
    for d, (a, _) in enumerate(pads):
        view = view.narrow(d, a, int(x.shape[d]))
    nd_copy(x, view)
    return out


def unpad(g, pads):
    """gradient of a constant pad: the interior view of g, contiguous."""
    view = g
    for d, (a, b) in enumerate(pads):
        view = view.narrow(d, a, int(g.shape[d]) - a - b)
    out = _NA.empty(view.shape, dtype=g.dtype, device=g.device)
    return nd_copy(view, out)


def roll(x, shifts, dims):
    out = _NA.empty(x.shape, dtype=x.dtype, device=x.device)
    sh = [0] * x.dim()
    md = [0] * x.dim()
    for s, d in zip(shifts, dims):
        d = d % x.dim()
        n = int(x.shape[d])
        if n:
            sh[d] = (n - (s % n)) % n
            md[d] = n
    return nd_copy(x, out, sh, md)


def repeat(x, reps):
    """torch.Tensor.repeat semantics (reps may add leading dims)."""
    reps = list(reps)
    xs = [1] * (len(reps) - x.dim()) + list(x.shape)
    xv = x.reshape(xs)
    out = _NA.empty([a * b for a, b in zip(xs, reps)], dtype=x.dtype, device=x.device)
    if not x.is_cuda:   # out viewed as [r0, s0, r1, s1, ...] = x broadcast over the r axes
        inter, src = [], []
        for r, n in zip(reps, xs):
            inter += [r, n]
            src += [1, n]
        nd_copy(xv.reshape(src).expand(inter), out.view(inter))
        return out
    return nd_copy(xv, out, [0] * len(xs), xs)


# ---- gather / scatter-add ----------------------------------------------------------------
def gather(x, dim, idx):
    x = x.contiguous()
    idx = idx.long().contiguous()
    dim = dim % x.dim()
    outer, nsrc, inner = _dims(x.shape, dim)
    oi, nidx, ii = _dims(idx.shape, dim)
    if oi != outer or ii != inner:
        raise ValueError('gather: index must match the input outside dim')
    out = _NA.empty(idx.shape, dtype=x.dtype, device=x.device)
    f = fn('hetu_gather_dim', [P, P, P, I64, I64, I64, I64, I32, P])
    check(f(x.data_ptr(), idx.data_ptr(), out.data_ptr(), outer, nidx, nsrc, inner, _bf(x), stream_ptr()), 'gather')
    record_native('gather')
    return out


def scatter_add(g, dim, idx, shape):
    """dx (fp32, ``shape``) with dx[..idx..] += g (the gather gradient)."""
    g = g.contiguous()
    idx = idx.long().contiguous()
    dim = dim % len(shape)
    outer, nsrc, inner = _dims(shape, dim)
    _, nidx, _ = _dims(idx.shape, dim)
    dx = _NA.zeros(shape, dtype=torch.float32, device=g.device)
    f = fn('hetu_scatter_add_dim', [P, P, P, I64, I64, I64, I64, I32, P])
    check(f(g.data_ptr(), idx.data_ptr(), dx.data_ptr(), outer, nidx, nsrc, inner, _bf(g), stream_ptr()),
          'scatter_add')
    record_native('scatter_add')
    return dx


# ---- scan / arg-reductions / sort / norm -------------------------------------------------------
def cumsum(x, dim, bias=0.0):
    x = x.contiguous()
    outer, n, inner = _dims(x.shape, dim)
    y = _NA.empty(x.shape, dtype=torch.float32, device=x.device)
    f = fn('hetu_scan_dim', [P, P, I64, I64, I64, F32, I32, P])
    check(f(x.data_ptr(), y.data_ptr(), outer, n, inner, float(bias), _bf(x), stream_ptr()), 'scan')
    record_native('cumsum')
    return y


def argmax(x, dim):
    x = x.contiguous()
    dim = dim % x.dim()
    outer, n, inner = _dims(x.shape, dim)
    shape = list(x.shape)
    shape.pop(dim)
    out = _NA.empty(shape, dtype=torch.int64, device=x.device)
    f = fn('hetu_argmax_dim', [P, P, I64, I64, I64, I32, P])
    check(f(x.data_ptr(), out.data_ptr(), outer, n, inner, _bf(x), stream_ptr()), 'argmax')
    record_native('argmax')
    return out


ARGSORT_MAX = 8192


def argsort(x, dim=-1, descending=False):
    """Per-row LDS bitonic sort (rows up to 8192 long); ties keep index order."""
    dim = dim % x.dim()
    xt = x.transpose(dim, -1).contiguous() if dim != x.dim() - 1 else x.contiguous()
    n = int(xt.shape[-1])
    if n > ARGSORT_MAX:
        return None
    rows = xt.numel() // max(n, 1)
    out = _NA.empty(xt.shape, dtype=torch.int64, device=x.device)
    f = fn('hetu_argsort_rows', [P, P, I64, I64, I32, I32, P])
    check(f(xt.data_ptr(), out.data_ptr(), rows, n, int(bool(descending)), _bf(xt), stream_ptr()), 'argsort')
    record_native('argsort')
    return out.transpose(dim, -1) if dim != x.dim() - 1 else out


def pnorm(x, dim, p=2.0, keepdim=True):
    x = x.contiguous()
    dim = dim % x.dim()
    outer, n, inner = _dims(x.shape, dim)
    shape = list(x.shape)
    shape[dim] = 1
    y = _NA.empty(shape, dtype=x.dtype, device=x.device)
    f = fn('hetu_pnorm_dim', [P, P, I64, I64, I64, F32, I32, P])
    check(f(x.data_ptr(), y.data_ptr(), outer, n, inner, float(p), _bf(x), stream_ptr()), 'pnorm')
    record_native('norm')
    return y if keepdim else y.squeeze(dim)


def pnorm_grad(x, y, g, dim, p=2.0):
    """y, g: the norm and its gradient with the reduced dim kept (size 1)."""
    x = x.contiguous()
    dim = dim % x.dim()
    outer, n, inner = _dims(x.shape, dim)
    y = y.to(x.dtype).contiguous()
    g = g.to(x.dtype).contiguous()
    dx = _NA.empty(x.shape, dtype=x.dtype, device=x.device)
    f = fn('hetu_pnorm_grad_dim', [P, P, P, P, I64, I64, I64, F32, I32, P])
    check(f(x.data_ptr(), y.data_ptr(), g.data_ptr(), dx.data_ptr(), outer, n, inner, float(p), _bf(x),
            stream_ptr()), 'pnorm_grad')
    record_native('norm_grad')
    return dx


# ---- losses ------------------------------------------------------------------------------
def _rows(y):
    cols = int(y.shape[-1])
    return y.numel() // max(cols, 1), cols


def _g(g, rows):
    g = g.float().contiguous()
    return g, int(g.numel() == 1 and rows != 1)


def ce_dense(y, lab):
    y, lab = y.contiguous(), lab.to(y.dtype).contiguous()
    rows, cols = _rows(y)
    out = _NA.empty(y.shape[:-1], dtype=torch.float32, device=y.device)
    check(fn('hetu_ce_dense', [P, P, P, I64, I64, I32, P])(y.data_ptr(), lab.data_ptr(), out.data_ptr(), rows,
                                                            cols, _bf(y), stream_ptr()), 'ce_dense')
    record_native('crossentropy')
    return out


def ce_dense_grad(g, y, lab):
    y, lab = y.contiguous(), lab.to(y.dtype).contiguous()
    rows, cols = _rows(y)
    g, gs = _g(g, rows)
    dy = _NA.empty(y.shape, dtype=y.dtype, device=y.device)
    check(fn('hetu_ce_dense_grad', [P, P, P, P, I64, I64, I32, I32, P])(
        g.data_ptr(), y.data_ptr(), lab.data_ptr(), dy.data_ptr(), rows, cols, gs, _bf(y), stream_ptr()),
        'ce_dense_grad')
    return dy


def ce_sparse(y, lab, ignore=-1):
    y = y.contiguous()
    rows, cols = _rows(y)
    lab = lab.long().reshape(-1).contiguous()
    out = _NA.empty(y.shape[:-1], dtype=torch.float32, device=y.device)
    check(fn('hetu_ce_sparse', [P, P, P, I64, I64, I64, I32, P])(y.data_ptr(), lab.data_ptr(), out.data_ptr(),
                                                                  rows, cols, int(ignore), _bf(y), stream_ptr()),
          'ce_sparse')
    record_native('crossentropy_sparse')
    return out


def ce_sparse_grad(g, y, lab, ignore=-1):
    y = y.contiguous()
    rows, cols = _rows(y)
    lab = lab.long().reshape(-1).contiguous()
    g, gs = _g(g, rows)
    dy = _NA.empty(y.shape, dtype=y.dtype, device=y.device)
    check(fn('hetu_ce_sparse_grad', [P, P, P, P, I64, I64, I64, I32, I32, P])(
        g.data_ptr(), y.data_ptr(), lab.data_ptr(), dy.data_ptr(), rows, cols, int(ignore), gs, _bf(y),
        stream_ptr()), 'ce_sparse_grad')
    return dy


def _as_dense(t, dtype):
    """t as a contiguous tensor of ``dtype`` through the native cast / strided-copy kernels"""
    if t.dtype == dtype and t.is_contiguous():
        return t
    if t.dtype != dtype:
        if not t.is_contiguous():
            t = copy_into(_NA.empty(tuple(t.shape), dtype=t.dtype, device=t.device), t)
        return copy_into(_NA.empty(tuple(t.shape), dtype=dtype, device=t.device), t)
    return copy_into(_NA.empty(tuple(t.shape), dtype=dtype, device=t.device), t)


def bce(y, lab):
    y, lab = _as_dense(y, y.dtype), _as_dense(lab, y.dtype)
    out = _NA.empty(y.shape, dtype=torch.float32, device=y.device)
    check(fn('hetu_bce', [P, P, P, I64, I32, P])(y.data_ptr(), lab.data_ptr(), out.data_ptr(), y.numel(), _bf(y),
                                                  stream_ptr()), 'bce')
    record_native('bce')
    return out


def bce_grad(y, lab, g):
    y, lab = _as_dense(y, y.dtype), _as_dense(lab, y.dtype)
    g = _as_dense(g, torch.float32)
    if g.numel() not in (1, y.numel()):
        g = copy_into(_NA.empty(tuple(y.shape), dtype=torch.float32, device=y.device), g.expand(y.shape))
    gs = int(g.numel() == 1 and y.numel() != 1)
    dy = _NA.empty(y.shape, dtype=y.dtype, device=y.device)
    check(fn('hetu_bce_grad', [P, P, P, P, I64, I32, I32, P])(y.data_ptr(), lab.data_ptr(), g.data_ptr(),
                                                               dy.data_ptr(), y.numel(), gs, _bf(y), stream_ptr()),
          'bce_grad')
    return dy


_LABEL_KIND = {torch.int64: 0, torch.int32: 1, torch.float32: 2}


def _labels(t):
    """labels as the kernels read them (int64 / int32 / fp32 class indices), converting only
    another dtype"""
    t = t.reshape(-1)
    if t.dtype not in _LABEL_KIND:
        t = t.long()
    return t.contiguous(), _LABEL_KIND[t.dtype]


def nll(x, t, cols):
    x = x.reshape(-1, cols).contiguous()
    t, tk = _labels(t)
    out = zeros((1,), torch.float32, x.device)
    check(fn('hetu_nll', [P, P, I32, P, I64, I64, I32, P])(x.data_ptr(), t.data_ptr(), tk, out.data_ptr(),
                                                            x.shape[0], cols, _bf(x), stream_ptr()), 'nll')
    record_native('nll')
    return out


def nll_grad(g, t, cols):
    t, tk = _labels(t)
    g = g.reshape(-1)[:1]
    if g.dtype != torch.float32:
        g = g.float()
    dx = _NA.empty((t.numel(), cols), dtype=torch.float32, device=t.device)
    check(fn('hetu_nll_grad', [P, P, I32, P, I64, I64, P])(g.data_ptr(), t.data_ptr(), tk, dx.data_ptr(), t.numel(),
                                                            cols, stream_ptr()), 'nll_grad')
    record_native('nll_grad')
    return dx


# ---- misc_ops.hip: SAM gate helpers, instance norm, bicubic ---------------------------------
def _i64(t):
    return t.long().reshape(-1).contiguous()


def sam_group_sum(x, G):
    x = x.float().contiguous()
    T, E = x.shape
    out = _NA.empty((T, G), dtype=torch.float32, device=x.device)
    check(fn('hetu_sam_group_sum', [P, P, I64, I32, I32, P])(x.data_ptr(), out.data_ptr(), T, E, G, stream_ptr()),
          'sam_group_sum')
    record_native('sam_group_sum')
    return out


def sam_group_sum_grad(g, T, E, G):
    g = g.float().contiguous()
    dx = _NA.empty((T, E), dtype=torch.float32, device=g.device)
    check(fn('hetu_sam_group_sum_grad', [P, P, I64, I32, I32, P])(g.data_ptr(), dx.data_ptr(), T, E, G,
                                                                   stream_ptr()), 'sam_group_sum_grad')
    record_native('sam_group_sum_grad')
    return dx


def sam_max(x, grp, tk, n):
    x = x.float().contiguous()
    T, E = x.shape
    grp, tk = _i64(grp), _i64(tk)
    y = _NA.empty((T, E), dtype=torch.float32, device=x.device)
    check(fn('hetu_sam_max', [P, P, P, P, I64, I32, I32, P])(x.data_ptr(), grp.data_ptr(), tk.data_ptr(),
                                                             y.data_ptr(), T, E, n, stream_ptr()), 'sam_max')
    record_native('sam_max')
    return y


def sam_max_grad(g, x, grp, tk, n):
    x, g = x.float().contiguous(), g.float().contiguous()
    T, E = x.shape
    grp, tk = _i64(grp), _i64(tk)
    dx = _NA.empty((T, E), dtype=torch.float32, device=x.device)
    check(fn('hetu_sam_max_grad', [P, P, P, P, P, I64, I32, I32, P])(
        g.data_ptr(), x.data_ptr(), grp.data_ptr(), tk.data_ptr(), dx.data_ptr(), T, E, n, stream_ptr()),
        'sam_max_grad')
    record_native('sam_max_grad')
    return dx


GROUP_TOPK_MAX = 64 * 64


def group_topk_idx(x, grp, k, n):
    """Top-k column ids of each row inside its group's columns (descending, ties to the
    lower id); None when the group is wider than the kernel's register stripes."""
    if n > GROUP_TOPK_MAX or k > n:
        return None
    x = x.float().contiguous()
    T, E = x.shape
    grp = _i64(grp)
    out = _NA.empty((T, k), dtype=torch.int64, device=x.device)
    check(fn('hetu_group_topk_idx', [P, P, P, I64, I32, I32, I32, P])(
        x.data_ptr(), grp.data_ptr(), out.data_ptr(), T, E, n, k, stream_ptr()), 'group_topk_idx')
    record_native('group_topk_idx')
    return out


def _plane_view(x):
    """Strides (sN, sC, sP) of an NCHW view whose H, W merge into one axis (contiguous
    NCHW: sP = 1; channels-last: sP = C); makes it contiguous otherwise."""
    if x.stride(2) != x.shape[3] * x.stride(3):
        x = x.contiguous()
    return x, (x.stride(0), x.stride(1), x.stride(3))


def instance_norm2d(x, eps):
    """x logical NCHW fp32/bf16 (NCHW or channels-last) -> (y, mean, rstd), stats [N, C, 1, 1] fp32."""
    x, (sN, sC, sP) = _plane_view(x)
    N, C, H, W = x.shape
    y = _NA.empty_like(x)
    if y.stride() != x.stride():
        x = x.contiguous()
        y = _NA.empty_like(x)
        sN, sC, sP = x.stride(0), x.stride(1), x.stride(3)
    mean = _NA.empty((N, C, 1, 1), dtype=torch.float32, device=x.device)
    rstd = _NA.empty_like(mean)
    check(fn('hetu_instance_norm2d', [P, P, P, P, I32, I32, I64, I64, I64, I64, F32, I32, P])(
        x.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), N, C, H * W, sN, sC, sP, float(eps), _bf(x),
        stream_ptr()), 'instance_norm2d')
    record_native('instance_norm2d')
    return y, mean, rstd


def instance_norm2d_grad(g, x, mean, rstd):
    x, (sN, sC, sP) = _plane_view(x)
    g = g.to(x.dtype)
    if g.stride() != x.stride():
        g = _NA.empty_like(x).copy_(g)
    dx = _NA.empty_like(x)
    if dx.stride() != x.stride():
        x = x.contiguous()
        g, dx = g.contiguous(), _NA.empty_like(x)
        sN, sC, sP = x.stride(0), x.stride(1), x.stride(3)
    N, C, H, W = x.shape
    mean, rstd = mean.float().contiguous(), rstd.float().contiguous()
    check(fn('hetu_instance_norm2d_grad', [P, P, P, P, P, I32, I32, I64, I64, I64, I64, I32, P])(
        g.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), N, C, H * W, sN, sC, sP,
        _bf(x), stream_ptr()), 'instance_norm2d_grad')
    record_native('instance_norm2d_grad')
    return dx


def _cubic_scale(inp, out, align, scale_factor):
    if align:
        return (inp - 1) / (out - 1) if out > 1 else 0.0
    if scale_factor is not None and scale_factor > 0:
        return 1.0 / scale_factor
    return inp / out


def bicubic(x, OH, OW, align_corners=False, scale_factor=None):
    """PyTorch-compatible bicubic upsampling (A = -0.75, border clamp), fp32 math."""
    N, C, H, W = x.shape
    xf = x.float().contiguous()
    y = _NA.empty((N, C, OH, OW), dtype=torch.float32, device=x.device)
    sh = _cubic_scale(H, OH, align_corners, scale_factor)
    sw = _cubic_scale(W, OW, align_corners, scale_factor)
    check(fn('hetu_bicubic', [P, P, I64, I32, I32, I32, I32, F32, F32, I32, P])(
        xf.data_ptr(), y.data_ptr(), N * C, H, W, OH, OW, sh, sw, int(bool(align_corners)), stream_ptr()), 'bicubic')
    record_native('bicubic')
    return y.to(x.dtype)


def bicubic_grad(g, shape, align_corners=False, scale_factor=None):
    N, C, H, W = (int(s) for s in shape)
    OH, OW = int(g.shape[2]), int(g.shape[3])
    gf = g.float().contiguous()
    dx = _NA.zeros((N, C, H, W), dtype=torch.float32, device=g.device)
    sh = _cubic_scale(H, OH, align_corners, scale_factor)
    sw = _cubic_scale(W, OW, align_corners, scale_factor)
    check(fn('hetu_bicubic_grad', [P, P, I64, I32, I32, I32, I32, F32, F32, I32, P])(
        gf.data_ptr(), dx.data_ptr(), N * C, H, W, OH, OW, sh, sw, int(bool(align_corners)), stream_ptr()),
        'bicubic_grad')
    record_native('bicubic_grad')
    return dx.to(g.dtype)
