"""2-D convolution (logical NCHW, physical channels-last on the GPU).

The forward/backward-data/backward-filter entry points run the hand-written MFMA
kernels: the implicit-GEMM tiles of ``gemm_core.h`` (``hip`` 128x128, ``hip256``,
``hip64`` 128x64, ``hip_lo`` single-stage), the 3x3 halo-tile kernels of
``conv3x3.hip`` (``hip33``), the direct stem kernels of ``stem.hip`` (``hip_stem``)
and the role-swapped 64-channel weight gradient (``hip64t``); per shape the fastest of
them is picked by measurement (``autotune.choose``).  There is no library path: a device
convolution no hand-written kernel takes raises ``NoKernelError`` (MIOpen / hipBLASLt
comparisons live in the A/B harness ``scripts/vendor_ref.py``).  CPU tensors take the
native OpenMP backend or torch's CPU convolution (the numerics reference).
Reference: ``src/ops/CudnnConv2d.cu:54-245``, ``CudnnConv2dAddBias.cu:93``.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from .. import native_array as _NA

from . import native, no_kernel  # noqa: F401

CL = torch.channels_last


def _masked_store():
    """dgrad epilogues that fuse a BN-backward reduction also store the ReLU-masked
    gradient (HETU_BN_MASKED_STORE=0: plain gradient, the BN backward masks it)"""
    return os.environ.get('HETU_BN_MASKED_STORE', '1') == '1'


def _pick(key, hip, more=None, tuned=None):
    """hip: the default hand-written implicit GEMM; more: other hand-written candidates
    ({name: fn}, timed against it per shape).  ``tuned()`` runs once the choice is made,
    before the call that produces the result (candidates that write in place time against
    scratch until then).  No candidate takes the shape: NoKernelError."""
    from .autotune import choose
    cands = {'hip': hip}
    if more is not None:
        cands.update(more)
    c = choose(key, cands)
    if tuned is not None:
        tuned()
    r = cands[c]()
    if r is None and c != 'hip':
        r = hip()
    if r is None:
        no_kernel('conv_' + key[0], str(key[1:]))
    return r


def _zeros(shape, device, dtype=torch.float32):
    from .tensor import zeros
    return zeros(shape, dtype, device)


def _copy_into(dst, src):
    from .tensor import copy_into
    return copy_into(dst, src)


def _short_k(k):
    """reduction length for which the single-stage, 4-blocks-per-CU tile (tile 3) is a
    candidate: short-K convolutions are bound by their operand / output streams"""
    return k <= 4608


def _add_cl(a, b):
    """a + b for 4-D activations on the native elementwise kernels, channels-last out
    (the NHWC views are dense, so the vector path runs; strided b takes the N-d kernel)"""
    from .elementwise import binary
    if a.dim() == 4 and b.dim() == 4:
        y = binary('add', a.contiguous(memory_format=CL).permute(0, 2, 3, 1), b.permute(0, 2, 3, 1))
        return y.permute(0, 3, 1, 2)
    return binary('add', a, b)


def _plain_1x1(ts, w_shape, stride, padding):
    """1x1 / stride 1 / no padding on channels-last bf16 tensors ``ts``: the
    convolution is a plain GEMM over [pixels, channels] views (no copies)."""
    return (w_shape[2] == 1 and w_shape[3] == 1 and tuple(stride) == (1, 1) and
            tuple(padding) == (0, 0) and
            all(t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous(memory_format=CL) for t in ts))


def _pad_c(t, q=8):
    """Zero-pad dim 1 (channels) of a channels-last tensor to a multiple of ``q`` (8
    bf16 / 4 fp32: one 16-byte chunk) so the implicit-GEMM kernels accept it -- the
    3-channel ResNet stem."""
    n, c, h, w = t.shape
    cp = -(-c // q) * q
    if cp == c:
        return t.contiguous(memory_format=CL)
    buf = _zeros((n, h, w, cp), t.device, t.dtype)
    _copy_into(buf[..., :c], t.permute(0, 2, 3, 1))
    return buf.permute(0, 3, 1, 2)


def _needs_pad(x, w):
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.shape[1] % 8 != 0
            and w.shape[0] % 8 == 0)


def _rows(t):
    """channels-last [N, C, H, W] -> [N*H*W, C] view"""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _match(x, w):
    if x.dtype != w.dtype:
        if w.dtype == torch.bfloat16 or x.dtype == torch.bfloat16:
            x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
        else:
            w = w.to(x.dtype)
    return x, w


def stats_replicas(x_shape, w_shape, stride, padding):
    """replicas of the fused forward BN totals of this convolution's output
    (conv_igemm.bn_sum_replicas of its rows): ``out_sums`` of conv2d_with_stats holds
    that many [2*Cout] copies"""
    from .conv_igemm import bn_sum_replicas
    n, _, h, w_ = x_shape
    oh = (h + 2 * padding[0] - w_shape[2]) // stride[0] + 1
    ow = (w_ + 2 * padding[1] - w_shape[3]) // stride[1] + 1
    return bn_sum_replicas(n * oh * ow)


def conv2d_with_stats(x, w, stride, padding, out_sums=None):
    """(y, sums): the convolution (no bias) and the [2*Cout] per-channel sum / sum of
    squares of y that a following training-mode BatchNorm needs ([R * 2*Cout] replicas,
    R = stats_replicas, folded by the BN forward), fused into the epilogue of every
    hand-written candidate.  ``out_sums``: a zeroed [R * 2*Cout] fp32 buffer the
    fused candidates accumulate into (a persistent one the BN re-zeroes: no fill launch
    per call); fresh zeros otherwise and while the shape is being timed."""
    x, w = _match(x, w)
    if not (x.is_cuda and x.dtype == torch.bfloat16):
        return conv2d(x, w, None, stride, padding), None
    from . import conv_igemm
    x = x.contiguous(memory_format=CL)
    w = w.contiguous(memory_format=CL)
    co = w.shape[0]
    rep = stats_replicas(x.shape, w.shape, stride, padding)
    assert out_sums is None or out_sums.numel() == rep * 2 * co
    key = ('fwd_stats', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(padding))
    from .autotune import _decisions
    tgt = [out_sums if key in _decisions else None]

    def fused(run):
        def f():
            s = tgt[0] if tgt[0] is not None else _zeros(rep * 2 * co, x.device)
            y = run(s)
            return None if y is None else (y, s)
        return f

    cands = {'hip': fused(lambda s: conv_igemm.try_forward(x, w, stride, padding, colstats=s))}
    if co >= 128:
        cands['hip256'] = fused(lambda s: conv_igemm.try_forward(x, w, stride, padding, tile=1, colstats=s))
    if co <= 64:
        cands['hip64'] = fused(lambda s: conv_igemm.try_forward(x, w, stride, padding, tile=2, colstats=s))
    if _short_k(w.shape[1] * w.shape[2] * w.shape[3]):
        cands['hip_lo'] = fused(lambda s: conv_igemm.try_forward(x, w, stride, padding, tile=3, colstats=s))
    if conv_igemm.stem_ok(x, w, stride, padding):
        cands['hip_stem'] = fused(lambda s: conv_igemm.try_stem_forward(x, w, stride, padding, colstats=s))
    if conv_igemm.conv3x3_ok(x.shape, w.shape, stride, padding):
        cands['hip33'] = fused(lambda s: conv_igemm.try_conv3x3_forward(x, w, stride, padding, colstats=s))
    if _needs_pad(x, w):
        cands['hip_pad'] = fused(lambda s: conv_igemm.try_forward(_pad_c(x), _pad_c(w), stride, padding,
                                                                   colstats=s))
    from .autotune import choose
    c = choose(key, cands)
    tgt[0] = out_sums
    r = cands[c]()
    if r is None and c != 'hip':
        r = cands['hip']()
    if r is None:
        no_kernel('conv_fwd_stats', str(key[1:]))
    return r


# ---- fp32 (the reference's only precision): exact-fp32 MFMA implicit GEMM -------------------
# (gemm_f32.hip, v_mfma_f32_16x16x4_f32); channel counts padded to 4 with zeros where needed
def _f32(*ts):
    return all(t is not None and t.is_cuda and t.dtype == torch.float32 for t in ts)


def _fwd_f32(x, w, b, stride, padding):
    from . import conv_igemm
    return conv_igemm.forward_f32(_pad_c(x, 4), _pad_c(w, 4), stride, padding, bias=b)


def _dgrad_f32(g, w, x_shape, stride, padding, acc):
    from . import conv_igemm
    n, c, h, ww = x_shape
    cp = -(-c // 4) * 4
    g = g.contiguous(memory_format=CL)
    if cp == c:
        return conv_igemm.backward_data_f32(g, w.contiguous(memory_format=CL), x_shape, stride, padding, acc=acc)
    d = conv_igemm.backward_data_f32(g, _pad_c(w, 4), (n, cp, h, ww), stride, padding)
    if d is None:
        return None
    d = d[:, :c]
    if acc is not None:
        return _add_cl(acc, d)
    return d.contiguous(memory_format=CL)


def _wgrad_f32(g, x, w_shape, stride, padding, out):
    from . import conv_igemm
    co, c, kh, kw = w_shape
    cp = -(-c // 4) * 4
    g = g.contiguous(memory_format=CL)
    if cp == c:
        return conv_igemm.backward_filter_f32(g, x.contiguous(memory_format=CL), w_shape, stride, padding, out=out,
                                              accumulate=False)
    d = conv_igemm.backward_filter_f32(g, _pad_c(x, 4), (co, cp, kh, kw), stride, padding, accumulate=False)
    if d is None:
        return None
    d = d[:, :c]
    if out is not None:
        _copy_into(out, d)
        return out
    return d.contiguous(memory_format=CL)


def conv2d(x, w, b, stride, padding):
    x, w = _match(x, w)
    from . import cpu_native
    if cpu_native.active(x, w, b) and x.dim() == 4:
        return cpu_native.conv2d(x, w, b, stride, padding)
    if _f32(x, w):
        x = x.contiguous(memory_format=CL)
        w = w.contiguous(memory_format=CL)
        return _pick(('fwd32', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(padding), b is not None),
                     lambda: _fwd_f32(x, w, b, stride, padding))
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            no_kernel('conv_fwd', str(x.dtype))
        x = x.contiguous(memory_format=CL)
        w = w.contiguous(memory_format=CL)
        from . import conv_igemm
        blas = None
        if _needs_pad(x, w):
            blas = {'hip_pad': lambda: conv_igemm.try_forward(_pad_c(x), _pad_c(w), stride, padding)}
            if conv_igemm.stem_ok(x, w, stride, padding):
                blas['hip_stem'] = lambda: conv_igemm.try_stem_forward(x, w, stride, padding)
        if w.shape[0] >= 128:   # 256x256-tile kernel: only with >= half a tile of output channels
            blas = dict(blas or {})
            blas['hip256'] = lambda: conv_igemm.try_forward(x, w, stride, padding, tile=1)
        if w.shape[0] <= 64:    # 128x64 tile: no MFMAs on zero output channels
            blas = dict(blas or {})
            blas['hip64'] = lambda: conv_igemm.try_forward(x, w, stride, padding, tile=2)
        if _short_k(w.shape[1] * w.shape[2] * w.shape[3]):
            blas = dict(blas or {})
            blas['hip_lo'] = lambda: conv_igemm.try_forward(x, w, stride, padding, tile=3)
        if conv_igemm.conv3x3_ok(x.shape, w.shape, stride, padding):
            blas = dict(blas or {})
            blas['hip33'] = lambda: conv_igemm.try_conv3x3_forward(x, w, stride, padding)
        y = _pick(('fwd', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(padding)),
                  lambda: conv_igemm.try_forward(x, w, stride, padding), blas)
        if b is not None:
            from .elementwise import binary
            n, c, h, ww = y.shape
            y = binary('add', y.permute(0, 2, 3, 1), b.to(y.dtype).contiguous()).permute(0, 3, 1, 2)
        return y
    y = F.conv2d(x, w, b.to(x.dtype) if b is not None else None, stride, padding)
    return y


def _scatter_s2(acc, x_shape):
    """[N, C, H/2, W/2] -> [N, C, H, W] with acc at the even positions, zeros elsewhere
    (fallback for the subgrid join when no hand-written kernel takes it)"""
    n, c, h, w = x_shape
    full = _zeros((n, h, w, c), acc.device, acc.dtype).permute(0, 3, 1, 2)     # channels-last
    _copy_into(full[:, :, ::2, ::2], acc)
    return full


def conv2d_backward_data(g, w, x_shape, stride, padding, acc=None, acc_inplace=False, bn=None, acc_s2=False):
    """dx (+ acc when given: a gradient joined at the conv input, fused into the
    epilogue on the HIP path).  ``acc_inplace``: acc is dead after this call and
    may receive the result (the library GEMM accumulates into it, C == D).
    ``bn`` = (sums, x, mask): dx is the gradient of a training BatchNorm's output
    (x: that BN's input, mask: its ReLU keep-bits or None); sums ([2C] fp32, zero)
    receive sum(dx') and sum(dx' * x), the BN backward's reduction -- in the data
    gradient's epilogue on the hand-written kernels, as a pass of its own after a
    library kernel -- and the result carries them as ``hetu_bn_bsums``.  With a mask the
    hand-written kernels store dx' (masked) and flag the result ``hetu_bn_masked``: the
    BN backward then reads no mask, and dx' itself is the residual-branch gradient.
    bf16 on the GPU only (otherwise ignored).
    ``acc_s2``: acc is [N, C, H/2, W/2] -- the data gradient of a 1x1 stride-2
    convolution of the same input, in compact form -- and is added at the even
    positions only (the ResNet downsample join, without scattering that gradient)."""
    if acc_s2:
        if not (g.is_cuda and g.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
                and acc.dtype == torch.bfloat16 and _plain_1x1((g, w), w.shape, stride, padding)
                and x_shape[2] % 2 == 0 and x_shape[3] % 2 == 0):
            return conv2d_backward_data(g, w, x_shape, stride, padding, acc=_scatter_s2(acc, x_shape), bn=bn)
        r, masked = _dgrad_s2join(g, w, x_shape, acc, bn)
        if bn is not None:
            r.hetu_bn_bsums = bn[0]
            r.hetu_bn_masked = masked
        return r
    if bn is not None:
        if not (g.is_cuda and g.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and
                (acc is None or acc.dtype == torch.bfloat16) and bn[1].dtype == torch.bfloat16 and
                bn[1].is_contiguous(memory_format=CL) and x_shape[1] % 8 == 0):
            return conv2d_backward_data(g, w, x_shape, stride, padding, acc, acc_inplace)
        r, masked = _dgrad_bn(g, w, x_shape, stride, padding, acc, acc_inplace, bn)
        r.hetu_bn_bsums = bn[0]
        r.hetu_bn_masked = masked
        return r
    g, w = _match(g, w)
    from . import cpu_native
    if cpu_native.active(g, w, acc):
        dx = cpu_native.conv2d_backward_data(g, w, x_shape, stride, padding)
        return dx + acc.float() if acc is not None else dx
    if _f32(g, w):
        acc32 = acc.contiguous(memory_format=CL) if acc is not None else None
        if acc32 is not None and acc32.dtype != torch.float32:
            acc32 = _copy_into(_NA.empty(tuple(acc32.shape), dtype=torch.float32, device=acc32.device,
                                         memory_format=CL), acc32)
        return _pick(('dgrad32', tuple(g.shape), tuple(w.shape), tuple(x_shape), tuple(stride), tuple(padding),
                      acc is not None),
                     lambda: _dgrad_f32(g, w, x_shape, stride, padding, acc32))
    if g.is_cuda:
        if g.dtype != torch.bfloat16:
            no_kernel('conv_dgrad', str(g.dtype))
        g = g.contiguous(memory_format=CL)
        w = w.contiguous(memory_format=CL)
        if acc is not None:
            acc = acc.contiguous(memory_format=CL)
        from . import conv_igemm
        blas = None
        tuned = None
        if _needs_pad(_NA.empty(0, x_shape[1], 1, 1, dtype=g.dtype, device=g.device), w) and acc is None:
            n, ci, h, ww_ = x_shape
            cp = -(-ci // 8) * 8

            def pad_dgrad():
                d = conv_igemm.try_backward_data(g, _pad_c(w), (n, cp, h, ww_), stride, padding)
                return None if d is None else d[:, :ci]
            blas = {'hip_pad': pad_dgrad}
        if x_shape[1] >= 128:
            blas = dict(blas or {})
            blas['hip256'] = lambda: conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc, tile=1)
        if x_shape[1] <= 64:
            blas = dict(blas or {})
            blas['hip64'] = lambda: conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc, tile=2)
        if _short_k(w.shape[0] * w.shape[2] * w.shape[3]):
            blas = dict(blas or {})
            blas['hip_lo'] = lambda: conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc, tile=3)
        if conv_igemm.conv3x3_ok(x_shape, w.shape, stride, padding, dgrad=True):
            blas = dict(blas or {})
            blas['hip33'] = lambda: conv_igemm.try_conv3x3_backward_data(g, w, x_shape, stride, padding, acc=acc)
        return _pick(('dgrad', tuple(g.shape), tuple(w.shape), tuple(stride), tuple(padding), acc is not None),
                     lambda: conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc), blas, tuned)
    return _ref_dgrad(g, w, x_shape, stride, padding, acc)


def _dgrad_bn(g, w, x_shape, stride, padding, acc, acc_inplace, bn):
    """conv2d_backward_data with the BatchNorm-backward reduction (see there)"""
    from . import conv_igemm
    from .autotune import _decisions
    sums, xb, mask = bn
    g = g.contiguous(memory_format=CL)
    w = w.contiguous(memory_format=CL)
    if acc is not None:
        acc = acc.contiguous(memory_format=CL)
    key = ('dgrad_bn', tuple(g.shape), tuple(w.shape), tuple(stride), tuple(padding), acc is not None)
    # candidates accumulate into scratch while the shape is being timed
    tgt = [sums if key in _decisions else _NA.zeros_like(sums)]
    masked = [False]

    def hip(tile=0):
        def f():
            r = conv_igemm.try_backward_data(g, w, x_shape, stride, padding, acc=acc, tile=tile,
                                             bnb=(tgt[0], xb, mask, _masked_store()))
            masked[0] = r is not None and mask is not None and _masked_store()
            return r
        return f

    blas = {}
    if x_shape[1] >= 128:
        blas['hip256'] = hip(1)
    if x_shape[1] <= 64:
        blas['hip64'] = hip(2)
    if _short_k(w.shape[0] * w.shape[2] * w.shape[3]):
        blas['hip_lo'] = hip(3)
    if conv_igemm.conv3x3_ok(x_shape, w.shape, stride, padding, dgrad=True):
        def hip33():
            r = conv_igemm.try_conv3x3_backward_data(g, w, x_shape, stride, padding, acc=acc,
                                                     bnb=(tgt[0], xb, mask, _masked_store()))
            masked[0] = r is not None and mask is not None and _masked_store()
            return r
        blas['hip33'] = hip33

    def tuned():
        tgt[0] = sums
    r = _pick(key, hip(0), blas, tuned)
    return r, masked[0]


def _dgrad_s2join(g, w, x_shape, acc, bn):
    """1x1 stride-1 data gradient + a compact stride-2 gradient at the even positions
    (conv2d_backward_data acc_s2), optionally with the BN-backward reduction"""
    from . import conv_igemm
    from .autotune import _decisions
    g = g.contiguous(memory_format=CL)
    w = w.contiguous(memory_format=CL)
    acc = acc.contiguous(memory_format=CL)
    key = ('dgrad_s2join', tuple(g.shape), tuple(w.shape), bn is not None)
    tgt = [None]
    if bn is not None:
        tgt[0] = bn[0] if key in _decisions else _NA.zeros_like(bn[0])
    masked = [False]

    def hip(tile):
        def f():
            bnb = None if bn is None else (tgt[0], bn[1], bn[2], _masked_store())
            r = conv_igemm.try_backward_data(g, w, x_shape, (1, 1), (0, 0), acc=acc, tile=tile, bnb=bnb,
                                             acc_s2=True)
            masked[0] = r is not None and bn is not None and bn[2] is not None and _masked_store()
            return r
        return f

    blas = {'hip_lo': hip(3)}
    if x_shape[1] >= 128:
        blas['hip256'] = hip(1)
    if x_shape[1] <= 64:
        blas['hip64'] = hip(2)

    def tuned():
        if bn is not None:
            tgt[0] = bn[0]
    r = _pick(key, hip(0), blas, tuned)
    return r, masked[0]


def _ref_dgrad(g, w, x_shape, stride, padding, acc=None):
    """the CPU reference data gradient (torch's CPU convolution backward)"""
    assert not g.is_cuda
    xs = torch.empty(x_shape, dtype=g.dtype)
    dx, _, _ = torch.ops.aten.convolution_backward(
        g, xs, w, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [True, False, False])
    if acc is not None:
        dx = dx + acc.to(dx.dtype)
    return dx


def conv2d_backward_filter(g, x, w_shape, stride, padding, out=None):
    """Weight gradient.  ``out`` (an fp32 channels-last view, e.g. the
    optimizer's flat gradient slot) receives the result in place."""
    g, x = _match(g, x)
    if out is not None and (out.dtype != torch.float32 or tuple(out.shape) != tuple(w_shape) or
                            not out.is_contiguous(memory_format=CL)):
        out = None
    from . import cpu_native
    if cpu_native.active(g, x):
        dw = cpu_native.conv2d_backward_filter(g, x, w_shape, stride, padding)
        if out is not None:
            _copy_into(out, dw)
            return out
        return dw
    if _f32(g, x):
        # every candidate overwrites ``out`` (no accumulation): timing repeats are harmless
        return _pick(('wgrad32', tuple(g.shape), tuple(x.shape), tuple(w_shape), tuple(stride), tuple(padding)),
                     lambda: _wgrad_f32(g, x, w_shape, stride, padding, out))
    if g.is_cuda:
        if g.dtype != torch.bfloat16:
            no_kernel('conv_wgrad', str(g.dtype))
        g = g.contiguous(memory_format=CL)
        x = x.contiguous(memory_format=CL)
        from . import conv_igemm
        blas = None
        if _needs_pad(x, _NA.empty((g.shape[1], 1, 1, 1), dtype=g.dtype, device=g.device)):
            co, ci, kh, kw = w_shape
            cp = -(-ci // 8) * 8

            def pad_wgrad():
                d = conv_igemm.try_backward_filter(g, _pad_c(x), (co, cp, kh, kw), stride, padding,
                                                   accumulate=False)
                if d is None:
                    return None
                if out is None:
                    return d[:, :ci]
                _copy_into(out, d[:, :ci])
                return out
            blas = {'hip_pad': pad_wgrad}
            if conv_igemm.stem_ok(x, _NA.empty(tuple(w_shape), dtype=g.dtype, device=g.device), stride, padding):
                blas['hip_stem'] = lambda: conv_igemm.try_stem_backward_filter(g, x, w_shape, stride, padding,
                                                                               out=out)
        if w_shape[0] >= 128:
            blas = dict(blas or {})
            blas['hip256'] = lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                                    accumulate=False, tile=1)
        if _plain_1x1((g, x), w_shape, stride, padding) and w_shape[0] % 64 == 0 and w_shape[1] % 64 == 0:
            from . import gemm_mfma
            co, ci = w_shape[0], w_shape[1]

            def lk():
                d = out.reshape(co, ci) if out is not None else _NA.empty((co, ci), dtype=torch.float32,
                                                                            device=g.device)
                r = gemm_mfma.wgrad_longk(_rows(g), _rows(x), d)
                if r is None:
                    return None
                return out if out is not None else d.view(co, ci, 1, 1)
            blas = dict(blas or {})
            blas['hip_lk'] = lk
        if w_shape[0] <= 64:   # 64-channel banks: a 64-wide N side (as is, and with the roles swapped)
            blas = dict(blas or {})
            blas['hip64'] = lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                                   accumulate=False, tile=2)
            blas['hip64t'] = lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                                    accumulate=False, tile=4)
        # the single-stage tile (4 blocks per CU) on the long pixel reduction
        blas = dict(blas or {})
        blas['hip_lo'] = lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                                accumulate=False, tile=3)
        if conv_igemm._s1p1_3x3(w_shape, stride, padding) and conv_igemm.conv3x3_wgrad_ok(x.shape, w_shape):
            blas = dict(blas or {})
            blas['hip33'] = lambda: conv_igemm.try_conv3x3_backward_filter(g, x, w_shape, stride, padding, out=out)
        return _pick(('wgrad', tuple(g.shape), tuple(x.shape), tuple(w_shape), tuple(stride), tuple(padding)),
                     lambda: conv_igemm.try_backward_filter(g, x, w_shape, stride, padding, out=out,
                                                            accumulate=False), blas)
    ws = torch.empty(w_shape, dtype=g.dtype)
    _, dw, _ = torch.ops.aten.convolution_backward(       # the CPU reference
        g, x, ws, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [False, True, False])
    if out is not None:
        _copy_into(out, dw)
        return out
    return dw
