"""Implicit-GEMM MFMA convolution (``csrc/kernels/gemm.hip``), NHWC bf16.

forward  : M = N*OH*OW pixels, N = Cout, K = KH*KW*Cin (im2col on the fly)
dgrad    : M = N*H*W pixels,  N = Cin,  K = KH*KW*Cout (stride handled by
           zero-filling the taps that do not hit an output pixel)
wgrad    : M = Cout, N = KH*KW*Cin, K = N*OH*OW, split-K with fp32 atomics
           straight into an fp32 gradient.

Shapes with Cin or Cout not a multiple of 8 (the 3-channel stem) return None; the caller
(kernels/conv.py) then takes a zero-padded or a direct (stem) hand-written kernel.
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import fn, stream_ptr, check, record_native, P, I32, I64

CL = torch.channels_last
_GEOM = [I32] * 11


def _ok(a, b, *channels):
    return (a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and
            a.is_contiguous(memory_format=CL) and b.is_contiguous(memory_format=CL) and
            all(c % 8 == 0 for c in channels) and a.data_ptr() % 16 == 0 and
            b.data_ptr() % 16 == 0)


def _ok32(a, b, *channels):
    """fp32 operands for the exact-fp32 MFMA convolution (gemm_f32.hip): channels-last,
    16-byte aligned, channel counts multiples of 4 (16-byte chunks of 4 floats)."""
    return (a.dtype == torch.float32 and b.dtype == torch.float32 and
            a.is_contiguous(memory_format=CL) and b.is_contiguous(memory_format=CL) and
            all(c % 4 == 0 for c in channels) and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def forward_f32(x, w, stride, padding, bias=None, act=None):
    """fp32 forward on the 16x16x4-f32 MFMA kernel; None when unsupported."""
    if not _ok32(x, w, x.shape[1], w.shape[0]):
        return None
    N, C, H, W = x.shape
    K, _, KH, KW = w.shape
    OH, OW = _out_hw(H, W, KH, KW, stride, padding)
    y = _NA.empty((N, OH, OW, K), dtype=torch.float32, device=x.device)
    f = fn('hetu_conv_fwd_f32', [P, P, P, P] + _GEOM + [I32, P])
    check(f(x.data_ptr(), w.data_ptr(), y.data_ptr(), bias.float().contiguous().data_ptr() if bias is not None
            else None, N, H, W, C, K, KH, KW, stride[0], stride[1], padding[0], padding[1],
            {None: 0, 'relu': 1}[act], stream_ptr()), 'conv_fwd_f32')
    record_native('conv_fwd_f32')
    return y.permute(0, 3, 1, 2)


def backward_data_f32(g, w, x_shape, stride, padding, acc=None):
    if not _ok32(g, w, x_shape[1], w.shape[0]):
        return None
    if acc is not None and (tuple(acc.shape) != tuple(x_shape) or acc.dtype != torch.float32 or
                            not acc.is_contiguous(memory_format=CL)):
        return None
    N, C, H, W = x_shape
    K, _, KH, KW = w.shape
    dx = _NA.empty((N, H, W, C), dtype=torch.float32, device=g.device)
    f = fn('hetu_conv_dgrad_f32', [P, P, P, P] + _GEOM + [P])
    check(f(g.data_ptr(), w.data_ptr(), dx.data_ptr(), acc.data_ptr() if acc is not None else None,
            N, H, W, C, K, KH, KW, stride[0], stride[1], padding[0], padding[1], stream_ptr()), 'conv_dgrad_f32')
    record_native('conv_dgrad_f32')
    return dx.permute(0, 3, 1, 2)


def backward_filter_f32(g, x, w_shape, stride, padding, out=None, accumulate=None):
    if not _ok32(x, g, x.shape[1], g.shape[1]):
        return None
    N, C, H, W = x.shape
    K, _, KH, KW = w_shape
    if accumulate is None:
        accumulate = out is not None
    if out is None:
        dw = _NA.empty((K, KH, KW, C), dtype=torch.float32, device=g.device)
    else:
        dw = out.permute(0, 2, 3, 1)
        if not dw.is_contiguous() or dw.dtype != torch.float32:
            return None
    f = fn('hetu_conv_wgrad_f32', [P, P, P] + _GEOM + [I32, P])
    check(f(g.data_ptr(), x.data_ptr(), dw.data_ptr(), N, H, W, C, K, KH, KW, stride[0], stride[1],
            padding[0], padding[1], int(bool(accumulate)), stream_ptr()), 'conv_wgrad_f32')
    record_native('conv_wgrad_f32')
    return dw.permute(0, 3, 1, 2)


def _out_hw(H, W, KH, KW, stride, padding):
    return (H + 2 * padding[0] - KH) // stride[0] + 1, (W + 2 * padding[1] - KW) // stride[1] + 1


def _reps(colstats, co):
    return colstats.numel() // (2 * co) if colstats is not None else 0


def try_forward(x, w, stride, padding, bias=None, act=None, tile=0, colstats=None):
    """``colstats`` ([R * 2*Cout] fp32, zeroed): receives the per-channel sum and sum of
    squares of the stored output (BatchNorm statistics fused into the epilogue), spread
    over R replicas (bn_sum_replicas; the BN forward folds them)."""
    if not _ok(x, w, x.shape[1], w.shape[0]):
        return None
    N, C, H, W = x.shape
    K, _, KH, KW = w.shape
    OH, OW = _out_hw(H, W, KH, KW, stride, padding)
    y = _NA.empty((N, OH, OW, K), dtype=torch.bfloat16, device=x.device)
    f = fn('hetu_conv_fwd_bf16', [P, P, P, P] + _GEOM + [I32, P, I32, I32, P])
    check(f(x.data_ptr(), w.data_ptr(), y.data_ptr(),
            bias.float().contiguous().data_ptr() if bias is not None else None,
            N, H, W, C, K, KH, KW, stride[0], stride[1], padding[0], padding[1],
            {None: 0, 'relu': 1}[act], colstats.data_ptr() if colstats is not None else None, int(tile),
            _reps(colstats, K), stream_ptr()), 'conv_fwd')
    record_native('conv_fwd')
    return y.permute(0, 3, 1, 2)


def stem_ok(x, w, stride, padding):
    """the direct few-channel stem kernel (``stem.hip``) takes this convolution"""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    co, c, kh, kw = w.shape
    return (co == 64 and kw * c <= 24 and kh <= 8 and stride[0] == stride[1] and padding[0] == padding[1]
            and (stride[0] * c) % 2 == 0 and x.shape[1] == c)


def try_stem_forward(x, w, stride, padding, colstats=None):
    """Direct convolution of a few-channel input (ResNet conv1: 3 channels, 7x7/2) without
    padding the channels to the 8-wide chunks of the implicit-GEMM kernels."""
    if not stem_ok(x, w, stride, padding):
        return None
    x = x.contiguous(memory_format=CL)
    w = w.contiguous(memory_format=CL)
    N, C, H, W = x.shape
    K, _, KH, KW = w.shape
    OH, OW = _out_hw(H, W, KH, KW, stride, padding)
    wp = _NA.empty(fn('hetu_stem_wp_elems', [I32], restype=I64)(KH), dtype=torch.bfloat16, device=x.device)
    y = _NA.empty((N, OH, OW, K), dtype=torch.bfloat16, device=x.device)
    f = fn('hetu_stem_fwd', [P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, I32, P])
    check(f(x.data_ptr(), w.data_ptr(), wp.data_ptr(), y.data_ptr(),
            colstats.data_ptr() if colstats is not None else None, N, H, W, C, KH, KW, stride[0], padding[0],
            _reps(colstats, K), stream_ptr()), 'stem_fwd')
    record_native('stem_fwd')
    return y.permute(0, 3, 1, 2)


def _s1p1_3x3(w_shape, stride, padding):
    return tuple(w_shape[2:]) == (3, 3) and tuple(stride) == (1, 1) and tuple(padding) == (1, 1)


def _c64(C, K, W):
    return bool(fn('hetu_conv3x3_c64_supported', [I32, I32, I32])(int(C), int(K), int(W)))


def _wide(C, K, H, W):
    return bool(fn('hetu_conv3x3_wide_supported', [I32, I32, I32, I32])(int(C), int(K), int(H), int(W)))


def conv3x3_ok(shape_x, w_shape, stride, padding, dgrad=False):
    """a halo-tile kernel (``conv3x3.hip``) takes this 3x3/s1/p1 pass: the 64-channel
    image-walking kernel, or the wide-channel pixel-tile kernel (its output channels in
    128-blocks: K for the forward, C for the data gradient)"""
    co, c = w_shape[0], w_shape[1]
    if not _s1p1_3x3(w_shape, stride, padding):
        return False
    H, W = int(shape_x[2]), int(shape_x[3])
    if _c64(c, co, W):
        return True
    return _wide(co, c, H, W) if dgrad else _wide(c, co, H, W)


def conv3x3_wgrad_ok(shape_x, w_shape):
    C, H, W = int(shape_x[1]), int(shape_x[2]), int(shape_x[3])
    K = int(w_shape[0])
    return _c64(C, K, W) or bool(fn('hetu_conv3x3_wide_wgrad_supported', [I32, I32, I32, I32])(C, K, H, W))


def try_conv3x3_forward(x, w, stride, padding, colstats=None):
    """3x3 / stride 1 / pad 1 on a halo-tile kernel: each input pixel crosses L2 once per
    block instead of once per tap.  64 -> 64 channels: one block per image, the filter
    bank resident in LDS and a DMA ring of halo rows; wider layers: pixel tiles x 128
    output channels, a halo per 64-channel chunk serving all 9 taps."""
    if not (_ok(x, w, x.shape[1], w.shape[0]) and conv3x3_ok(x.shape, w.shape, stride, padding)):
        return None
    N, C, H, W = x.shape
    K = w.shape[0]
    y = _NA.empty((N, H, W, K), dtype=torch.bfloat16, device=x.device)
    st = colstats.data_ptr() if colstats is not None else None
    if _c64(C, K, W):
        f = fn('hetu_conv3x3_c64_fwd', [P, P, P, P, I32, I32, I32, I32, P])
        check(f(x.data_ptr(), w.data_ptr(), y.data_ptr(), st, N, H, W, _reps(colstats, K), stream_ptr()),
              'conv3x3_fwd')
    else:
        f = fn('hetu_conv3x3_wide_fwd', [P, P, P, P, I32, I32, I32, I32, I32, I32, P])
        check(f(x.data_ptr(), w.data_ptr(), y.data_ptr(), st, N, H, W, C, K, _reps(colstats, K), stream_ptr()),
              'conv3x3_wide_fwd')
    record_native('conv3x3_fwd')
    return y.permute(0, 3, 1, 2)


def try_conv3x3_backward_data(g, w, x_shape, stride, padding, acc=None, bnb=None):
    if not (_ok(g, w, x_shape[1], w.shape[0]) and conv3x3_ok(x_shape, w.shape, stride, padding, dgrad=True)):
        return None
    if acc is not None and (tuple(acc.shape) != tuple(x_shape) or not acc.is_contiguous(memory_format=CL) or
                            acc.dtype not in (torch.bfloat16, torch.float32) or acc.data_ptr() % 16):
        return None
    bn = _bnb_args(bnb, x_shape)
    if bn is False:
        return None
    N, C, H, W = x_shape
    K = w.shape[0]
    dx = _NA.empty((N, H, W, C), dtype=torch.bfloat16, device=g.device)
    wt = _NA.empty(w.numel(), dtype=torch.bfloat16, device=g.device)
    a = acc.data_ptr() if acc is not None else None
    af = int(acc is not None and acc.dtype == torch.float32)
    if _c64(C, K, W):
        f = fn('hetu_conv3x3_c64_dgrad', [P, P, P, P, P, I32, I32, I32, I32, P, P, P, I32, I32, P])
        check(f(g.data_ptr(), w.data_ptr(), wt.data_ptr(), dx.data_ptr(), a, af, N, H, W, *bn, stream_ptr()),
              'conv3x3_dgrad')
    else:
        f = fn('hetu_conv3x3_wide_dgrad', [P, P, P, P, P, I32, I32, I32, I32, I32, I32, P, P, P, I32, I32, P])
        check(f(g.data_ptr(), w.data_ptr(), wt.data_ptr(), dx.data_ptr(), a, af, N, H, W, C, K, *bn,
                stream_ptr()), 'conv3x3_wide_dgrad')
    record_native('conv3x3_dgrad')
    return dx.permute(0, 3, 1, 2)


def try_conv3x3_backward_filter(g, x, w_shape, stride, padding, out=None, accumulate=False):
    """weight gradient of the 64-channel 3x3/s1/p1 convolution on the halo-tile kernel
    (per-image fp32 partials in a slab, then one reduce) into ``out`` (fp32 channels-last
    [K, C, 3, 3] view) or a new tensor"""
    if not (_ok(x, g, x.shape[1], g.shape[1]) and _s1p1_3x3(w_shape, stride, padding) and
            conv3x3_wgrad_ok(x.shape, w_shape)):
        return None
    N, C, H, W = x.shape
    K = w_shape[0]
    if out is None:
        dw = _NA.empty((K, 3, 3, C), dtype=torch.float32, device=g.device)
        accumulate = False
    else:
        dw = out.permute(0, 2, 3, 1)
        if not dw.is_contiguous() or dw.dtype != torch.float32 or dw.data_ptr() % 16:
            return None
    if _c64(C, K, W):
        ws = _NA.empty(int(fn('hetu_conv3x3_c64_wgrad_ws', [I32], restype=I64)(N)), dtype=torch.float32,
                         device=g.device)
        f = fn('hetu_conv3x3_c64_wgrad', [P, P, P, P, I32, I32, I32, I32, P])
        check(f(x.data_ptr(), g.data_ptr(), dw.data_ptr(), ws.data_ptr(), int(bool(accumulate)), N, H, W,
                stream_ptr()), 'conv3x3_wgrad')
    else:
        nws = int(fn('hetu_conv3x3_wide_wgrad_ws', [I32, I32], restype=I64)(C, K))
        ws = _NA.empty(nws, dtype=torch.float32, device=g.device)
        f = fn('hetu_conv3x3_wide_wgrad', [P, P, P, P, I64, I32, I32, I32, I32, I32, I32, P])
        check(f(x.data_ptr(), g.data_ptr(), dw.data_ptr(), ws.data_ptr(), nws, int(bool(accumulate)), N, H, W, C, K,
                stream_ptr()), 'conv3x3_wide_wgrad')
    record_native('conv3x3_wgrad')
    return dw.permute(0, 3, 1, 2)


STEM_WGRAD_BLOCKS = 512


def try_stem_backward_filter(g, x, w_shape, stride, padding, out=None, accumulate=False):
    """Weight gradient of the few-channel stem (``stem.hip``: transpose-read MFMA over
    LDS-staged input rows, per-block fp32 partials + one reduce) into ``out`` (fp32,
    channels-last [Cout, C, KH, KW] view) or a new tensor."""
    co, c, kh, kw = w_shape
    if not (co == 64 and kw * c <= 24 and kh * 24 <= 176 and stride[0] == stride[1] and padding[0] == padding[1]
            and (stride[0] * c) % 2 == 0 and x.shape[1] == c and x.dtype == torch.bfloat16
            and g.dtype == torch.bfloat16 and g.shape[1] == co):
        return None
    x = x.contiguous(memory_format=CL)
    g = g.contiguous(memory_format=CL)
    N, C, H, W = x.shape
    OW = (W + 2 * padding[1] - kw) // stride[1] + 1
    # the kernel stages 16-byte pieces of input rows (W*C % 8) and of 2 dy rows per task
    if (W * C) % 8 or (stride[0] + kh) * (W * C // 8) > 1024 or 2 * OW * 8 > 2048 or x.data_ptr() % 16 \
            or g.data_ptr() % 16:
        return None
    if out is None:
        dw = _NA.empty((co, kh, kw, c), dtype=torch.float32, device=g.device)
        accumulate = False
    else:
        dw = out.permute(0, 2, 3, 1)
        if not dw.is_contiguous() or dw.dtype != torch.float32:
            return None
    nb = STEM_WGRAD_BLOCKS
    ws = _NA.empty(int(fn('hetu_stem_wgrad_ws', [I32], restype=I64)(nb)), dtype=torch.float32, device=g.device)
    f = fn('hetu_stem_wgrad', [P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P])
    check(f(x.data_ptr(), g.data_ptr(), dw.data_ptr(), ws.data_ptr(), nb, N, H, W, C, kh, kw, stride[0], padding[0],
            int(bool(accumulate)), stream_ptr()), 'stem_wgrad')
    record_native('stem_wgrad')
    return dw.permute(0, 3, 1, 2)


def _bnb_args(bnb, x_shape):
    """(sums ptr, x ptr, mask ptr, store, replicas) of a BatchNorm-backward reduction fused
    into a data-gradient epilogue: ``bnb`` = (sums [R * 2C] fp32 zeroed, BN input x (bf16,
    channels-last, the gradient's shape), ReLU keep-bit mask or None[, store]) -- store:
    the gradient is stored masked; R replicas of the [2C] totals spread the blocks'
    atomics (bn_sum_replicas; the BN backward folds them); False when the operands do not
    fit the epilogue"""
    if bnb is None:
        return None, None, None, 0, 0
    sums, x, mask = bnb[:3]
    store = bool(bnb[3]) if len(bnb) > 3 else False
    N, C, H, W = x_shape
    if (tuple(x.shape) != tuple(x_shape) or x.dtype != torch.bfloat16 or not x.is_contiguous(memory_format=CL)
            or x.data_ptr() % 16 or C % 8 or sums.numel() % (2 * C) or sums.dtype != torch.float32
            or (mask is not None and mask.numel() != x.numel() // 8)):
        return False
    return (sums.data_ptr(), x.data_ptr(), mask.data_ptr() if mask is not None else None, int(store and mask is not None),
            sums.numel() // (2 * C))


def bn_sum_replicas(M):
    """replicas of the fused BN-backward totals for M gradient rows: about 64 blocks of 128
    rows per replica (thousands of blocks adding into one [2C] serialise on it), at most 64"""
    return max(1, min(64, M // 8192))


def try_backward_data(g, w, x_shape, stride, padding, acc=None, tile=0, bnb=None, acc_s2=False):
    """``bnb``: see _bnb_args -- the sums receive sum(dx') and sum(dx' * x).
    ``acc_s2``: acc is [N, C, H/2, W/2], added at the even positions only (a 1x1
    stride-2 convolution's data gradient joined without scattering it)"""
    if not _ok(g, w, x_shape[1], w.shape[0]):
        return None
    acc_shape = tuple(x_shape) if not acc_s2 else (x_shape[0], x_shape[1], x_shape[2] // 2, x_shape[3] // 2)
    if acc is not None and (tuple(acc.shape) != acc_shape or
                            not acc.is_contiguous(memory_format=CL) or
                            acc.dtype not in (torch.bfloat16, torch.float32)):
        return None
    if acc_s2 and (acc is None or x_shape[2] % 2 or x_shape[3] % 2):
        return None
    bn = _bnb_args(bnb, x_shape)
    if bn is False:
        return None
    N, C, H, W = x_shape
    K, _, KH, KW = w.shape
    dx = _NA.empty((N, H, W, C), dtype=torch.bfloat16, device=g.device)
    f = fn('hetu_conv_dgrad_bf16', [P, P, P, P, I32] + _GEOM + [I32, P, P, P, I32, I32, I32, P])
    check(f(g.data_ptr(), w.data_ptr(), dx.data_ptr(), acc.data_ptr() if acc is not None else None,
            int(acc is not None and acc.dtype == torch.float32), N, H, W, C, K, KH, KW,
            stride[0], stride[1], padding[0], padding[1], int(tile), *bn[:4], int(acc_s2), bn[4], stream_ptr()),
          'conv_dgrad')
    record_native('conv_dgrad')
    return dx.permute(0, 3, 1, 2)


def _splitk(M, Nc, P_, tile=0):
    name = 'hetu_gemm_pick_splitk_big' if tile == 1 else 'hetu_gemm_pick_splitk'
    return int(fn(name, [I64, I64, I64])(M, Nc, P_))


def try_backward_filter(g, x, w_shape, stride, padding, out=None, accumulate=None, tile=0):
    """Returns the fp32 weight gradient (channels-last) written into ``out`` when
    given: accumulated onto its contents (default) or overwriting them
    (``accumulate=False``)."""
    if not _ok(x, g, x.shape[1], g.shape[1]):
        return None
    N, C, H, W = x.shape
    K, _, KH, KW = w_shape
    OH, OW = g.shape[2], g.shape[3]
    if accumulate is None:
        accumulate = out is not None
    if out is None:
        dw = _NA.empty((K, KH, KW, C), dtype=torch.float32, device=g.device)
    else:
        dw = out.permute(0, 2, 3, 1)
        assert dw.is_contiguous() and dw.dtype == torch.float32
    Nc = KH * KW * C
    if tile == 4 and K > 64:
        return None
    # tile 4 (roles swapped): M = Nc taps on 128-row tiles, N = K channels on 64-col tiles
    sk = _splitk(Nc, 2 * K, N * OH * OW, 0) if tile == 4 else _splitk(K, Nc, N * OH * OW, tile)
    ws = _NA.empty(sk * K * Nc, dtype=torch.float32, device=g.device) if (sk > 1 or tile == 4) else None
    # a single slice without accumulation stores straight into dw (plain fp32 epilogue,
    # no zero fill + atomics)
    f = fn('hetu_conv_wgrad_bf16', [P, P, P] + _GEOM + [I32, I32, P, I32, P])
    check(f(g.data_ptr(), x.data_ptr(), dw.data_ptr(), N, H, W, C, K, KH, KW, stride[0], stride[1],
            padding[0], padding[1], sk, int(accumulate), ws.data_ptr() if ws is not None else None,
            int(tile), stream_ptr()), 'conv_wgrad')
    record_native('conv_wgrad')
    return dw.permute(0, 3, 1, 2)
