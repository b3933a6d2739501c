"""GEMM entry points (reference ``src/ops/MatrixMult.cu:22``, ``BatchMatrixMult.cu:31-36``,
``Linear.cu:50-55``, ``Addmm.cu:29``).

``matmul(a, b, ta, tb, bias, activation)``: 2-D product with optional fused bias and
ReLU/GELU epilogue.  On the GPU every product runs on a hand-written MFMA kernel
(``gemm.hip``: 128x128 / 256x256 / 128x96 tiles, LDS double buffer or two-ahead K loop,
hardware transpose reads for MN-contiguous operands, XCD-aware block remap, fused
epilogues, split-K, a one-wave-per-output kernel for tiny products, zero-padded aligned
operands as the last resort), the candidates timed against each other per shape.  There
is no library path: a device product no hand-written kernel takes raises
``NoKernelError``.  The vendor GEMMs live in the A/B harnesses (``scripts/vendor_ref.py``,
``csrc/bench/gemm_bench.hip``).  CPU tensors take the native OpenMP backend or torch's
CPU GEMM (the numerics reference).
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import native, no_kernel


def _sig(t):
    return (tuple(t.shape), tuple(t.stride()), t.dtype)


def _match(a, b):
    if a.dtype != b.dtype:
        dt = torch.bfloat16 if torch.bfloat16 in (a.dtype, b.dtype) else torch.float32
        return _as_dtype(a, dt), _as_dtype(b, dt)
    return a, b


def _tr(t, f):
    return t.transpose(-1, -2) if f else t


def matmul_pre(a, b, ta, tb, bias, activation):
    """(act(op(a) @ op(b) + bias), the pre-activation) -- one GEMM epilogue storing both
    when a bf16 MFMA tile takes the shape (autotuned per shape like ``matmul``), else the
    plain GEMM plus a separate activation pass."""
    a, b = _match(a, b)
    A2, B2 = _tr(a, ta), _tr(b, tb)
    if native(a) and a.dtype == torch.bfloat16 and A2.dim() in (2, 3):
        from . import gemm_mfma
        from .autotune import choose
        shape = tuple(A2.shape[:-1]) + (B2.shape[-1],)
        pre = _NA.empty(shape, dtype=torch.bfloat16, device=a.device)

        def cand(tile):
            return lambda: gemm_mfma.gemm(A2, B2, bias=bias, act=activation, tile=tile, pre_out=pre)
        cands = {'hip': cand(0)}
        if A2.dim() == 2 and _big_ok(a, b, ta, tb):
            cands['hip256'] = cand(1)
        if A2.shape[-1] <= 2048:
            cands['hip_lo'] = cand(3)
        if B2.shape[-1] % 96 == 0 and A2.shape[-2] >= 1024:
            cands['hip96'] = cand(5)
        if A2.shape[-1] >= 3 * 64:
            cands['hip_2a'] = cand(6)
            if B2.shape[-1] % 96 == 0 and A2.shape[-2] >= 1024:
                cands['hip96_2a'] = cand(7)
        key = ('gemm_pre', _sig(a), _sig(b), ta, tb, bias is not None, activation)
        c = choose(key, cands, 'hip')
        y = cands[c]()
        if y is None and c != 'hip':
            y = cands['hip']()
        if y is not None:
            return y, pre
    from .elementwise import unary
    pre = matmul(a, b, ta, tb, bias=bias)
    return unary(activation, pre), pre


def matmul_act_dropout(a, b, activation, keep, seed):
    """dropout(act(a @ b)) (bf16, 2-D) with the activation and the dropout -- the standalone
    dropout kernel's Philox counters over the output -- in the GEMM epilogue; tiles autotuned
    per shape.  Elsewhere: the plain GEMM with the activation epilogue, then the dropout kernel."""
    a, b = _match(a, b)
    if native(a) and a.dtype == torch.bfloat16 and a.dim() == 2 \
            and keep < 1.0 and b.shape[-1] % 8 == 0:
        from . import gemm_mfma
        from .autotune import choose

        def cand(tile):
            return lambda: gemm_mfma.gemm(a, b, act=activation, tile=tile, drop=(keep, seed))
        cands = {'hip': cand(0)}
        if _big_ok(a, b, False, False):
            cands['hip256'] = cand(1)
        if a.shape[-1] <= 2048:
            cands['hip_lo'] = cand(3)
        if b.shape[-1] % 96 == 0 and a.shape[0] >= 1024:
            cands['hip96'] = cand(5)
        if a.shape[-1] >= 3 * 64:
            cands['hip_2a'] = cand(6)
            if b.shape[-1] % 96 == 0 and a.shape[0] >= 1024:
                cands['hip96_2a'] = cand(7)
        c = choose(('gemm_drop', _sig(a), _sig(b), activation), cands, 'hip')
        y = cands[c]()
        if y is None and c != 'hip':
            y = cands['hip']()
        if y is not None:
            return y
    y = matmul(a, b, activation=activation)
    if keep < 1.0:
        from .dropout import dropout
        y = dropout(y, keep, seed)
    return y


def matmul_relu_mask(a, b, ta, tb, g, scale):
    """(op(a) @ op(b)) * scale where g > 0, else 0: a ReLU (+ dropout) backward fused into the
    data-gradient GEMM (bf16, 2-D; tiles autotuned per shape), else the GEMM and the
    ``relu_grad_c`` elementwise kernel."""
    a, b = _match(a, b)
    A2, B2 = _tr(a, ta), _tr(b, tb)
    if native(a) and a.dtype == torch.bfloat16 and A2.dim() == 2 \
            and g.dtype == torch.bfloat16 and g.is_contiguous():
        from . import gemm_mfma
        from .autotune import choose

        def cand(tile):
            return lambda: gemm_mfma.gemm_gmask(A2, B2, g, scale, tile=tile)
        cands = {'hip': cand(0)}
        if _big_ok(a, b, ta, tb):
            cands['hip256'] = cand(1)
        if A2.shape[-1] <= 2048:
            cands['hip_lo'] = cand(3)
        if A2.shape[-1] >= 3 * 64:
            cands['hip_2a'] = cand(6)
        c = choose(('gemm_gmask', _sig(a), _sig(b), ta, tb), cands, 'hip')
        y = cands[c]()
        if y is None and c != 'hip':
            y = cands['hip']()
        if y is not None:
            return y
    from .elementwise import binary
    y = matmul(a, b, ta, tb)
    return binary('relu_grad_c', g.contiguous(), y.contiguous(), float(scale))


def matmul_act_dropout_bits(a, b, activation, keep, seed):
    """(y, mask): ``matmul_act_dropout`` and the mask its backward reads -- uint8 keep bits
    (one byte per 8 outputs) from the same epilogue on the native bf16 path, else y itself
    (its positive elements are the kept ones)"""
    a, b = _match(a, b)
    if native(a) and a.dtype == torch.bfloat16 and a.dim() == 2 \
            and keep < 1.0 and b.shape[-1] % 8 == 0:
        from . import gemm_mfma
        from .autotune import choose

        def cand(tile):
            return lambda: gemm_mfma.gemm_drop_bits(a, b, activation, keep, seed, tile=tile)
        cands = {'hip': cand(0)}
        if _big_ok(a, b, False, False):
            cands['hip256'] = cand(1)
        if a.shape[-1] <= 2048:
            cands['hip_lo'] = cand(3)
        if b.shape[-1] % 96 == 0 and a.shape[0] >= 1024:
            cands['hip96'] = cand(5)
        if a.shape[-1] >= 3 * 64:
            cands['hip_2a'] = cand(6)
            if b.shape[-1] % 96 == 0 and a.shape[0] >= 1024:
                cands['hip96_2a'] = cand(7)
        c = choose(('gemm_dropb', _sig(a), _sig(b), activation), cands, 'hip')
        r = cands[c]()
        if r is None and c != 'hip':
            r = cands['hip']()
        if r is not None:
            return r
    y = matmul_act_dropout(a, b, activation, keep, seed)
    return y, y


def matmul_mask(a, b, ta, tb, mask, scale):
    """``matmul_relu_mask`` with the mask of ``matmul_act_dropout_bits``: keep bits (uint8)
    read by the GEMM epilogue, or the bf16 forward output"""
    if mask.dtype != torch.uint8:
        return matmul_relu_mask(a, b, ta, tb, mask.contiguous(), scale)
    a, b = _match(a, b)
    A2, B2 = _tr(a, ta), _tr(b, tb)
    if native(a) and a.dtype == torch.bfloat16 and A2.dim() == 2:
        from . import gemm_mfma
        from .autotune import choose

        def cand(tile):
            return lambda: gemm_mfma.gemm_gbits(A2, B2, mask, scale, tile=tile)
        cands = {'hip': cand(0)}
        if _big_ok(a, b, ta, tb):
            cands['hip256'] = cand(1)
        if A2.shape[-1] <= 2048:
            cands['hip_lo'] = cand(3)
        if A2.shape[-1] >= 3 * 64:
            cands['hip_2a'] = cand(6)
        c = choose(('gemm_gbits', _sig(a), _sig(b), ta, tb), cands, 'hip')
        y = cands[c]()
        if y is None and c != 'hip':
            y = cands['hip']()
        if y is not None:
            return y
    y = matmul(a, b, ta, tb)
    keep = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    return torch.where(keep.view(y.shape).bool(), y * scale, torch.zeros((), dtype=y.dtype, device=y.device))


def matmul(a, b, ta=False, tb=False, bias=None, activation=None):
    a, b = _match(a, b)
    from . import cpu_native
    if cpu_native.active(a, b, bias) and a.dim() == 2 and b.dim() == 2 and activation in (None, 'relu', 'gelu'):
        y = cpu_native.gemm(_tr(a, ta), _tr(b, tb), bias)
        return cpu_native.unary(activation, y) if activation else y
    if not a.is_cuda:
        return _cpu_matmul(a, b, ta, tb, bias, activation)
    if not (native(a) and a.dtype in (torch.bfloat16, torch.float32)):
        no_kernel('matmul', '%s %s' % (a.dtype, tuple(a.shape)))
    from . import gemm_mfma
    from .autotune import choose, _decisions
    key = ('gemm', _sig(a), _sig(b), ta, tb, bias is not None, activation)
    d = _decisions.get(key)
    if d is not None:
        # decided shape: run the chosen tile directly (building every candidate closure
        # per call cost more host time than the launch on the launch-bound models)
        y = _run_decided(gemm_mfma, d, a, b, ta, tb, bias, activation)
        if y is not None:
            return y
    cands = {'hip': lambda: gemm_mfma.try_gemm(a, b, ta, tb, bias, activation)}
    if a.dtype == torch.bfloat16 and _big_ok(a, b, ta, tb):
        cands['hip256'] = lambda: gemm_mfma.gemm(_tr(a, ta), _tr(b, tb), bias=bias, act=activation, tile=1)
    if a.dtype == torch.bfloat16 and _tr(b, tb).shape[-1] <= 64:
        cands['hip64'] = lambda: gemm_mfma.gemm(_tr(a, ta), _tr(b, tb), bias=bias, act=activation, tile=2)
    if a.dtype == torch.bfloat16 and _tr(a, ta).shape[-1] <= 2048:   # short K: the 4-blocks-per-CU tile
        cands['hip_lo'] = lambda: gemm_mfma.gemm(_tr(a, ta), _tr(b, tb), bias=bias, act=activation, tile=3)
    A2, B2 = _tr(a, ta), _tr(b, tb)
    if a.dtype == torch.bfloat16 and B2.shape[-1] % 96 == 0 and A2.shape[-2] >= 1024:
        # 128x96 tile: N = 768 products fill the CUs in one round (512 tiles at M 8192)
        cands['hip96'] = lambda: gemm_mfma.gemm(A2, B2, bias=bias, act=activation, tile=5)
    if a.dtype == torch.bfloat16 and A2.shape[-1] >= 3 * 64:
        # two-ahead K loop (operand DMA two K-tiles ahead of the MFMAs)
        cands['hip_2a'] = lambda: gemm_mfma.gemm(A2, B2, bias=bias, act=activation, tile=6)
        if B2.shape[-1] % 96 == 0 and A2.shape[-2] >= 1024:
            cands['hip96_2a'] = lambda: gemm_mfma.gemm(A2, B2, bias=bias, act=activation, tile=7)
    if a.dtype == torch.bfloat16 and A2.dim() == 2 and bias is None and activation is None and \
            A2.shape[1] >= 8192:
        # long reductions over few output tiles (the MLM head's data gradient, K = vocab):
        # split K over fp32 slabs + one reduce
        # (BERT's masked-position head: 60 tiles at K = 30 528 -- 4 slices left 240 blocks
        # on 256 CUs; the single-stage tile holds 4 blocks per CU)
        tiles = -(-A2.shape[0] // 128) * -(-B2.shape[1] // 128)
        for s_ in (2, 4, 6, 8, 12, 16):
            if tiles * s_ <= 2048 and A2.shape[1] // s_ >= 512:
                cands['hip_sk%d' % s_] = (lambda s_=s_: gemm_mfma.gemm(A2, B2, splitk=s_))
                cands['hip_lo_sk%d' % s_] = (lambda s_=s_: gemm_mfma.gemm(A2, B2, splitk=s_, tile=3))
    if A2.dim() == 2 and B2.dim() == 2 and A2.shape[0] * B2.shape[1] <= gemm_mfma.SMALL_MAX_OUT:
        cands['hip_small'] = lambda: gemm_mfma.gemm_small(A2, B2, bias=bias, act=activation)
    # any shape: zero-padded aligned operands on the MFMA tile (last hand-written resort)
    cands['hip_pad'] = lambda: gemm_mfma.padded(A2, B2, bias=bias, act=activation)
    c = choose(key, cands)
    y = cands[c]()
    if y is None:
        y = gemm_mfma.padded(A2, B2, bias=bias, act=activation)
    if y is None:
        no_kernel('matmul', '%s x %s' % (tuple(A2.shape), tuple(B2.shape)))
    return y


_TILE_OF = {'hip256': 1, 'hip64': 2, 'hip_lo': 3, 'hip96': 5, 'hip_2a': 6, 'hip96_2a': 7}


def _run_decided(gemm_mfma, d, a, b, ta, tb, bias, activation):
    """the autotuned candidate ``d`` of ``matmul`` (None: not a plain tile choice / refused)"""
    if d == 'hip':
        return gemm_mfma.try_gemm(a, b, ta, tb, bias, activation)
    A2, B2 = _tr(a, ta), _tr(b, tb)
    t = _TILE_OF.get(d)
    if t is not None:
        return gemm_mfma.gemm(A2, B2, bias=bias, act=activation, tile=t)
    if d == 'hip_small':
        return gemm_mfma.gemm_small(A2, B2, bias=bias, act=activation)
    if d == 'hip_pad':
        return gemm_mfma.padded(A2, B2, bias=bias, act=activation)
    if d.startswith('hip_sk'):
        return gemm_mfma.gemm(A2, B2, splitk=int(d[6:]))
    if d.startswith('hip_lo_sk'):
        return gemm_mfma.gemm(A2, B2, splitk=int(d[9:]), tile=3)
    return None


def _big_ok(a, b, ta, tb):
    """the 256x256-tile kernel is a candidate once both output dims fill a tile"""
    A, B = _tr(a, ta), _tr(b, tb)
    return A.dim() == 2 and B.dim() == 2 and A.shape[0] >= 256 and B.shape[1] >= 256


def _as_dtype(t, dt):
    """t in dtype dt; an fp32 master parameter carries its bf16 compute copy (the
    optimizer's shadow, refreshed by the fused update) as ``hetu_bf16``."""
    if t.dtype == dt:
        return t
    sh = getattr(t, 'hetu_bf16', None)
    if sh is not None and sh.dtype == dt:
        return sh
    if t.is_cuda:   # the native cast, keeping a dense operand's stride order
        from .tensor import copy_into
        return copy_into(_NA.empty_like(t, dtype=dt), t)
    return t.to(dt)


def _cpu_matmul(a, b, ta, tb, bias, activation):
    """the CPU reference product (torch's CPU GEMM) with the elementwise epilogue"""
    A, B = _tr(a, ta), _tr(b, tb)
    if bias is not None and A.dim() == 2 and B.dim() == 2 and bias.dim() == 1:
        y = torch.addmm(_as_dtype(bias, A.dtype), A, B)
        bias = None
    else:
        y = torch.matmul(A, B)
    if bias is not None or activation is not None:
        from .elementwise import binary, unary
        if bias is not None:
            y = binary('add', y, bias.to(y.dtype).contiguous())
        if activation == 'relu':
            y = unary('relu', y)
        elif activation == 'gelu':
            y = unary('gelu', y)
    return y


def bmm(a, b, ta=False, tb=False):
    a, b = _match(a, b)
    if not a.is_cuda:
        return torch.matmul(_tr(a, ta), _tr(b, tb))
    if not (native(a) and a.dtype in (torch.bfloat16, torch.float32)):
        no_kernel('bmm', '%s %s' % (a.dtype, tuple(a.shape)))
    from . import gemm_mfma
    from .autotune import choose
    key = ('bmm', _sig(a), _sig(b), ta, tb)
    hip = lambda: gemm_mfma.try_bmm(a, b, ta, tb)

    def hip_pad():
        A, B = _tr(a, ta), _tr(b, tb)
        if A.dim() < 3 or A.shape[:-2] != B.shape[:-2]:
            return None
        lead = A.shape[:-2]
        y = gemm_mfma.padded(A.reshape(-1, *A.shape[-2:]), B.reshape(-1, *B.shape[-2:]))
        return None if y is None else y.view(*lead, *y.shape[-2:])
    c = choose(key, {'hip': hip, 'hip_pad': hip_pad})
    y = hip() if c == 'hip' else None
    if y is None:
        y = hip_pad()
    if y is None:
        no_kernel('bmm', '%s x %s' % (tuple(a.shape), tuple(b.shape)))
    return y


def _splitk_sum(part, out):
    """out = part.sum(0) for the [s, M, N] fp32 split-K partials: the vectorised
    ``hetu_splitk_sum_f32`` (all s loads in flight per lane) when ``out`` is a
    contiguous aligned fp32 buffer, else torch."""
    s = part.shape[0]
    n = out.numel()
    if part.is_contiguous() and out.is_contiguous() and out.dtype == torch.float32 and s <= 64 and n % 4 == 0 \
            and part.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0 and part[0].numel() == n:
        from . import fn, check, P, I32, I64, stream_ptr
        f = fn('hetu_splitk_sum_f32', [P, I32, P, I64, P])
        check(f(part.data_ptr(), s, out.data_ptr(), n, stream_ptr()), 'splitk_sum')
        return out
    torch.sum(part, 0, out=out)
    return out


def matmul_out(a, b, out):
    """out[M, N] = a[M, K] @ b[K, N] written into ``out`` -- a bf16 row block of a larger
    buffer (row stride >= N): the producers of a row concatenation write their slices in
    place (ops.linalg.RowConcatMatMulOp).  Autotuned over the MFMA tiles.  Returns ``out``."""
    a, b = _match(a, b)
    if not a.is_cuda:
        out.copy_(torch.matmul(a, b))
        return out
    if not (native(a) and a.dtype == torch.bfloat16 and out.dtype == torch.bfloat16):
        no_kernel('matmul_out', '%s %s -> %s' % (a.dtype, tuple(a.shape), out.dtype))
    from . import gemm_mfma
    from .autotune import choose
    key = ('gemm_out', _sig(a), _sig(b), _sig(out))
    cands = {'hip': lambda: gemm_mfma.gemm(a, b, out=out)}
    if _big_ok(a, b, False, False):
        cands['hip256'] = lambda: gemm_mfma.gemm(a, b, out=out, tile=1)
    if a.shape[-1] <= 2048:
        cands['hip_lo'] = lambda: gemm_mfma.gemm(a, b, out=out, tile=3)
    if a.shape[-1] >= 3 * 64:
        cands['hip_2a'] = lambda: gemm_mfma.gemm(a, b, out=out, tile=6)
    c = choose(key, cands)
    if cands[c]() is None and (c == 'hip' or gemm_mfma.gemm(a, b, out=out) is None):
        no_kernel('matmul_out', '%s x %s' % (tuple(a.shape), tuple(b.shape)))
    return out


def matmul_into(a, b, ta, tb, out):
    """out (fp32, e.g. a slot of the flat gradient buffer) = op(a) @ op(b): the MFMA
    kernels write fp32 directly (split-K candidates for long reductions).  Returns ``out``."""
    a, b = _match(a, b)
    if not a.is_cuda:
        out.copy_(torch.matmul(_tr(a, ta), _tr(b, tb)))
        return out
    if native(a) and a.dtype in (torch.bfloat16, torch.float32):
        from . import gemm_mfma
        from .autotune import choose, _decisions
        key = ('gemm_into', _sig(a), _sig(b), ta, tb)
        d = _decisions.get(key)
        if d is not None and _into_decided(gemm_mfma, d, _tr(a, ta), _tr(b, tb), out) is not None:
            return out

        def hip():
            return gemm_mfma.gemm(_tr(a, ta), _tr(b, tb), out=out)
        cands = {'hip': hip}
        # weight gradients: small M x N output, long K (= tokens): too few 128x128
        # tiles to fill 256 CUs -> split K over more workgroups (fp32 slab + reduce)
        A, B = _tr(a, ta), _tr(b, tb)
        if A.dim() == 2 and a.dtype == torch.float32:
            # fp32 (the reference's precision): the exact-fp32 MFMA kernel, or the one-wave
            # kernel for small outputs
            if A.shape[0] * B.shape[1] <= gemm_mfma.SMALL_MAX_OUT:
                cands['hip_small'] = lambda: gemm_mfma.gemm_small(A, B, out=out)
        elif A.dim() == 2:
            M, K, N = A.shape[0], A.shape[1], B.shape[1]
            tiles = -(-M // 128) * -(-N // 128)
            for s in (2, 3, 4, 6, 8, 12, 16):
                if tiles * s <= 1536 and K // s >= 512:
                    cands['hip_sk%d' % s] = (lambda s=s: gemm_mfma.gemm(A, B, out=out, splitk=s))
            # the single-stage tile at 4 blocks per CU: 892 vs 592 TF for the 2-stage tile on
            # 3072x3072x8192 TN (profiles/gemm_tn_r4.txt) -- and 1024 resident slots for splits
            if K >= 1024:
                cands['hip_lo'] = lambda: gemm_mfma.gemm(A, B, out=out, tile=3)
                for s in (2, 3, 4, 5, 6, 7, 8, 12, 16):
                    if tiles * s <= 2048 and K // s >= 512:
                        cands['hip_lo_sk%d' % s] = (lambda s=s: gemm_mfma.gemm(A, B, out=out, splitk=s, tile=3))
            if K >= 3 * 64:
                cands['hip_2a'] = lambda: gemm_mfma.gemm(A, B, out=out, tile=6)
                for s in (2, 3, 4, 6, 8, 12, 16):
                    if tiles * s <= 1536 and K // s >= 512:
                        cands['hip_2a_sk%d' % s] = (lambda s=s: gemm_mfma.gemm(A, B, out=out, splitk=s, tile=6))
            if M >= 256 and N >= 256:
                cands['hip256'] = lambda: gemm_mfma.gemm(A, B, out=out, tile=1)
                t256 = -(-M // 256) * -(-N // 256)
                # one 256x256 block per CU: split counts that fill the 256 CUs in one round
                # (36 tiles x 7 = 252 for BERT's FFN weight gradients) as well as the powers of 2
                for s in (2, 3, 4, 5, 6, 7, 8):
                    if t256 * s <= 512 and K // s >= 1024:
                        cands['hip256_sk%d' % s] = (lambda s=s: gemm_mfma.gemm(A, B, out=out, splitk=s, tile=1))
            if M * N <= gemm_mfma.SMALL_MAX_OUT:
                cands['hip_small'] = lambda: gemm_mfma.gemm_small(A, B, out=out)
            if N < 8 and M % 8 == 0 and K >= 4096 and out.dtype == torch.float32 and out.is_contiguous():
                # a few output columns over a long reduction (the MoE gate's weight gradient,
                # 2048 x 2 over 16384 tokens): B zero-padded to 8 columns on the MFMA tiles
                # with a deep K split (one wave per output read the 67 MB operand at 300 us)
                for s in (16, 32, 64):
                    if K // s >= 128:
                        cands['hip_pad8_sk%d' % s] = (lambda s=s: _pad8_into(A, B, out, s))
            if A.stride(0) == 1 and B.stride(1) == 1 and M % 64 == 0 and N % 64 == 0 and K >= 4096:
                # both operands token-major (weight gradients): the 64x64 split-K tile
                cands['hip_lk'] = lambda: gemm_mfma.wgrad_longk(A.t(), B, out)
        if A.dim() == 2:
            cands['hip_pad'] = lambda: gemm_mfma.padded(A, B, out=out)
        c = choose(key, cands)
        if cands[c]() is not None:
            return out
        if A.dim() == 2 and gemm_mfma.padded(A, B, out=out) is not None:
            return out
    no_kernel('matmul_into', '%s %s x %s' % (a.dtype, tuple(a.shape), tuple(b.shape)))


_INTO_TILE = {'hip': 0, 'hip_lo': 3, 'hip_2a': 6, 'hip256': 1}


def _into_decided(gemm_mfma, d, A, B, out):
    """the autotuned candidate ``d`` of ``matmul_into`` (None: refused / unknown name)"""
    if d == 'hip_small':
        return gemm_mfma.gemm_small(A, B, out=out)
    if d == 'hip_pad':
        return gemm_mfma.padded(A, B, out=out)
    if d == 'hip_lk':
        return gemm_mfma.wgrad_longk(A.t(), B, out)
    if d.startswith('hip_pad8_sk'):
        return _pad8_into(A, B, out, int(d[11:]))
    base, _, sk = d.partition('_sk') if '_sk' in d else (d, '', '')
    t = _INTO_TILE.get(base)
    if t is None:
        return None
    return gemm_mfma.gemm(A, B, out=out, splitk=int(sk) if sk else 1, tile=t)


def _pad8_into(A, B, out, splitk):
    """out[M, N<8] (fp32, contiguous) = A @ B with B padded to 8 columns (native zero fill
    and strided copies), split-K over ``splitk`` slices on the single-stage tile"""
    from . import gemm_mfma
    from .tensor import zeros, copy_into
    K, N = B.shape
    bp = zeros((K, 8), B.dtype, B.device)
    copy_into(bp[:, :N], B)
    op = _NA.empty((A.shape[0], 8), dtype=torch.float32, device=A.device)
    if gemm_mfma.gemm(A, bp, out=op, splitk=splitk, tile=3) is None:
        return None
    copy_into(out, op[:, :N])
    return out


def matmul_acc(a, b, ta, tb, acc, inplace=False):
    """op(a) @ op(b) + acc with the addition in the GEMM epilogue (beta = 1: the MFMA
    kernel reads ``acc`` as Cin).  ``inplace`` (acc dead after this call) is accepted for
    the graph rewrite's interface; the epilogue writes a new output either way."""
    a, b = _match(a, b)
    A, B = _tr(a, ta), _tr(b, tb)
    if not A.is_cuda:
        if A.dim() == 2 and acc.dim() == 2 and acc.dtype == A.dtype:
            return torch.addmm(acc, A, B)
        y = torch.matmul(A, B)
        return y + acc.to(y.dtype)
    if native(a) and a.dtype in (torch.bfloat16, torch.float32) and A.dim() == 2 and \
            tuple(acc.shape) == (A.shape[0], B.shape[1]):
        from . import gemm_mfma
        from .autotune import choose
        key = ('gemm_acc', _sig(a), _sig(b), ta, tb)
        cands = {'hip': lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0)}
        bf = a.dtype == torch.bfloat16       # fp32: the exact-fp32 kernel (``hip``) only
        if bf and A.shape[0] >= 256 and B.shape[1] >= 256:
            cands['hip256'] = lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0, tile=1)
        if bf and A.shape[1] <= 2048:
            cands['hip_lo'] = lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0, tile=3)
        if bf and B.shape[1] % 96 == 0 and A.shape[0] >= 1024:
            cands['hip96'] = lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0, tile=5)
        if bf and A.shape[1] >= 3 * 64:
            cands['hip_2a'] = lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0, tile=6)
            if B.shape[1] % 96 == 0 and A.shape[0] >= 1024:
                cands['hip96_2a'] = lambda: gemm_mfma.gemm(A, B, cin=acc, beta=1.0, tile=7)
        if A.shape[0] * B.shape[1] <= gemm_mfma.SMALL_MAX_OUT:
            cands['hip_small'] = lambda: gemm_mfma.gemm_small(A, B, cin=acc, beta=1.0)
        cands['hip_pad'] = lambda: gemm_mfma.padded(A, B, cin=acc, beta=1.0)
        ch = choose(key, cands)
        y = cands[ch]()
        if y is None:
            y = gemm_mfma.padded(A, B, cin=acc, beta=1.0)
        if y is not None:
            return y
    no_kernel('matmul_acc', '%s %s x %s + %s' % (a.dtype, tuple(A.shape), tuple(B.shape), tuple(acc.shape)))
