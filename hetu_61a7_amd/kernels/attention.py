"""Fused multi-head attention over a packed QKV projection (``attention.hip``).

``qkv`` is the [B*S, 3H] output of the QKV linear layer (head h of Q/K/V at
columns h*D, H + h*D, 2H + h*D); the context comes back as [B*S, H] and the
gradient as one packed [B*S, 3H] tensor -- no head transposes, slices or
concatenations around the kernel.  ``mask`` is an additive key mask [B, S].
Dropout on the probabilities uses Philox(seed, flat index of P / 4), so the
backward regenerates it.  GPU fast path: bf16, head dim 64, S % 32 == 0,
S <= 128 (S <= 256 forward-only); elsewhere a torch reference with the same
semantics (the CPU backend and the numerics oracle).
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, check, record_native, P, I64, I32, F32



# HETU_ATTN_BWD: the fixed-length backward's form.
#   split -- two launches, P_drop^T / dS^T through a 2 x S^2 bf16 global workspace per head
#            (small LDS, several workgroups per CU; BERT-base 4715/4715 vs 4691/4663
#            samples/s against fused in round 4);
#   fused -- one 4-wave launch with the images in ~122 KiB of LDS (one wave per SIMD);
#   w8    -- one 8-wave launch, same images plus a 32 KiB dQ exchange (two waves per SIMD).
# (HETU_ATTN_BWD_SPLIT=0 / 1 is the older spelling of fused / split.)
# Default w8: 53.9 us vs split 65.1 / fused 57.6 at BERT-base's shape with dropout 0.1
# (profiles/attention_kernels_r6.txt).
_BWD_MODE = os.environ.get('HETU_ATTN_BWD') or {'0': 'fused', '1': 'split'}.get(
    os.environ.get('HETU_ATTN_BWD_SPLIT', ''), 'w8')
_BWD_SPLIT = _BWD_MODE == 'split'


def _bwd_call(*args, device=None):
    """hetu_attn_bwd2 (fused, or split with a workspace) / hetu_attn_bwd8; args as
    hetu_attn_bwd's up to seed"""
    if _BWD_MODE == 'w8':
        f = fn('hetu_attn_bwd8', [P, P, P, I64, I64, I64, P, P, I64, P, P, I64, P, P, P, I64, I64, I64,
                                  I32, I32, I32, F32, F32, I64, P])
        check(f(*args, stream_ptr()), 'attn_bwd8')
        return
    B, NH, S = args[18], args[19], args[20]
    ws = _NA.empty(2 * B * NH * S * S, dtype=torch.bfloat16, device=device) if _BWD_SPLIT else None
    f = fn('hetu_attn_bwd2', [P, P, P, I64, I64, I64, P, P, I64, P, P, I64, P, P, P, I64, I64, I64,
                              I32, I32, I32, F32, F32, I64, P, P])
    check(f(*args, ws.data_ptr() if ws is not None else None, stream_ptr()), 'attn_bwd')


def fused_ok(qkv, S, D, need_bwd=True):
    return (native(qkv) and qkv.dtype == torch.bfloat16 and D == 64 and S % 32 == 0 and 0 < S <= (128 if need_bwd else 256)
            and qkv.is_contiguous())


def _key_mask(mask, B, S):
    """additive key mask [B, S] -> [B, 1, 1, S] (broadcast over heads and queries)"""
    return None if mask is None else mask.reshape(B, 1, 1, S)


def _heads(qkv, B, S, NH, D):
    H = NH * D
    x = qkv.reshape(B, S, 3, NH, D)
    return x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)


def _ref_probs(qkv, mask, B, S, NH, D, scale):
    q, k, v = _heads(qkv.float(), B, S, NH, D)
    s = q @ k.transpose(-1, -2) * scale
    if mask is not None:
        s = s + mask.float().reshape(B, 1, 1, S)
    return torch.softmax(s, -1), v


def _ref_dropmask(shape, keep, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) & 0x7FFFFFFF)
    return (torch.rand(shape, generator=g, device=device) < keep).float() / keep


_mask_memo = {}


def _mask_f32(mask):
    """fp32 contiguous copy of the attention mask, made once per mask tensor: every
    layer's forward and backward of a step receives the same (bf16 in mixed
    precision) mask (views of one tensor).  Keyed on that tensor, the view and the
    version counter; never
    memoised inside a hipGraph capture (a replay must re-read its fed buffer)."""
    if mask is None:
        return None
    if mask.dtype == torch.float32 and mask.is_contiguous():
        return mask
    from ..utils.hipgraph import capturing
    if mask.is_cuda and capturing():
        return _f32(mask)
    root = mask._base if mask._base is not None else mask     # ops hand in fresh views of it
    sig = (mask.data_ptr(), tuple(mask.shape), mask.stride(), mask._version)
    ent = _mask_memo.get(id(root))
    if ent is not None and ent[0]() is root and ent[1] == sig:
        return ent[2]
    m = _f32(mask)
    _mask_memo.clear()
    _mask_memo[id(root)] = (weakref.ref(root), sig, m)
    return m


def _f32(t):
    """contiguous fp32 copy of a device tensor on the native cast / copy kernels"""
    if not t.is_cuda:
        return t.float().contiguous()
    from .tensor import copy_into
    return copy_into(_NA.empty(t.shape, dtype=torch.float32, device=t.device), t)


# fp32 on the GPU (the reference's precision, parity runs): the reference's materialised
# chain -- scores, mask, softmax, dropout, P.V (examples/nlp/bert/hetu_bert.py:220-271) --
# on the hand-written exact-fp32 MFMA GEMM and the native softmax / dropout / broadcast
# kernels; the probabilities are saved for the backward.
def _f32_heads(qkv, B, S, NH, D):
    """contiguous fp32 [B*NH, S, D] copies of Q, K, V (native strided copies)"""
    from .tensor import copy_into
    if qkv.dtype != torch.float32:
        qkv = copy_into(_NA.empty(tuple(qkv.shape), dtype=torch.float32, device=qkv.device), qkv)
    out = []
    for t in packed_heads(qkv, B, S, NH):
        out.append(copy_into(_NA.empty((B, NH, S, D), dtype=torch.float32, device=qkv.device), t).view(B * NH, S, D))
    return out


def _f32_fwd(qkv, mask, B, S, NH, D, keep, seed, scale):
    from . import gemm as KG
    from .elementwise import unary, binary
    from .softmax import softmax
    from .dropout import dropout
    from .tensor import copy_into
    H = NH * D
    q, k, v = _f32_heads(qkv, B, S, NH, D)
    sc = unary('mul_c', KG.bmm(q, k, tb=True), scale).view(B, NH, S, S)
    if mask is not None:
        sc = binary('add', sc, _mask_f32(mask).reshape(B, 1, 1, S))
    p = softmax(sc)
    pd = dropout(p, keep, seed) if keep < 1.0 else p
    o = KG.bmm(pd.view(B * NH, S, S), v)
    out = _NA.empty((B * S, H), dtype=torch.float32, device=qkv.device)
    copy_into(out.view(B, S, NH, D).permute(0, 2, 1, 3), o.view(B, NH, S, D))
    if qkv.dtype != torch.float32:
        out = copy_into(_NA.empty((B * S, H), dtype=qkv.dtype, device=qkv.device), out)
    return out, p


def _f32_bwd(dout, qkv, p, B, S, NH, D, keep, seed, scale):
    from . import gemm as KG
    from .elementwise import unary, binary
    from .softmax import softmax_backward
    from .dropout import dropout
    from .tensor import copy_into, fill_
    H = NH * D
    q, k, v = _f32_heads(qkv, B, S, NH, D)
    if dout.dtype != torch.float32 or not dout.is_contiguous():
        dout = copy_into(_NA.empty(tuple(dout.shape), dtype=torch.float32, device=dout.device),
                         dout.contiguous() if dout.dtype == torch.float32 else dout)
    do = copy_into(_NA.empty((B, NH, S, D), dtype=torch.float32, device=qkv.device),
                   dout.reshape(B, S, NH, D).permute(0, 2, 1, 3)).view(B * NH, S, D)
    dm = None
    if keep < 1.0:       # the forward's mask, regenerated from the seed
        dm = dropout(fill_(_NA.empty(tuple(p.shape), dtype=torch.float32, device=p.device), 1.0), keep, seed)
    pd = binary('mul', p, dm) if dm is not None else p
    dv = KG.bmm(pd.view(B * NH, S, S), do, ta=True)
    dp = KG.bmm(do, v, tb=True).view(B, NH, S, S)
    if dm is not None:
        dp = binary('mul', dp, dm)
    ds = unary('mul_c', softmax_backward(p, dp), scale).view(B * NH, S, S)
    dq = KG.bmm(ds, k)
    dk = KG.bmm(ds, q, ta=True)
    dqkv = _NA.empty((B * S, 3 * H), dtype=torch.float32, device=qkv.device)
    gq, gk, gv = packed_heads(dqkv, B, S, NH)
    for dst, src in ((gq, dq), (gk, dk), (gv, dv)):
        copy_into(dst, src.view(B, NH, S, D))
    if qkv.dtype != torch.float32:
        dqkv = copy_into(_NA.empty((B * S, 3 * H), dtype=qkv.dtype, device=qkv.device), dqkv)
    return dqkv


def attention_fwd(qkv, mask, B, S, NH, keep=1.0, seed=0, scale=None):
    """-> (out [B*S, H], lse [B*NH*S] fp32 or probs (reference path))."""
    H = qkv.shape[1] // 3
    D = H // NH
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if fused_ok(qkv, S, D, need_bwd=False):
        out = _NA.empty((B * S, H), dtype=qkv.dtype, device=qkv.device)
        lse = _NA.empty((B * NH * S,), dtype=torch.float32, device=qkv.device)
        m = _mask_f32(mask)
        f = fn('hetu_attn_fwd', [P, P, P, I64, I64, I64, P, P, I64, P, I32, I32, I32, F32, F32, I64, P])
        base = qkv.data_ptr()
        es = qkv.element_size()
        check(f(base, base + H * es, base + 2 * H * es, 3 * H, 3 * H, 3 * H, m.data_ptr() if m is not None else None,
                out.data_ptr(), H, lse.data_ptr(), B, NH, S, float(scale), float(keep), int(seed), stream_ptr()),
              'attn_fwd')
        return out, lse
    q, k, v = packed_heads(qkv, B, S, NH)
    if flash_ok(q, k, v):
        # any other length / head dim: the general flash kernels, on the packed views
        out = _NA.empty((B * S, H), dtype=qkv.dtype, device=qkv.device)
        _, lse = flash_fwd(q, k, v, _key_mask(mask, B, S), False, keep, seed, scale,
                           out=out.view(B, S, NH, D).permute(0, 2, 1, 3))
        return out, lse
    if qkv.is_cuda:
        # fp32 (parity runs) or a head dim the flash kernels do not take: the materialised
        # chain on the native kernels, in fp32
        return _f32_fwd(qkv, mask, B, S, NH, D, keep, seed, scale)
    p, v = _ref_probs(qkv, mask, B, S, NH, D, scale)
    pd = p * _ref_dropmask(p.shape, keep, seed, p.device) if keep < 1.0 else p
    o = (pd @ v).transpose(1, 2).reshape(B * S, H)
    return o.to(qkv.dtype), p


def attention_bwd(dout, qkv, out, saved, mask, B, S, NH, keep=1.0, seed=0, scale=None):
    """-> dqkv [B*S, 3H] (same dtype as qkv)."""
    H = qkv.shape[1] // 3
    D = H // NH
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if fused_ok(qkv, S, D) and saved.dim() == 1:
        if dout.dtype != qkv.dtype or not dout.is_contiguous():
            from .tensor import copy_into
            dout = copy_into(_NA.empty(dout.shape, dtype=qkv.dtype, device=dout.device), dout)
        dqkv = _NA.empty_like(qkv)
        m = _mask_f32(mask)
        es = qkv.element_size()
        b, g = qkv.data_ptr(), dqkv.data_ptr()
        _bwd_call(b, b + H * es, b + 2 * H * es, 3 * H, 3 * H, 3 * H, m.data_ptr() if m is not None else None,
                  out.data_ptr(), H, saved.data_ptr(), dout.data_ptr(), H, g, g + H * es, g + 2 * H * es,
                  3 * H, 3 * H, 3 * H, B, NH, S, float(scale), float(keep), int(seed), device=qkv.device)
        return dqkv
    if saved.dim() == 1 and qkv.is_cuda:
        # the flash backward (its lse and dropout bits are the fused forward's: same
        # log-sum-exp of the scaled, masked scores; Philox(seed, row * S/4 + key/4))
        q, k, v = packed_heads(qkv, B, S, NH)
        if flash_ok(q, k, v):
            dqkv = _NA.empty_like(qkv)
            gq, gk, gv = packed_heads(dqkv, B, S, NH)
            o4 = out.view(B, S, NH, D).permute(0, 2, 1, 3)
            g4 = dout.reshape(B, S, NH, D).permute(0, 2, 1, 3)
            flash_bwd(g4, q, k, v, o4, saved, _key_mask(mask, B, S), False, keep, seed, scale, grads=(gq, gk, gv))
            return dqkv
        raise RuntimeError('attention backward: no hand-written kernel for S=%d D=%d' % (S, D))
    if qkv.is_cuda and saved.dim() == 4:
        return _f32_bwd(dout, qkv, saved, B, S, NH, D, keep, seed, scale)
    if saved.dim() == 1:    # fused forward (S <= 256) but no fused backward: recompute probs
        saved, _ = _ref_probs(qkv, mask, B, S, NH, D, scale)
    p = saved
    q, k, v = _heads(qkv.float(), B, S, NH, D)
    do = dout.float().reshape(B, S, NH, D).transpose(1, 2)
    dm = _ref_dropmask(p.shape, keep, seed, p.device) if keep < 1.0 else None
    pd = p * dm if dm is not None else p
    dv = pd.transpose(-1, -2) @ do
    dpd = do @ v.transpose(-1, -2)
    dp = dpd * dm if dm is not None else dpd
    ds = p * (dp - (dp * p).sum(-1, keepdim=True)) * scale
    dq = ds @ k
    dk = ds.transpose(-1, -2) @ q
    pack = torch.stack([dq, dk, dv], 2)               # [B, NH, 3, S, D]
    return pack.permute(0, 3, 2, 1, 4).reshape(B * S, 3 * H).to(qkv.dtype)


# ---------------------------------------------------------------------------
# Separate (strided) Q / K / V operands: the kernels take one pointer and row
# stride per operand, so a query block and a key/value block that live in
# different buffers (ring attention, ``parallel/ring_attention.py``) run
# through the same MFMA kernels without packing.  All operands are 2-D
# [B*S, H]-shaped row-major views (stride(1) == 1); lse is [B*NH*S] fp32.

def blocks_fused_ok(q, k, v, S, D):
    return (all(native(t) and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1
                for t in (q, k, v)) and D == 64 and S % 32 == 0 and 0 < S <= 128)


def attention_fwd_blocks(q, k, v, mask, B, S, NH, scale):
    """-> (out [B*S, H] bf16, lse [B*NH*S] fp32) of softmax(q k^T * scale + mask) v."""
    H = q.shape[1]
    out = _NA.empty((B * S, H), dtype=q.dtype, device=q.device)
    lse = _NA.empty((B * NH * S,), dtype=torch.float32, device=q.device)
    m = _mask_f32(mask)
    f = fn('hetu_attn_fwd', [P, P, P, I64, I64, I64, P, P, I64, P, I32, I32, I32, F32, F32, I64, P])
    check(f(q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0), v.stride(0),
            m.data_ptr() if m is not None else None, out.data_ptr(), H, lse.data_ptr(), B, NH, S,
            float(scale), 1.0, 0, stream_ptr()), 'attn_fwd')
    return out, lse


def attention_bwd_blocks(dout, q, k, v, out, lse, mask, B, S, NH, scale):
    """Gradient of one (query block, key block) pair given the GLOBAL softmax
    statistics: ``out`` and ``lse`` are the final merged output and row
    log-sum-exp of the query block, so P = exp(s - lse) and
    D = rowsum(dout * out) are the exact global terms and the returned
    (dq, dk, dv) [B*S, H] are this key block's exact contributions."""
    H = q.shape[1]
    dout = dout.to(q.dtype).contiguous()
    out = out.to(q.dtype).contiguous()
    dq = _NA.empty((B * S, H), dtype=q.dtype, device=q.device)
    dk = _NA.empty_like(dq)
    dv = _NA.empty_like(dq)
    m = _mask_f32(mask)
    _bwd_call(q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0), v.stride(0),
              m.data_ptr() if m is not None else None, out.data_ptr(), H, lse.contiguous().data_ptr(),
              dout.data_ptr(), H, dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), H, H, H, B, NH, S,
              float(scale), 1.0, 0, device=q.device)
    return dq, dk, dv


# ---------------------------------------------------------------------------
# BERT-length fast path for [B, NH, S, D] views (attention_op): when Q / K / V are head
# views of token-major rows ([B, S, NH*64]-like storage: strides (S*ld, 64, ld, 1)), S is a
# multiple of 32 up to 128 and the mask is a key mask, the one-workgroup-per-head kernels of
# ``attention.hip`` take them as they are -- at S = 128 they run 1.3-1.5x faster than the
# general flash tiles.  Same softmax statistics and Philox dropout layout as flash.

def _rows_ld(t, S):
    """row stride of a [B, NH, S, 64] head view of token-major rows, or None"""
    B, NH, S_, D = t.shape
    if D != 64 or S_ != S or t.stride(3) != 1 or t.stride(1) != 64:
        return None
    ld = t.stride(2)
    if t.stride(0) != S * ld or ld % 8 or t.data_ptr() % 16:
        return None
    return ld


def seqblock_ok(q, k, v, mask, causal):
    if causal or not all(native(t) and t.dtype == torch.bfloat16 and t.dim() == 4 for t in (q, k, v)):
        return False
    B, NH, S, D = q.shape
    if D != 64 or S % 32 or not 0 < S <= 128 or tuple(k.shape) != tuple(q.shape) or tuple(v.shape) != tuple(q.shape):
        return False
    if any(_rows_ld(t, S) is None for t in (q, k, v)):
        return False
    if mask is not None:
        # a key mask only: [B, 1, 1, S] / [B, S] (broadcast over heads and queries)
        if mask.numel() != B * S or (mask.dim() == 4 and (mask.shape[1] != 1 or mask.shape[2] != 1)):
            return False
    return True


def seqblock_fwd(q, k, v, mask, keep, seed, scale):
    """-> (o [B, NH, S, 64] view of token-major rows, lse [B*NH*S] fp32)"""
    B, NH, S, D = q.shape
    H = NH * D
    o = _NA.empty((B, S, H), dtype=q.dtype, device=q.device)
    lse = _NA.empty((B * NH * S,), dtype=torch.float32, device=q.device)
    m = _mask_f32(mask.reshape(B, S)) if mask is not None else None
    f = fn('hetu_attn_fwd', [P, P, P, I64, I64, I64, P, P, I64, P, I32, I32, I32, F32, F32, I64, P])
    check(f(q.data_ptr(), k.data_ptr(), v.data_ptr(), _rows_ld(q, S), _rows_ld(k, S), _rows_ld(v, S),
            m.data_ptr() if m is not None else None, o.data_ptr(), H, lse.data_ptr(), B, NH, S,
            float(scale), float(keep), int(seed), stream_ptr()), 'attn_fwd')
    return o.view(B, S, NH, D).permute(0, 2, 1, 3), lse


def seqblock_bwd(do, q, k, v, o, lse, mask, keep, seed, scale):
    """(dq, dk, dv) as [B, NH, S, 64] views of token-major rows"""
    B, NH, S, D = q.shape
    H = NH * D
    if do.dtype != q.dtype or _rows_ld(do, S) is None:
        from .tensor import copy_into
        do = copy_into(_NA.empty((B, S, NH, D), dtype=q.dtype, device=q.device).permute(0, 2, 1, 3), do)
    grads = [_NA.empty((B, S, H), dtype=q.dtype, device=q.device) for _ in range(3)]
    m = _mask_f32(mask.reshape(B, S)) if mask is not None else None
    _bwd_call(q.data_ptr(), k.data_ptr(), v.data_ptr(), _rows_ld(q, S), _rows_ld(k, S), _rows_ld(v, S),
              m.data_ptr() if m is not None else None, o.data_ptr(), _rows_ld(o, S), lse.data_ptr(),
              do.data_ptr(), _rows_ld(do, S), grads[0].data_ptr(), grads[1].data_ptr(), grads[2].data_ptr(),
              H, H, H, B, NH, S, float(scale), float(keep), int(seed), device=q.device)
    return tuple(g.view(B, S, NH, D).permute(0, 2, 1, 3) for g in grads)


# ---------------------------------------------------------------------------
# General fused attention (``flash_attn.hip``): any Sq / Sk, head dim 32 / 64 / 128,
# causal, an additive mask broadcastable to [B, NH, Sq, Sk], dropout; Q / K / V / O
# as strided [B, NH, S, D] views (head dim contiguous), so packed projections and
# transposed head views are read and written in place.

FLASH_D = (32, 64, 128)


def _st3(t):
    """(batch, head, row) strides of a [B, NH, S, D] view"""
    return (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2))


def flash_ok(q, k, v):
    D = q.shape[-1]
    return (all(native(t) and t.dtype == torch.bfloat16 and t.dim() == 4 and t.stride(-1) == 1
                and t.data_ptr() % 16 == 0 and all(s % 8 == 0 for s in t.stride()[:3]) for t in (q, k, v))
            and D in FLASH_D and k.shape[-1] == D and v.shape[-1] == D and k.shape[2] == v.shape[2])


def _flash_mask(mask, B, NH, Sq, Sk):
    """(fp32 mask, its [b, h, q, k] strides) -- 0 strides on broadcast dims"""
    if mask is None:
        return None, None
    m = mask
    if m.dtype != torch.float32 or not m.is_contiguous():
        m = _mask_f32(m) if m.dim() == 2 else _f32(m)
    me = m.expand(B, NH, Sq, Sk) if m.dim() <= 4 else None
    if me is None:
        raise ValueError('attention mask of shape %s does not broadcast to [B, NH, Sq, Sk]' % (tuple(mask.shape),))
    return m, (ctypes.c_int64 * 4)(*me.stride())


def flash_fwd(q, k, v, mask=None, causal=False, keep=1.0, seed=0, scale=None, out=None):
    """-> (o [B, NH, Sq, D] (a view of a [B, Sq, NH, D] buffer, or ``out``), lse [B*NH*Sq] fp32)"""
    B, NH, Sq, D = q.shape
    Sk = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if out is None:
        out = _NA.empty((B, Sq, NH, D), dtype=q.dtype, device=q.device).permute(0, 2, 1, 3)
    lse = _NA.empty((B * NH * Sq,), dtype=torch.float32, device=q.device)
    m, mst = _flash_mask(mask, B, NH, Sq, Sk)
    f = fn('hetu_flash_fwd', [P, P, P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, F32, I64, P])
    check(f(q.data_ptr(), k.data_ptr(), v.data_ptr(), _st3(q), _st3(k), _st3(v), out.data_ptr(), _st3(out),
            lse.data_ptr(), m.data_ptr() if m is not None else None, mst, B, NH, Sq, Sk, D, int(bool(causal)),
            float(scale), float(keep), int(seed), stream_ptr()), 'flash_fwd')
    record_native('flash_fwd')
    return out, lse


def flash_bwd(dout, q, k, v, o, lse, mask=None, causal=False, keep=1.0, seed=0, scale=None, grads=None):
    """-> (dq, dk, dv) shaped like q, k, v ([B, S, NH, D] buffers seen as [B, NH, S, D]),
    or written into ``grads`` (three such views)"""
    B, NH, Sq, D = q.shape
    Sk = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if dout.dtype != q.dtype or dout.stride(-1) != 1 or dout.data_ptr() % 16 or any(s % 8 for s in dout.stride()[:3]):
        from .tensor import copy_into
        dout = copy_into(_NA.empty((B, Sq, NH, D), dtype=q.dtype, device=q.device).permute(0, 2, 1, 3), dout)
    if grads is None:
        mk = lambda S: _NA.empty((B, S, NH, D), dtype=q.dtype, device=q.device).permute(0, 2, 1, 3)
        grads = (mk(Sq), mk(Sk), mk(Sk))
    dq, dk, dv = grads
    dsum = _NA.empty((B * NH * Sq,), dtype=torch.float32, device=q.device)
    m, mst = _flash_mask(mask, B, NH, Sq, Sk)
    f = fn('hetu_flash_bwd', [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P,
                              I32, I32, I32, I32, I32, I32, F32, F32, I64, P])
    check(f(q.data_ptr(), k.data_ptr(), v.data_ptr(), _st3(q), _st3(k), _st3(v), o.data_ptr(), _st3(o),
            lse.data_ptr(), dout.data_ptr(), _st3(dout), dq.data_ptr(), _st3(dq), dk.data_ptr(), _st3(dk),
            dv.data_ptr(), _st3(dv), m.data_ptr() if m is not None else None, mst, dsum.data_ptr(),
            B, NH, Sq, Sk, D, int(bool(causal)), float(scale), float(keep), int(seed), stream_ptr()), 'flash_bwd')
    record_native('flash_bwd')
    return dq, dk, dv


def lse_merge(o, lse, ob, lb):
    """ring attention merge: (o fp32 [B, S, NH, D], lse fp32 [B, NH, S]) <- log-sum-exp
    combination with one block's (ob bf16 [B, S, NH, D] dense, lb [B*NH*S]); in place"""
    B, S, NH, D = o.shape
    assert o.is_contiguous() and lse.is_contiguous() and ob.is_contiguous() and ob.dtype == torch.bfloat16
    f = fn('hetu_flash_lse_merge', [P, P, P, P, I32, I32, I32, I32, P])
    check(f(o.data_ptr(), lse.data_ptr(), ob.data_ptr(), lb.data_ptr(), B, S, NH, D, stream_ptr()), 'lse_merge')
    record_native('lse_merge')


def acc_rows(acc, x):
    """acc (fp32 [R, C], unit column stride) += x (bf16 [R, C], unit column stride); in place"""
    R, C = x.shape
    assert acc.shape == x.shape and acc.stride(1) == 1 and x.stride(1) == 1 and x.dtype == torch.bfloat16
    f = fn('hetu_acc_rows_bf16', [P, I64, P, I64, I64, I32, P])
    check(f(acc.data_ptr(), acc.stride(0), x.data_ptr(), x.stride(0), R, C, stream_ptr()), 'acc_rows')
    record_native('acc_rows')


def packed_heads(qkv, B, S, NH):
    """[B*S, 3H] packed projection -> q, k, v as [B, NH, S, D] views (no copies)"""
    H = qkv.shape[1] // 3
    D = H // NH
    x = qkv.view(B, S, 3, NH, D)
    return x[:, :, 0].permute(0, 2, 1, 3), x[:, :, 1].permute(0, 2, 1, 3), x[:, :, 2].permute(0, 2, 1, 3)
