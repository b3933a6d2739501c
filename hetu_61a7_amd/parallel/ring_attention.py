"""Ring attention / context parallelism (SURVEY §5.7 item 3, §2.3 S13 -- absent
in the reference, whose attention materialises the full [B, H, S, S] scores:
``examples/nlp/bert/hetu_bert.py:220-271``).

Each of the P ranks of the context-parallel group holds ``S/P`` consecutive
tokens: its packed QKV projection ``qkv`` [B*S/P, 3H] and its additive key
mask slice [B, S/P].  Queries never move.  The K/V block (and its mask slice)
travels once around the ring: at step s rank r attends to the block owned by
rank (r - s) mod P while the next block is already in flight from rank r-1
(one grouped RCCL send/recv per step, so on xGMI every rank drives one
point-to-point link per step and the transfer hides behind the block's
matmuls).  Partial results are merged with the online-softmax rule, so no
rank ever holds more than an [S/P, S/P] score tile per head, and the saved
state for backward is just O and the row log-sum-exp.  Each non-causal block
pair runs through the general flash kernels (``kernels/attention.py``
``flash_{fwd,bwd}``: bf16, any S/P, head dim 32 / 64 / 128, the causal diagonal
block included) with Q and the travelling K/V block read in place as strided
head views; the block's (out, lse) is merged into the fp32 running output by a
log-sum-exp merge kernel.  The backward kernels are handed the GLOBAL out and
lse, which makes their dQ/dK/dV the exact per-block terms; fp32 accumulators
take them through a row-accumulate kernel.  CPU tensors (the gloo tests) take
the torch block math below.

Backward re-runs the ring: the K/V block travels together with an fp32 dK/dV
accumulator; every rank adds its queries' contribution to the block it holds,
and after P hops the accumulator arrives back at the block's owner complete.

Compared with Ulysses (``sequence.py``, two all-to-alls, heads must divide
over P) ring attention has no head-count constraint and its per-step traffic
is one K/V block to one neighbour; it is the choice for P > NH or very long S.
``causal=True`` skips blocks strictly above the diagonal and masks the
diagonal block.
"""
from __future__ import annotations

import math

import torch

from .. import native_array as _NA
from ..ops.node import Op
from ..ops.nn import AuxResult


def _heads(x, B, S_l, NH, D):
    """[B*S_l, NH*D] row view -> [B, NH, S_l, D]"""
    return x.reshape(B, S_l, NH, D).transpose(1, 2)


def _rows(x):
    """[B, NH, S_l, D] -> [B*S_l, NH*D]"""
    B, NH, S_l, D = x.shape
    return x.transpose(1, 2).reshape(B * S_l, NH * D)


def _rotate(comm, tensors):
    """Send each tensor to rank+1, receive the same-shaped tensors from rank-1."""
    P, r = comm.nrank, comm.rank
    outs = [_NA.empty_like(t) for t in tensors]
    ops = []
    for t, o in zip(tensors, outs):
        ops += [('send', t.contiguous(), (r + 1) % P), ('recv', o, (r - 1) % P)]
    return outs, comm.batch_p2p(ops)


def _scores(q, k, kmask, scale, causal_diag):
    s = torch.matmul(q, k.transpose(-1, -2)).float() * scale        # [B, NH, S_l, S_l]
    if kmask is not None:
        s = s + kmask.reshape(kmask.shape[0], 1, 1, -1).float()
    if causal_diag:
        n = s.shape[-1]
        tri = torch.ones(n, n, dtype=torch.bool, device=s.device).triu_(1)
        s = s.masked_fill(tri, float('-inf'))
    return s


def _use_fused(q, k, v, S_l, D, diag):
    if diag:                     # the MFMA kernel has no causal mask: diagonal block on the torch path
        return False
    from ..kernels import attention as KA
    return KA.blocks_fused_ok(q, k, v, S_l, D)


def _block_fwd(q, k, v, kmask, B, S_l, NH, D, scale, diag):
    """One (query block, key block) pair -> (out [B, S_l, NH, D], lse [B, NH, S_l] fp32)."""
    if _use_fused(q, k, v, S_l, D, diag):
        from ..kernels import attention as KA
        o, lse = KA.attention_fwd_blocks(q, k, v, kmask, B, S_l, NH, scale)
        return o.reshape(B, S_l, NH, D), lse.reshape(B, NH, S_l)
    sc = _scores(_heads(q, B, S_l, NH, D), _heads(k, B, S_l, NH, D), kmask, scale, diag)
    m = sc.amax(-1, keepdim=True)
    p = torch.exp(sc - m)
    l = p.sum(-1, keepdim=True)
    vh = _heads(v, B, S_l, NH, D)
    o = torch.matmul(p.to(vh.dtype), vh).float() / l
    return o.transpose(1, 2), (m + torch.log(l)).squeeze(-1)


def _block_bwd(dout, q, k, v, out, lse, kmask, B, S_l, NH, D, scale, diag):
    """Exact contribution of one key block given the global (out, lse) -> (dq, dk, dv) [B*S_l, H]."""
    if _use_fused(q, k, v, S_l, D, diag):
        from ..kernels import attention as KA
        return KA.attention_bwd_blocks(dout, q, k, v, out, lse, kmask, B, S_l, NH, scale)
    qh, kh, vh = _heads(q, B, S_l, NH, D), _heads(k, B, S_l, NH, D), _heads(v, B, S_l, NH, D)
    doh = _heads(dout, B, S_l, NH, D).to(q.dtype)
    delta = (doh.float() * _heads(out, B, S_l, NH, D).float()).sum(-1, keepdim=True)
    p = torch.exp(_scores(qh, kh, kmask, scale, diag) - lse.reshape(B, NH, S_l, 1))
    dv = torch.matmul(p.transpose(-1, -2).to(doh.dtype), doh)
    dp = torch.matmul(doh, vh.transpose(-1, -2)).float()
    ds = (p * (dp - delta) * scale).to(q.dtype)
    return _rows(torch.matmul(ds, kh)), _rows(torch.matmul(ds.transpose(-1, -2), qh)), _rows(dv)


def _flash_ring_ok(qkv, NH):
    from ..kernels import attention as KA
    from ..kernels import native
    H = qkv.shape[1] // 3
    return (native(qkv) and qkv.dtype == torch.bfloat16 and H % NH == 0 and (H // NH) in KA.FLASH_D
            and qkv.stride(1) == 1 and qkv.stride(0) % 8 == 0 and qkv.data_ptr() % 16 == 0)


def _cpu_only(qkv, NH):
    """the per-block torch math below is the CPU reference (gloo rehearsals); on the GPU
    every ring block runs on the flash kernels (bf16, head dim 32 / 64 / 128)"""
    if qkv.is_cuda:
        from ..kernels import no_kernel
        no_kernel('ring_attention', '%s, head dim %d' % (qkv.dtype, qkv.shape[1] // 3 // NH))


def _kv_heads(kv, B, S_l, NH, D):
    """[B*S_l, 2H] travelling block -> k, v as [B, NH, S_l, D] views"""
    x = kv.view(B, S_l, 2, NH, D)
    return x[:, :, 0].permute(0, 2, 1, 3), x[:, :, 1].permute(0, 2, 1, 3)


def _send_copy(x):
    from ..kernels import tensor as KT
    return KT.copy_into(_NA.empty(tuple(x.shape), dtype=x.dtype, device=x.device), x)


def _ring_fwd_flash(qkv, kmask, comm, B, S_l, NH, causal, scale):
    from ..kernels import attention as KA
    from ..kernels import tensor as KT
    from ..kernels import elementwise as KE
    P, r = comm.nrank, comm.rank
    H = qkv.shape[1] // 3
    D = H // NH
    q4, _, _ = KA.packed_heads(qkv, B, S_l, NH)
    o = KT.zeros((B, S_l, NH, D), dtype=torch.float32, device=qkv.device)
    lse = KT.fill_(_NA.empty((B, NH, S_l), dtype=torch.float32, device=qkv.device), float('-inf'))
    kv = qkv[:, H:]
    km = kmask.contiguous() if kmask is not None else None
    for s in range(P):
        j = (r - s) % P
        reqs, nxt = [], None
        if s < P - 1:
            send = [kv if kv.is_contiguous() else _send_copy(kv)] + ([km] if km is not None else [])
            nxt, reqs = _rotate(comm, send)
        if not (causal and j > r):
            k4, v4 = _kv_heads(kv, B, S_l, NH, D)
            m4 = km.reshape(B, 1, 1, S_l) if km is not None else None
            ob, lb = KA.flash_fwd(q4, k4, v4, m4, causal and j == r, 1.0, 0, scale)
            KA.lse_merge(o, lse, ob.permute(0, 2, 1, 3), lb)
        for w in reqs:
            w.wait()
        if nxt is not None:
            kv = nxt[0]
            km = nxt[1] if km is not None else None
    return KE.cast(o.reshape(B * S_l, H), qkv.dtype), lse


def _ring_bwd_flash(dout, qkv, kmask, out, lse, comm, B, S_l, NH, causal, scale):
    from ..kernels import attention as KA
    from ..kernels import tensor as KT
    P, r = comm.nrank, comm.rank
    H = qkv.shape[1] // 3
    D = H // NH
    q4, _, _ = KA.packed_heads(qkv, B, S_l, NH)
    if dout.dtype != qkv.dtype or not dout.is_contiguous():
        dout = KT.copy_into(_NA.empty(tuple(dout.shape), dtype=qkv.dtype, device=dout.device), dout)
    if not out.is_contiguous():
        out = _send_copy(out)
    g4 = dout.view(B, S_l, NH, D).permute(0, 2, 1, 3)
    o4 = out.view(B, S_l, NH, D).permute(0, 2, 1, 3)
    lsef = lse.reshape(-1)
    dq = KT.zeros((B * S_l, H), dtype=torch.float32, device=qkv.device)
    dkv = KT.zeros((B * S_l, 2 * H), dtype=torch.float32, device=qkv.device)
    kv = qkv[:, H:]
    km = kmask.contiguous() if kmask is not None else None
    rows = lambda t: t.permute(0, 2, 1, 3).reshape(B * S_l, H)
    for s in range(P):
        j = (r - s) % P
        if not (causal and j > r):
            k4, v4 = _kv_heads(kv, B, S_l, NH, D)
            m4 = km.reshape(B, 1, 1, S_l) if km is not None else None
            gq, gk, gv = KA.flash_bwd(g4, q4, k4, v4, o4, lsef, m4, causal and j == r, 1.0, 0, scale)
            KA.acc_rows(dq, rows(gq))
            KA.acc_rows(dkv[:, :H], rows(gk))
            KA.acc_rows(dkv[:, H:], rows(gv))
        if P == 1:
            break
        if s < P - 1:
            send = [dkv, kv if kv.is_contiguous() else _send_copy(kv)] + ([km] if km is not None else [])
        else:
            send = [dkv]
        nxt, reqs = _rotate(comm, send)
        for w in reqs:
            w.wait()
        dkv = nxt[0]
        if s < P - 1:
            kv = nxt[1]
            km = nxt[2] if km is not None else None
    res = _NA.empty((B * S_l, 3 * H), dtype=qkv.dtype, device=qkv.device)
    KT.copy_into(res[:, :H], dq)
    KT.copy_into(res[:, H:], dkv)
    return res


def ring_attention_fwd(qkv, kmask, comm, B, S_l, NH, causal=False, scale=None):
    """qkv [B*S_l, 3H] (this rank's tokens), kmask [B, S_l] or None.
    Returns (out [B*S_l, H] in qkv's dtype, lse [B, NH, S_l] fp32)."""
    if _flash_ring_ok(qkv, NH):
        return _ring_fwd_flash(qkv, kmask, comm, B, S_l, NH, causal,
                               scale or 1.0 / math.sqrt(qkv.shape[1] // 3 // NH))
    _cpu_only(qkv, NH)
    P, r = comm.nrank, comm.rank
    H = qkv.shape[1] // 3
    D = H // NH
    scale = scale or 1.0 / math.sqrt(D)
    q = qkv[:, :H]
    o = torch.zeros((B, S_l, NH, D), dtype=torch.float32, device=qkv.device)
    lse = torch.full((B, NH, S_l), float('-inf'), dtype=torch.float32, device=qkv.device)
    cur = [qkv[:, H:].contiguous()] + ([kmask.contiguous()] if kmask is not None else [])
    for s in range(P):
        j = (r - s) % P
        nxt, reqs = _rotate(comm, cur) if s < P - 1 else (None, [])
        if not (causal and j > r):
            kv = cur[0]
            ob, lb = _block_fwd(q, kv[:, :H], kv[:, H:], cur[1] if kmask is not None else None,
                                B, S_l, NH, D, scale, causal and j == r)
            new = torch.logaddexp(lse, lb)
            wa = torch.exp(lse - new).transpose(1, 2).unsqueeze(-1)     # [B, S_l, NH, 1]
            wb = torch.exp(lb - new).transpose(1, 2).unsqueeze(-1)
            o = o * wa + ob.float() * wb
            lse = new
        for w in reqs:
            w.wait()
        if nxt is not None:
            cur = nxt
    return o.reshape(B * S_l, H).to(qkv.dtype), lse


def ring_attention_bwd(dout, qkv, kmask, out, lse, comm, B, S_l, NH, causal=False, scale=None):
    """Returns dqkv [B*S_l, 3H] in qkv's dtype."""
    if _flash_ring_ok(qkv, NH):
        return _ring_bwd_flash(dout, qkv, kmask, out, lse, comm, B, S_l, NH, causal,
                               scale or 1.0 / math.sqrt(qkv.shape[1] // 3 // NH))
    _cpu_only(qkv, NH)
    P, r = comm.nrank, comm.rank
    H = qkv.shape[1] // 3
    D = H // NH
    scale = scale or 1.0 / math.sqrt(D)
    q = qkv[:, :H]
    dout = dout.to(qkv.dtype).contiguous()
    dq = torch.zeros((B * S_l, H), dtype=torch.float32, device=qkv.device)
    dkv = torch.zeros((B * S_l, 2 * H), dtype=torch.float32, device=qkv.device)
    cur = [qkv[:, H:].contiguous()] + ([kmask.contiguous()] if kmask is not None else [])
    for s in range(P):
        j = (r - s) % P
        if not (causal and j > r):
            kv = cur[0]
            gq, gk, gv = _block_bwd(dout, q, kv[:, :H], kv[:, H:], out, lse, cur[1] if kmask is not None else None,
                                    B, S_l, NH, D, scale, causal and j == r)
            dq += gq.float()
            dkv[:, :H] += gk.float()
            dkv[:, H:] += gv.float()
        if P == 1:
            break
        # the K/V block moves on with its gradient; the last hop only returns dK/dV to the owner
        (nxt, reqs) = _rotate(comm, ([dkv] + cur) if s < P - 1 else [dkv])
        for w in reqs:
            w.wait()
        dkv = nxt[0]
        if s < P - 1:
            cur = nxt[1:]
    return torch.cat([dq, dkv], 1).to(qkv.dtype)


class RingAttentionOp(Op):
    """out [B*S/P, H] = MHA over the whole sequence, context-parallel over ``comm``."""

    def __init__(self, qkv, mask, batch, local_seq_len, num_heads, comm=None, causal=False, scale=None, ctx=None):
        super().__init__(RingAttentionOp, [qkv] + ([mask] if mask is not None else []), ctx)
        self.has_mask = mask is not None
        self.B, self.S_l, self.NH = int(batch), int(local_seq_len), int(num_heads)
        self.comm = comm
        self.causal = bool(causal)
        self.scale = scale

    def _comm(self):
        from . import comm as C
        if self.comm is None:
            self.comm = C.init_process_group()
        return self.comm

    def compute(self, input_vals, output_val=None, stream_handle=None):
        comm = self._comm()
        qkv = input_vals[0]
        H = qkv.shape[1] // 3
        D = H // self.NH
        assert qkv.shape[0] == self.B * self.S_l, (qkv.shape, self.B, self.S_l)
        kmask = input_vals[1].reshape(self.B, self.S_l) if self.has_mask else None
        out, lse = ring_attention_fwd(qkv, kmask, comm, self.B, self.S_l, self.NH, self.causal, self.scale)
        return AuxResult(out, (qkv, kmask, lse))

    def gradient(self, output_grad):
        return [RingAttentionGradientOp(output_grad, self, ctx=self.raw_ctx)] + ([None] if self.has_mask else [])

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], input_shapes[0][1] // 3)


class RingAttentionGradientOp(Op):
    value_and_aux_inputs = (1,)

    def __init__(self, dout, fwd, ctx=None):
        super().__init__(RingAttentionGradientOp, [dout, fwd], ctx)
        self.fwd = fwd

    def compute(self, input_vals, output_val=None, stream_handle=None):
        f = self.fwd
        dout, (out, (qkv, kmask, lse)) = input_vals
        return ring_attention_bwd(dout, qkv, kmask, out, lse, f.comm, f.B, f.S_l, f.NH, f.causal, f.scale)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def ring_attention_op(qkv, mask, batch, local_seq_len, num_heads, comm=None, causal=False, scale=None, ctx=None):
    return RingAttentionOp(qkv, mask, batch, local_seq_len, num_heads, comm, causal, scale, ctx=ctx)
