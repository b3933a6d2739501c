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
state for backward is just O and the row log-sum-exp.

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

from ..ops.node import Op
from ..ops.nn import AuxResult


def _split(qkv, B, S_l, NH, D):
    x = qkv.reshape(B, S_l, 3, NH, D).permute(2, 0, 3, 1, 4)     # [3, B, NH, S_l, D]
    return x[0], x[1:].contiguous()


def _rotate(comm, tensors):
    """Send each tensor to rank+1, receive the same-shaped tensors from rank-1."""
    P, r = comm.nrank, comm.rank
    outs = [torch.empty_like(t) for t in tensors]
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


def ring_attention_fwd(q, kv, kmask, comm, causal=False, scale=None):
    """q [B, NH, S_l, D]; kv [2, B, NH, S_l, D]; kmask [B, S_l] or None.
    Returns (out [B, NH, S_l, D] in q's dtype, lse [B, NH, S_l, 1] fp32)."""
    P, r = comm.nrank, comm.rank
    scale = scale or 1.0 / math.sqrt(q.shape[-1])
    B, NH, S_l, D = q.shape
    o = torch.zeros((B, NH, S_l, D), dtype=torch.float32, device=q.device)
    m = torch.full((B, NH, S_l, 1), float('-inf'), dtype=torch.float32, device=q.device)
    l = torch.zeros_like(m)
    cur = [kv] + ([kmask.contiguous()] if kmask is not None else [])
    for s in range(P):
        j = (r - s) % P
        nxt, reqs = _rotate(comm, cur) if s < P - 1 else (None, [])
        if not (causal and j > r):
            k, v = cur[0][0], cur[0][1]
            sc = _scores(q, k, cur[1] if kmask is not None else None, scale, causal and j == r)
            m_new = torch.maximum(m, sc.amax(-1, keepdim=True))
            p = torch.exp(sc - m_new)
            alpha = torch.exp(m - m_new)
            l = l * alpha + p.sum(-1, keepdim=True)
            o = o * alpha + torch.matmul(p.to(v.dtype), v).float()
            m = m_new
        for w in reqs:
            w.wait()
        if nxt is not None:
            cur = nxt
    out = (o / l).to(q.dtype)
    return out, m + torch.log(l)


def ring_attention_bwd(dout, q, kv, kmask, out, lse, comm, causal=False, scale=None):
    """Returns (dq [B, NH, S_l, D], dkv [2, B, NH, S_l, D]) in fp32."""
    P, r = comm.nrank, comm.rank
    scale = scale or 1.0 / math.sqrt(q.shape[-1])
    dout = dout.to(q.dtype)
    delta = (dout.float() * out.float()).sum(-1, keepdim=True)      # rowsum(dO * O)
    dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    dkv = torch.zeros(kv.shape, dtype=torch.float32, device=q.device)
    cur = [kv] + ([kmask.contiguous()] if kmask is not None else [])
    for s in range(P):
        j = (r - s) % P
        if not (causal and j > r):
            k, v = cur[0][0], cur[0][1]
            p = torch.exp(_scores(q, k, cur[1] if kmask is not None else None, scale, causal and j == r) - lse)
            dkv[1] += torch.matmul(p.transpose(-1, -2).to(dout.dtype), dout).float()
            dp = torch.matmul(dout, v.transpose(-1, -2)).float()
            ds = (p * (dp - delta) * scale).to(q.dtype)
            dq += torch.matmul(ds, k).float()
            dkv[0] += torch.matmul(ds.transpose(-1, -2), q).float()
        # the K/V block moves on with its gradient; the last hop only returns dK/dV to the owner
        (nxt, reqs) = _rotate(comm, ([dkv] + cur) if s < P - 1 else [dkv])
        for w in reqs:
            w.wait()
        dkv = nxt[0]
        if s < P - 1:
            cur = nxt[1:]
    return dq, dkv


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
        q, kv = _split(qkv, self.B, self.S_l, self.NH, D)
        kmask = input_vals[1].reshape(self.B, self.S_l) if self.has_mask else None
        out, lse = ring_attention_fwd(q, kv, kmask, comm, self.causal, self.scale)
        flat = out.permute(0, 2, 1, 3).reshape(self.B * self.S_l, H)
        return AuxResult(flat, (q, kv, kmask, out, lse))

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
        dflat, (_, (q, kv, kmask, out, lse)) = input_vals
        B, NH, S_l, D = q.shape
        dout = dflat.reshape(B, S_l, NH, D).permute(0, 2, 1, 3)
        dq, dkv = ring_attention_bwd(dout, q, kv, kmask, out, lse, f.comm, f.causal, f.scale)
        d = torch.cat([dq.unsqueeze(0), dkv], 0)                        # [3, B, NH, S_l, D]
        return d.permute(1, 3, 0, 2, 4).reshape(B * S_l, 3 * NH * D).to(dflat.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def ring_attention_op(qkv, mask, batch, local_seq_len, num_heads, comm=None, causal=False, scale=None, ctx=None):
    return RingAttentionOp(qkv, mask, batch, local_seq_len, num_heads, comm, causal, scale, ctx=ctx)
