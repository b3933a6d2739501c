"""Scaled-dot-product attention as ONE graph op (forward) + ONE gradient op.

The reference materialises attention as batch_matmul -> broadcast mask add ->
softmax -> dropout -> batch_matmul, i.e. ~8 graph nodes and their grads
(examples/nlp/bert/hetu_bert.py:220-270, hetu_transformer.py:99-130).  Here the
chain is a single op so the executor keeps only (P, seed) for backward and the
kernels run back to back on the compute stream: QK^T and PV are the bf16 MFMA
batched GEMM (``gemm.hip`` via ``kernels.gemm.bmm``), the masked softmax and
dropout are the wave64 HIP kernels.

q, k, v: [B, H, S, D]; mask: additive, broadcastable to [B, H, S, S] (BERT's
[B, 1, 1, S] extended mask), or None; ``causal`` adds the upper-triangular -inf.
"""
from __future__ import annotations

import math

import torch

from .node import Op, OutputSelectOp
from .nn import AuxResult
from ..kernels import gemm as KG, softmax as KS, dropout as KD


def _scores(q, k, mask, scale, causal):
    s = KG.bmm(q, k, False, True)
    s = s.float() * scale
    if mask is not None:
        s = s + mask.float()
    if causal:
        S = s.shape[-1]
        tri = torch.triu(torch.ones(S, S, dtype=torch.bool, device=s.device), 1)
        s = s.masked_fill(tri, float('-inf'))
    return s



def _next_seed(key, x):
    from .nn import _next_seed as ns
    return ns(key, x)


class AttentionOp(Op):
    def __init__(self, q, k, v, mask=None, dropout=0.0, causal=False, scale=None, ctx=None):
        inputs = [q, k, v] + ([mask] if mask is not None else [])
        super().__init__(AttentionOp, inputs, ctx)
        self.has_mask = mask is not None
        self.keep_prob = 1.0 - float(dropout)
        self.causal = causal
        self.scale = scale
        self.seed = 0
        self.inference = False

    def _scale(self, d):
        return self.scale if self.scale is not None else 1.0 / math.sqrt(d)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        q, k, v = input_vals[:3]
        mask = input_vals[3] if self.has_mask else None
        from ..kernels import attention as KA
        if q.is_cuda and KA.seqblock_ok(q, k, v, mask, self.causal):
            # BERT-length head views of token-major rows: the one-workgroup-per-head kernels
            keep = 1.0 if self.inference else self.keep_prob
            seed = _next_seed(self.id, q) if keep < 1.0 else 0
            o, lse = KA.seqblock_fwd(q, k, v, mask, keep, seed, self._scale(q.shape[-1]))
            return AuxResult(o, ('seqblock', lse, keep, seed))
        if q.is_cuda and KA.flash_ok(q, k, v):
            # one fused kernel: scores, mask, causal mask, online softmax, dropout, P.V
            keep = 1.0 if self.inference else self.keep_prob
            seed = _next_seed(self.id, q) if keep < 1.0 else 0
            o, lse = KA.flash_fwd(q, k, v, mask, self.causal, keep, seed, self._scale(q.shape[-1]))
            return AuxResult(o, ('flash', lse, keep, seed))
        if q.is_cuda:
            raise RuntimeError('attention_op: no hand-written kernel for %s %s (head dim 32/64/128, bf16)'
                               % (q.dtype, tuple(q.shape)))
        s = _scores(q, k, mask, self._scale(q.shape[-1]), self.causal)
        p = KS.softmax(s.to(q.dtype) if q.dtype == torch.bfloat16 else s)
        seed = None
        pd = p
        if self.keep_prob < 1.0 and not self.inference:
            seed = _next_seed(self.id, q)
            pd = KD.dropout(p, self.keep_prob, seed)
        o = KG.bmm(pd.to(v.dtype), v, False, False)
        return AuxResult(o, (p, seed))

    def gradient(self, output_grad):
        g = AttentionGradientOp(output_grad, self, ctx=self.raw_ctx)
        grads = [OutputSelectOp(g, i, ctx=self.raw_ctx) for i in range(3)]
        return grads + ([None] if self.has_mask else [])

    def infer_shape(self, input_shapes):
        q, v = input_shapes[0], input_shapes[2]
        return tuple(q[:-1]) + (v[-1],)


class AttentionGradientOp(Op):
    """(dq, dk, dv) from dO and the saved probabilities P (dropout mask
    regenerated from its seed, as the reference's recompute dropout)."""
    value_and_aux_inputs = (1,)

    def __init__(self, dout, fwd, ctx=None):
        # the mask (if any) rides along: the flash backward recomputes P from it
        super().__init__(AttentionGradientOp, [dout, fwd] + fwd.inputs[:3] + fwd.inputs[3:4], ctx)
        self.fwd = fwd

    def compute(self, input_vals, output_val=None, stream_handle=None):
        do, (o, aux), q, k, v = input_vals[:5]
        f = self.fwd
        if aux[0] == 'seqblock':
            from ..kernels import attention as KA
            _, lse, keep, seed = aux
            mask = input_vals[5] if f.has_mask else None
            return KA.seqblock_bwd(do, q, k, v, o, lse, mask, keep, seed, f._scale(q.shape[-1]))
        if aux[0] == 'flash':
            from ..kernels import attention as KA
            _, lse, keep, seed = aux
            mask = input_vals[5] if f.has_mask else None
            return KA.flash_bwd(do, q, k, v, o, lse, mask, f.causal, keep, seed, f._scale(q.shape[-1]))
        p, seed = aux
        dt = q.dtype
        pd = p if seed is None else KD.dropout(p, f.keep_prob, seed)
        dv = KG.bmm(pd.to(dt), do.to(dt), True, False)
        dpd = KG.bmm(do.to(dt), v, False, True)
        if seed is not None:
            dp = KD.dropout(dpd, f.keep_prob, seed)  # same mask and 1/keep scale
        else:
            dp = dpd
        ds = KS.softmax_backward(p, dp.to(p.dtype))
        scale = f._scale(q.shape[-1])
        ds = (ds.float() * scale).to(dt)
        dq = KG.bmm(ds, k, False, False)
        dk = KG.bmm(ds, q, True, False)
        return (dq, dk, dv)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return (input_shapes[2], input_shapes[3], input_shapes[4])


def attention_op(q, k, v, mask=None, dropout=0.0, causal=False, scale=None, ctx=None):
    return AttentionOp(q, k, v, mask, dropout, causal, scale, ctx=ctx)


# ---------------------------------------------------------------------------
# Packed-QKV fused attention (MI355X path for the BERT / Transformer encoder):
# one HIP kernel forward, one backward, reading Q/K/V out of the QKV projection
# and producing the gradient as one packed tensor.
class PackedAttentionOp(Op):
    """out [B*S, H] = MHA(qkv [B*S, 3H]); mask: additive key mask [B, S] (or None)."""

    def __init__(self, qkv, mask, batch, seq_len, num_heads, dropout=0.0, scale=None, ctx=None):
        super().__init__(PackedAttentionOp, [qkv] + ([mask] if mask is not None else []), ctx)
        self.has_mask = mask is not None
        self.B, self.S, self.NH = int(batch), int(seq_len), int(num_heads)
        self.keep_prob = 1.0 - float(dropout)
        self.scale = scale
        self.seed = 0
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import attention as KA
        qkv = input_vals[0]
        mask = input_vals[1].reshape(self.B, self.S) if self.has_mask else None
        keep = 1.0 if self.inference else self.keep_prob
        seed = _next_seed(self.id, qkv) if keep < 1.0 else 0
        out, saved = KA.attention_fwd(qkv.contiguous(), mask, self.B, self.S, self.NH, keep, seed, self.scale)
        return AuxResult(out, (saved, keep, seed))

    def gradient(self, output_grad):
        g = PackedAttentionGradientOp(output_grad, self, ctx=self.raw_ctx)
        return [g] + ([None] if self.has_mask else [])

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], input_shapes[0][1] // 3)


class PackedAttentionGradientOp(Op):
    value_and_aux_inputs = (1,)

    def __init__(self, dout, fwd, ctx=None):
        super().__init__(PackedAttentionGradientOp, [dout, fwd] + fwd.inputs, ctx)
        self.fwd = fwd

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import attention as KA
        f = self.fwd
        dout, (out, (saved, keep, seed)), qkv = input_vals[:3]
        mask = input_vals[3].reshape(f.B, f.S) if f.has_mask else None
        return KA.attention_bwd(dout, qkv.contiguous(), out, saved, mask, f.B, f.S, f.NH, keep, seed, f.scale)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def packed_attention_op(qkv, mask, batch, seq_len, num_heads, dropout=0.0, scale=None, ctx=None):
    return PackedAttentionOp(qkv, mask, batch, seq_len, num_heads, dropout, scale, ctx=ctx)
