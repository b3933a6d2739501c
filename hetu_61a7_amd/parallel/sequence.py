"""Sequence parallelism for long contexts: Ulysses attention (SURVEY §2.3 S13,
§5.7 -- absent in the reference, planned for the MI355X build).

Each of the P ranks of a sequence-parallel group holds ``S/P`` consecutive
tokens of every sequence: ``qkv`` [B*S/P, 3H] (the packed QKV projection of
its tokens) and the key mask slice [B, S/P].  One all-to-all over the xGMI
mesh regroups Q/K/V from "all heads, my tokens" to "my NH/P heads, all
tokens", the fused packed-QKV attention kernel (``kernels.attention``) runs on
the full sequence for those heads, and a second all-to-all returns the context
to the token sharding [B*S/P, H].  The backward mirrors the two exchanges
around the fused backward kernel, so the S x S score matrix never exists and
each GPU moves 2 x (P-1)/P of its activations per layer -- the same
mesh-shaped traffic as the MoE all-to-all.

Everything outside attention (projections, LayerNorm, FFN) is token-parallel
and runs unchanged on the local tokens.
"""
from __future__ import annotations

import torch

from ..ops.node import Op
from ..ops.nn import AuxResult


def _a2a(comm, x):
    out = torch.empty_like(x)
    comm.all_to_all(out, x.contiguous())
    return out


def scatter_heads(qkv, comm, B, S_l, NH, D):
    """[B*S_l, 3*NH*D] (all heads, my tokens) -> [B*S, 3*(NH/P)*D] (my heads, all tokens)."""
    P = comm.nrank
    hl = NH // P
    x = qkv.reshape(B, S_l, 3, P, hl, D).permute(3, 0, 1, 2, 4, 5).contiguous()   # [P(dst), B, S_l, 3, hl, D]
    y = _a2a(comm, x.reshape(P, -1)).reshape(P, B, S_l, 3, hl, D)                # [P(src seq chunk), ...]
    return y.permute(1, 0, 2, 3, 4, 5).reshape(B * P * S_l, 3 * hl * D)


def gather_heads(out, comm, B, S_l, NH, D):
    """[B*S, (NH/P)*D] (my heads, all tokens) -> [B*S_l, NH*D] (all heads, my tokens)."""
    P = comm.nrank
    hl = NH // P
    x = out.reshape(B, P, S_l, hl, D).permute(1, 0, 2, 3, 4).contiguous()          # [P(dst seq chunk), B, S_l, hl, D]
    y = _a2a(comm, x.reshape(P, -1)).reshape(P, B, S_l, hl, D)                    # [P(src head group), ...]
    return y.permute(1, 2, 0, 3, 4).reshape(B * S_l, NH * D)


def scatter_heads_grad(dqkv_full, comm, B, S_l, NH, D):
    """Adjoint of scatter_heads: [B*S, 3*(NH/P)*D] -> [B*S_l, 3*NH*D]."""
    P = comm.nrank
    hl = NH // P
    x = dqkv_full.reshape(B, P, S_l, 3, hl, D).permute(1, 0, 2, 3, 4, 5).contiguous()   # [P(dst seq), ...]
    y = _a2a(comm, x.reshape(P, -1)).reshape(P, B, S_l, 3, hl, D)                        # [P(src heads), ...]
    return y.permute(1, 2, 3, 0, 4, 5).reshape(B * S_l, 3 * NH * D)


def gather_heads_grad(dout_local, comm, B, S_l, NH, D):
    """Adjoint of gather_heads: [B*S_l, NH*D] -> [B*S, (NH/P)*D]."""
    P = comm.nrank
    hl = NH // P
    x = dout_local.reshape(B, S_l, P, hl, D).permute(2, 0, 1, 3, 4).contiguous()   # [P(dst heads), B, S_l, hl, D]
    y = _a2a(comm, x.reshape(P, -1)).reshape(P, B, S_l, hl, D)                     # [P(src seq), ...]
    return y.permute(1, 0, 2, 3, 4).reshape(B * P * S_l, hl * D)


class UlyssesAttentionOp(Op):
    """out [B*S/P, H] = MHA over the whole sequence, sequence-sharded over ``comm``."""

    def __init__(self, qkv, mask, batch, local_seq_len, num_heads, comm=None, dropout=0.0, scale=None, ctx=None):
        super().__init__(UlyssesAttentionOp, [qkv] + ([mask] if mask is not None else []), ctx)
        self.has_mask = mask is not None
        self.B, self.S_l, self.NH = int(batch), int(local_seq_len), int(num_heads)
        self.comm = comm
        self.keep_prob = 1.0 - float(dropout)
        self.scale = scale
        self.seed = 0
        self.inference = False

    def _comm(self):
        from . import comm as C
        if self.comm is None:
            self.comm = C.init_process_group()
        return self.comm

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import attention as KA
        comm = self._comm()
        P = comm.nrank
        qkv = input_vals[0]
        H = qkv.shape[1] // 3
        D = H // self.NH
        assert self.NH % P == 0, 'heads (%d) must divide over the sequence-parallel group (%d)' % (self.NH, P)
        S = self.S_l * P
        mask = None
        if self.has_mask:
            ml = input_vals[1].reshape(self.B, self.S_l).float().contiguous()
            full = torch.empty((P * self.B, self.S_l), dtype=ml.dtype, device=ml.device)
            comm.all_gather(full, ml)                                    # [P, B, S_l] -> [B, S]
            mask = full.reshape(P, self.B, self.S_l).permute(1, 0, 2).reshape(self.B, S)
        keep = 1.0 if self.inference else self.keep_prob
        seed = 0
        if keep < 1.0:
            from ..ops.nn import _next_seed
            seed = _next_seed(self.id, qkv) ^ ((comm.rank + 1) << 48)   # distinct masks per head group
        qkv_full = scatter_heads(qkv, comm, self.B, self.S_l, self.NH, D)
        out_full, saved = KA.attention_fwd(qkv_full, mask, self.B, S, self.NH // P, keep, seed, self.scale)
        out = gather_heads(out_full, comm, self.B, self.S_l, self.NH, D)
        return AuxResult(out, (qkv_full, out_full, saved, mask, keep, seed))

    def gradient(self, output_grad):
        return [UlyssesAttentionGradientOp(output_grad, self, ctx=self.raw_ctx)] + ([None] if self.has_mask else [])

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], input_shapes[0][1] // 3)


class UlyssesAttentionGradientOp(Op):
    value_and_aux_inputs = (1,)

    def __init__(self, dout, fwd, ctx=None):
        super().__init__(UlyssesAttentionGradientOp, [dout, fwd], ctx)
        self.fwd = fwd

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import attention as KA
        f = self.fwd
        comm = f.comm
        P = comm.nrank
        dout, (out, (qkv_full, out_full, saved, mask, keep, seed)) = input_vals
        H = out.shape[1]
        D = H // f.NH
        S = f.S_l * P
        dfull = gather_heads_grad(dout.to(qkv_full.dtype), comm, f.B, f.S_l, f.NH, D)
        dqkv_full = KA.attention_bwd(dfull, qkv_full, out_full, saved, mask, f.B, S, f.NH // P, keep, seed, f.scale)
        return scatter_heads_grad(dqkv_full, comm, f.B, f.S_l, f.NH, D)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def ulysses_attention_op(qkv, mask, batch, local_seq_len, num_heads, comm=None, dropout=0.0, scale=None, ctx=None):
    return UlyssesAttentionOp(qkv, mask, batch, local_seq_len, num_heads, comm, dropout, scale, ctx=ctx)
