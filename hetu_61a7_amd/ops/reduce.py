"""Reductions, n-ary sum, sort/select (reference ReduceSum.py, ReduceMean.py,
ReduceSumAxisZero.py, Sum.py, Norm.py, Argmax.py, Argsort.py, TopKIdx.py,
TopKVal.py, Cumsum.py; SURVEY §2.4 "Reductions / sort / select").

Leading/trailing-axis reductions of contiguous tensors run on the HIP
``reduce_mid`` / ``reduce_last`` kernels (fp32 accumulation); other axis sets
fall back to torch reductions.
"""
from __future__ import annotations

import numpy as np
import torch

from .node import Op
from ..kernels import reduce as KR
from .. import ndarray


def _norm_axes(axes, nd):
    if axes is None:
        return list(range(nd))
    if isinstance(axes, int):
        axes = [axes]
    return sorted(a % nd for a in axes)


def _reduce_sum(x, axes, keepdims, scale=1.0):
    nd = x.dim()
    axes = _norm_axes(axes, nd)
    out_shape = [d for i, d in enumerate(x.shape) if i not in axes]
    keep_shape = [1 if i in axes else d for i, d in enumerate(x.shape)]
    if x.is_contiguous() and x.dtype in (torch.float32, torch.bfloat16) and axes:
        # contiguous axis block -> [B, R, C] view
        if axes == list(range(axes[0], axes[-1] + 1)):
            B = int(np.prod(x.shape[:axes[0]])) if axes[0] > 0 else 1
            R = int(np.prod([x.shape[a] for a in axes]))
            C = int(np.prod(x.shape[axes[-1] + 1:])) if axes[-1] < nd - 1 else 1
            if C == 1:
                r = KR.reduce_last(x.reshape(B, R), scale)
            else:
                r = KR.reduce_mid(x.reshape(B, R, C), scale)
            return r.reshape(keep_shape if keepdims else out_shape)
    r = x.float().sum(dim=axes, keepdim=keepdims) * scale
    return r.to(x.dtype)


from ..kernels import native as _native, record_fallback as _record_fallback
from ..kernels import tensor as KT


def _gpu(t):
    return isinstance(t, torch.Tensor) and _native(t) and t.dtype in (torch.float32, torch.bfloat16)


def _fallback(name, t):
    if isinstance(t, torch.Tensor) and t.is_cuda:
        _record_fallback(name)


class ReduceSumOp(Op):
    def __init__(self, node, axes=None, keepdims=False, ctx=None):
        super().__init__(ReduceSumOp, [node], ctx)
        self.axes = axes
        self.keepdims = keepdims if isinstance(keepdims, bool) else bool(np.all(keepdims))

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return _reduce_sum(input_vals[0], self.axes, self.keepdims)

    def gradient(self, output_grad):
        return [ReduceGradOp(output_grad, self.inputs[0], self.axes, self.keepdims, 1.0, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = input_shapes[0]
        axes = _norm_axes(self.axes, len(s))
        if self.keepdims:
            return tuple(1 if i in axes else d for i, d in enumerate(s))
        r = tuple(d for i, d in enumerate(s) if i not in axes)
        return r if r else (1,)


class ReduceMeanOp(ReduceSumOp):
    def __init__(self, node, axes=None, keepdims=False, ctx=None):
        super().__init__(node, axes, keepdims, ctx)
        self.op_type = 'ReduceMeanOp'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        axes = _norm_axes(self.axes, x.dim())
        cnt = int(np.prod([x.shape[a] for a in axes])) if axes else 1
        return _reduce_sum(x, self.axes, self.keepdims, 1.0 / max(cnt, 1))

    def gradient(self, output_grad):
        return [ReduceGradOp(output_grad, self.inputs[0], self.axes, self.keepdims, None, ctx=self.raw_ctx)]


class ReduceGradOp(Op):
    """Broadcast a reduction gradient back; scale None = 1/count (mean)."""
    shape_only_inputs = (1,)

    def __init__(self, grad, ref, axes, keepdims, scale, ctx=None):
        super().__init__(ReduceGradOp, [grad, ref], ctx)
        self.axes, self.keepdims, self.scale = axes, keepdims, scale

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        shape = tuple(shape)
        axes = _norm_axes(self.axes, len(shape))
        keep = [1 if i in axes else d for i, d in enumerate(shape)]
        scale = self.scale
        if scale is None:
            scale = 1.0 / max(int(np.prod([shape[a] for a in axes])), 1)
        g = g.reshape(keep)
        if scale != 1.0:
            from ..kernels import cpu_native
            if (_gpu(g) and g.is_contiguous()) or cpu_native.active(g):
                from ..kernels.elementwise import unary
                g = unary('mul_c', g, float(scale))
            else:
                g = g * scale
        return g.expand(shape)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def reduce_sum_op(node, axes=None, keepdims=False, ctx=None):
    return ReduceSumOp(node, axes, keepdims, ctx=ctx)


def reduce_mean_op(node, axes=None, keepdims=False, ctx=None):
    return ReduceMeanOp(node, axes, keepdims, ctx=ctx)


class ReduceSumAxisZeroOp(Op):
    grad_dest = None   # bias gradients: fp32 slot of the flat gradient buffer

    def __init__(self, node, ctx=None):
        super().__init__(ReduceSumAxisZeroOp, [node], ctx)

    def set_grad_dest(self, dest):
        if dest.dtype == torch.float32 and dest.is_contiguous():
            self.grad_dest = dest
            return True
        return False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0].contiguous()
        d = self.grad_dest
        if d is not None and x.is_cuda and d.numel() == x[0].numel():
            return KR.reduce_mid(x.reshape(1, x.shape[0], -1), out=d.view(1, -1)).reshape(x.shape[1:])
        return KR.reduce_mid(x.reshape(1, x.shape[0], -1)).reshape(x.shape[1:])

    def gradient(self, output_grad):
        from .shape import broadcastto_op
        return [broadcastto_op(output_grad, self.inputs[0], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][1:])


def reducesumaxiszero_op(node, ctx=None):
    return ReduceSumAxisZeroOp(node, ctx=ctx)


class SumOp(Op):
    """N-ary add; IndexedSlices inputs are merged (reference Sum.py:13-193)."""

    def __init__(self, nodes, ctx=None, sparse=False):
        super().__init__(SumOp, list(nodes), ctx)
        self.sparse = sparse

    def compute(self, input_vals, output_val=None, stream_handle=None):
        sparse = [v for v in input_vals if isinstance(v, ndarray.IndexedSlices)]
        dense = [v for v in input_vals if not isinstance(v, ndarray.IndexedSlices)]
        if sparse and not dense:
            r = sparse[0]
            for s in sparse[1:]:
                r = r.merge(s)
            return r
        dt = max(dense, key=lambda t: t.numel()).dtype
        acc = None
        from ..kernels import cpu_native
        if all(_gpu(v) for v in dense) or (dense and cpu_native.active(*dense)):
            from ..kernels.elementwise import binary, cast
            for v in dense:          # native adds (mixed bf16 / fp32 operands read as they are)
                if acc is None:
                    acc = v if v.dtype == dt else cast(v.contiguous(), dt)
                else:
                    acc = binary('add', acc, v)
            dense = []
        for v in dense:
            acc = v.to(dt) if acc is None else acc + v.to(dt)
        for s in sparse:
            acc = acc + s.to_dense().to(dt)
        return acc

    def gradient(self, output_grad):
        from .basic import reduce_to_shape_op
        return [reduce_to_shape_op(output_grad, n, ctx=self.raw_ctx) for n in self.inputs]

    def infer_shape(self, input_shapes):
        from .basic import _shape_bcast
        s = input_shapes[0]
        for x in input_shapes[1:]:
            s = _shape_bcast(s, x)
        return s


def sum_op(node_list, ctx=None, sparse=False):
    return SumOp(node_list, ctx=ctx, sparse=sparse)


class NormOp(Op):
    def __init__(self, node, axis, p=2, keepdims=True, ctx=None):
        super().__init__(NormOp, [node], ctx)
        self.axis, self.p, self.keepdims = axis, p, keepdims

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if _gpu(x) and isinstance(self.axis, int):
            return KT.pnorm(x, self.axis, self.p, self.keepdims)
        return torch.linalg.vector_norm(x.float(), self.p, dim=self.axis, keepdim=self.keepdims).to(x.dtype)

    def gradient(self, output_grad):
        return [norm_gradient_op(self.inputs[0], self, output_grad, self.axis, self.p, self.keepdims, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        if self.keepdims:
            s[self.axis] = 1
        else:
            s.pop(self.axis)
        return tuple(s)


class NormGradientOp(Op):
    def __init__(self, x, y, g, axis, p, keepdims=True, ctx=None):
        super().__init__(NormGradientOp, [x, y, g], ctx)
        self.axis, self.p, self.keepdims = axis, p, keepdims

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, y, g = input_vals
        if not self.keepdims:
            y, g = y.unsqueeze(self.axis), g.unsqueeze(self.axis)
        if _gpu(x) and isinstance(self.axis, int):
            return KT.pnorm_grad(x, y, g, self.axis, self.p)
        xf = x.float()
        d = torch.sign(xf) * torch.abs(xf) ** (self.p - 1) / (y.float() ** (self.p - 1)).clamp_min(1e-12)
        return (d * g.float()).to(x.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def norm_op(node, axis, p=2, keepdims=True, ctx=None):
    return NormOp(node, axis, p, keepdims, ctx=ctx)


def norm_gradient_op(node, node_y, grad_y, axis, p, keepdims=True, ctx=None):
    return NormGradientOp(node, node_y, grad_y, axis, p, keepdims, ctx=ctx)


class ArgmaxOp(Op):
    def __init__(self, node, dim=0, ctx=None):
        super().__init__(ArgmaxOp, [node], ctx)
        self.dim = dim

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if _gpu(input_vals[0]):
            return KT.argmax(input_vals[0], self.dim)
        return torch.argmax(input_vals[0], self.dim)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        s.pop(self.dim)
        return tuple(s)


def argmax_op(node, dim=0, ctx=None):
    return ArgmaxOp(node, dim, ctx=ctx)


class ArgsortOp(Op):
    def __init__(self, node, dim=1, descending=False, ctx=None):
        super().__init__(ArgsortOp, [node], ctx)
        self.dim, self.descending = dim, descending

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if _gpu(x):
            r = KT.argsort(x, self.dim, self.descending)
            if r is not None:
                return r
            _fallback('argsort', x)
        return torch.argsort(x, dim=self.dim, descending=self.descending)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def argsort_op(node, dim=1, descending=False, ctx=None):
    return ArgsortOp(node, dim, descending, ctx=ctx)


class TopKIdxOp(Op):
    def __init__(self, node, topk, ctx=None):
        super().__init__(TopKIdxOp, [node], ctx)
        self.k = topk

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import moe as KM
        return KM.topk(input_vals[0], self.k)[1]

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][:-1]) + (self.k,)


def topk_idx_op(node, topk, ctx=None):
    return TopKIdxOp(node, topk, ctx=ctx)


class TopKValOp(Op):
    """Values of ``values`` at ``indices`` along the last dim."""

    def __init__(self, values, indices, ctx=None):
        super().__init__(TopKValOp, [values, indices], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        v, i = input_vals
        if _gpu(v):
            return KT.gather(v, -1, i)
        return torch.gather(v, -1, i.long())

    def gradient(self, output_grad):
        from .shape import gather_gradient_op
        return [gather_gradient_op(self.inputs[0], output_grad, -1, self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def topk_val_op(nodeA, nodeB, ctx=None):
    return TopKValOp(nodeA, nodeB, ctx=ctx)


class CumsumOp(Op):
    def __init__(self, node, bias=-1, dim=0, ctx=None):
        super().__init__(CumsumOp, [node], ctx)
        self.bias, self.dim = bias, dim

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if _gpu(input_vals[0]):
            return KT.cumsum(input_vals[0], self.dim, self.bias)
        x = input_vals[0].float()
        d = self.dim % x.dim()
        if x.is_cuda and d != x.dim() - 1 and x.shape[d] > 4 * x.numel() // max(x.shape[d], 1):
            # long scan over few columns: an outer-dim scan runs one serial thread
            # per column -- scan the innermost dim of the transposed copy instead
            return torch.cumsum(x.transpose(d, -1).contiguous(), -1).transpose(d, -1) + self.bias
        return torch.cumsum(x, self.dim) + self.bias

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def cumsum_with_bias_op(node, bias=-1, dim=0, ctx=None):
    return CumsumOp(node, bias, dim, ctx=ctx)
