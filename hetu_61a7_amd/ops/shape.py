"""Shape / layout / indexing operators.

Parity: reference gpu_ops Reshape.py, Transpose.py, Broadcast.py,
BroadcastShape.py, Slice.py, SliceAssign.py, SliceByMatrix.py, Split.py,
Concat.py, Concatenate.py, Pad.py, Repeat.py, Roll.py, Interpolate.py,
Gather.py, Indexing.py, Scatter.py, Scatter1D.py, Conv2dBroadcast.py,
Conv2dReduceSum.py (SURVEY §2.4 "Shape / layout / indexing").

Reshape, slice, transpose and broadcast are zero-copy views whenever the
source layout allows (the reference needs ``enable_lazy`` plus a lazy-callback
kernel for this); consumers that need dense memory call ``.contiguous()``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from .. import native_array as _NA

from ..kernels import native as _native, record_fallback as _record_fallback
from ..kernels import tensor as KT


def _gpu(t):
    """hand-written kernel path for a GPU tensor (kernels.native)"""
    return isinstance(t, torch.Tensor) and _native(t)


def _cpu(*ts):
    """native C++ CPU backend for fp32 host tensors (kernels.cpu_native)"""
    from ..kernels import cpu_native
    return all(isinstance(t, torch.Tensor) for t in ts) and cpu_native.active(*ts)


def _fallback(name, t):
    if isinstance(t, torch.Tensor) and t.is_cuda:
        _record_fallback(name)

from .node import Op
from .basic import reduce_to_shape_op, _shape_bcast
from ..kernels import reduce as KR


def _resolve_shape(shape, numel):
    shape = list(shape)
    if -1 in shape:
        known = 1
        for s in shape:
            if s != -1:
                known *= s
        shape[shape.index(-1)] = numel // known
    return tuple(shape)


class Array_ReshapeOp(Op):
    def __init__(self, node, output_shape, ctx=None):
        super().__init__(Array_ReshapeOp, [node], ctx)
        self.output_shape = tuple(output_shape)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        shp = _resolve_shape(self.output_shape, x.numel())
        if x.dim() == 4 and not x.is_contiguous():
            x = x.contiguous()
        return x.reshape(shp)

    def gradient(self, output_grad):
        return [array_reshape_gradient_op(self.inputs[0], output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return _resolve_shape(self.output_shape, int(np.prod(input_shapes[0])))


class Array_Reshape_GradientOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, node_in, node_out, ctx=None):
        super().__init__(Array_Reshape_GradientOp, [node_in, node_out], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        shape, g = input_vals
        return g.reshape(tuple(shape))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def array_reshape_op(node, output_shape, ctx=None):
    return Array_ReshapeOp(node, output_shape, ctx=ctx)


def array_reshape_gradient_op(node_in, node_out, ctx=None):
    return Array_Reshape_GradientOp(node_in, node_out, ctx=ctx)


class TransposeOp(Op):
    def __init__(self, node, perm=None, ctx=None):
        super().__init__(TransposeOp, [node], ctx)
        self.perm = perm

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        perm = self.perm if self.perm is not None else list(range(x.dim()))[::-1]
        return x.permute(*perm)

    def gradient(self, output_grad):
        if self.perm is None:
            return [transpose_op(output_grad, None, ctx=self.raw_ctx)]
        inv = list(np.argsort(self.perm))
        return [transpose_op(output_grad, inv, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = input_shapes[0]
        perm = self.perm if self.perm is not None else list(range(len(s)))[::-1]
        return tuple(s[p] for p in perm)


def transpose_op(node_A, perm=None, ctx=None):
    return TransposeOp(node_A, perm, ctx=ctx)


class BroadcastToOp(Op):
    """Broadcast A to the shape of B (B used for its shape only)."""
    shape_only_inputs = (1,)

    def __init__(self, a, b, ctx=None):
        super().__init__(BroadcastToOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, shape = input_vals
        shape = tuple(shape)
        if x.dim() < len(shape) and tuple(x.shape) != shape[len(shape) - x.dim():]:
            # reference semantics: leading-aligned when trailing does not match
            x = x.reshape(tuple(x.shape) + (1,) * (len(shape) - x.dim()))
        return x.expand(shape)

    def gradient(self, output_grad):
        return [reduce_to_shape_op(output_grad, self.inputs[0], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def broadcastto_op(node_A, node_B, ctx=None):
    return BroadcastToOp(node_A, node_B, ctx=ctx)


class BroadcastShapeOp(Op):
    def __init__(self, node, shape, add_axes=(), ctx=None):
        super().__init__(BroadcastShapeOp, [node], ctx)
        self.shape, self.add_axes = tuple(shape), tuple(add_axes)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if self.add_axes:
            for ax in sorted(self.add_axes):
                x = x.unsqueeze(ax)
        return x.expand(self.shape)

    def gradient(self, output_grad):
        return [reduce_to_shape_op(output_grad, self.inputs[0], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return self.shape


def broadcast_shape_op(node_A, shape, add_axes=(), ctx=None):
    return BroadcastShapeOp(node_A, shape, add_axes, ctx=ctx)


def _slices(begin, size, shape):
    sl = []
    for b, s, d in zip(begin, size, shape):
        e = d if s == -1 else b + s
        sl.append(slice(b, e))
    return tuple(sl)


class SliceOp(Op):
    def __init__(self, node, begin, size, ctx=None):
        super().__init__(SliceOp, [node], ctx)
        self.begin, self.size = tuple(begin), tuple(size)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        return x[_slices(self.begin, self.size, x.shape)]

    def gradient(self, output_grad):
        return [slice_gradient_op(output_grad, self.begin, self.inputs[0], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return tuple((d - b) if s == -1 else s for b, s, d in zip(self.begin, self.size, input_shapes[0]))


class SliceGradientOp(Op):
    shape_only_inputs = (1,)

    def __init__(self, grad, begin, ref, ctx=None):
        super().__init__(SliceGradientOp, [grad, ref], ctx)
        self.begin = tuple(begin)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        if g.is_cuda:
            from ..kernels.tensor import zeros, copy_into
            out = zeros(tuple(shape), g.dtype, g.device)
            copy_into(out[_slices(self.begin, g.shape, shape)], g)
            return out
        out = _NA.zeros(tuple(shape), dtype=g.dtype, device=g.device)
        out[_slices(self.begin, g.shape, shape)] = g
        return out

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def slice_op(node, begin, size, ctx=None):
    return SliceOp(node, begin, size, ctx=ctx)


def slice_gradient_op(node, begin, size=None, ctx=None):
    # reference signature (grad, begin, size); here the third argument may be
    # the forward input node (shape source) or an explicit output shape
    if isinstance(size, Op):
        return SliceGradientOp(node, begin, size, ctx=ctx)
    op = SliceGradientOp(node, begin, node, ctx=ctx)
    op.explicit_shape = tuple(size)
    op.shape_only_inputs = ()
    op.inputs = [node]

    def compute(input_vals, output_val=None, stream_handle=None, _op=op):
        g = input_vals[0]
        out = _NA.zeros(_op.explicit_shape, dtype=g.dtype, device=g.device)
        out[_slices(_op.begin, g.shape, _op.explicit_shape)] = g
        return out
    op.compute = compute
    return op


class SliceAssignOp(Op):
    def __init__(self, node, begin, size, val, ctx=None):
        super().__init__(SliceAssignOp, [node], ctx)
        self.begin, self.size, self.val = tuple(begin), tuple(size), val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0].clone()
        x[_slices(self.begin, self.size, x.shape)] = self.val
        return x

    def gradient(self, output_grad):
        return [SliceAssignOp(output_grad, self.begin, self.size, 0.0, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class SliceAssignMatrixOp(Op):
    def __init__(self, a, b, begin_a, size_a, begin_b, size_b, ctx=None):
        super().__init__(SliceAssignMatrixOp, [a, b], ctx)
        self.ba, self.sa, self.bb, self.sb = tuple(begin_a), tuple(size_a), tuple(begin_b), tuple(size_b)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        x = a.clone()
        x[_slices(self.ba, self.sa, x.shape)] = b[_slices(self.bb, self.sb, b.shape)].to(x.dtype)
        return x

    def gradient(self, output_grad):
        return [SliceAssignOp(output_grad, self.ba, self.sa, 0.0, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def slice_assign_op(node, begin, size, val, ctx=None):
    return SliceAssignOp(node, begin, size, val, ctx=ctx)


def slice_assign_matrix_op(node_A, node_B, begin_A, size_A, begin_B, size_B, ctx=None):
    return SliceAssignMatrixOp(node_A, node_B, begin_A, size_A, begin_B, size_B, ctx=ctx)


class SliceByMatrixOp(Op):
    """out[r, :] = in[i1[r], i2[r], :] (reference SliceByMatrix.cu)."""

    def __init__(self, a, i1, i2, ctx=None):
        super().__init__(SliceByMatrixOp, [a, i1, i2], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, i1, i2 = input_vals
        return a[i1.long().reshape(-1), i2.long().reshape(-1)]

    def gradient(self, output_grad):
        return [slice_by_matrix_gradient_op(self.inputs[0], output_grad, self.inputs[1], self.inputs[2], ctx=self.raw_ctx), None, None]

    def infer_shape(self, input_shapes):
        return (int(np.prod(input_shapes[1])), input_shapes[0][-1])


class SliceByMatrixGradientOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, ref, grad, i1, i2, ctx=None):
        super().__init__(SliceByMatrixGradientOp, [ref, grad, i1, i2], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        shape, g, i1, i2 = input_vals
        out = _NA.zeros(tuple(shape), dtype=torch.float32, device=g.device)
        out.index_put_((i1.long().reshape(-1), i2.long().reshape(-1)), g.float(), accumulate=True)
        return out.to(g.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def slice_by_matrix_op(node_A, index1, index2, ctx=None):
    return SliceByMatrixOp(node_A, index1, index2, ctx=ctx)


def slice_by_matrix_gradient_op(input, grad, index1, index2, ctx=None):
    return SliceByMatrixGradientOp(input, grad, index1, index2, ctx=ctx)


def _split_slices(shape, axes, indices, splits):
    sl = [slice(None)] * len(shape)
    for ax, ind, spl in zip(axes, indices, splits):
        part = shape[ax] // spl
        b = ind * part
        e = b + part if ind != spl - 1 else shape[ax]
        sl[ax] = slice(b, e)
    return tuple(sl)


class SplitOp(Op):
    def __init__(self, node, axes, indices, splits, ctx=None):
        super().__init__(SplitOp, [node], ctx)
        self.axes, self.indices, self.splits = list(axes), list(indices), list(splits)
        assert len(self.axes) == len(self.splits)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        return x[_split_slices(x.shape, self.axes, self.indices, self.splits)]

    def gradient(self, output_grad):
        return [SplitGradientOp(output_grad, self.inputs[0], self.axes, self.indices, self.splits, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        for ax, ind, spl in zip(self.axes, self.indices, self.splits):
            part = s[ax] // spl
            s[ax] = part if ind != spl - 1 else s[ax] - ind * part
        return tuple(s)


class SplitGradientOp(Op):
    shape_only_inputs = (1,)

    def __init__(self, grad, ref, axes, indices, splits, ctx=None):
        super().__init__(SplitGradientOp, [grad, ref], ctx)
        self.axes, self.indices, self.splits = axes, indices, splits

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        out = _NA.zeros(tuple(shape), dtype=g.dtype, device=g.device)
        out[_split_slices(tuple(shape), self.axes, self.indices, self.splits)] = g
        return out

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def split_op(node, axes, indices, splits, ctx=None):
    return SplitOp(node, axes, indices, splits, ctx=ctx)


def split_gradient_op(node, axes, indices, splits, ref=None, ctx=None):
    return SplitGradientOp(node, ref if ref is not None else node, axes, indices, splits, ctx=ctx)


class ConcatenateOp(Op):
    """N-input concat in a single launch (reference Concatenate.py)."""

    def __init__(self, nodes, axis=0, ctx=None):
        super().__init__(ConcatenateOp, list(nodes), ctx)
        self.axis = axis

    def compute(self, input_vals, output_val=None, stream_handle=None):
        dt = input_vals[0].dtype
        if _gpu(input_vals[0]) or _cpu(*input_vals):
            return KT.concat([v.to(dt) for v in input_vals], self.axis)
        return torch.cat([v.to(dt) for v in input_vals], self.axis)

    def gradient(self, output_grad):
        return [ConcatGradientOp(output_grad, n, self.inputs, i, self.axis, ctx=self.raw_ctx)
                for i, n in enumerate(self.inputs)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        s[self.axis] = sum(x[self.axis] for x in input_shapes)
        return tuple(s)


class ConcatGradientOp(Op):
    """Slice of the concat gradient belonging to input ``idx``."""

    def __init__(self, grad, node, all_nodes, idx, axis, ctx=None):
        super().__init__(ConcatGradientOp, [grad] + list(all_nodes), ctx)
        self.idx, self.axis = idx, axis
        self.shape_only_inputs = tuple(range(1, len(all_nodes) + 1))

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g = input_vals[0]
        shapes = input_vals[1:]
        off = sum(s[self.axis] for s in shapes[:self.idx])
        return g.narrow(self.axis, off, shapes[self.idx][self.axis])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1 + self.idx]


def concatenate_op(node_list, axis=0, ctx=None):
    return ConcatenateOp(node_list, axis, ctx=ctx)


def concatenate_gradient_op(grad_node, input_node, axis, idx=0, all_nodes=None, ctx=None):
    return ConcatGradientOp(grad_node, input_node, all_nodes or [input_node], idx, axis, ctx=ctx)


def concat_op(node_A, node_B, axis=0, ctx=None):
    op = ConcatenateOp([node_A, node_B], axis, ctx=ctx)
    op.op_type = 'ConcatOp'
    return op


def concat_gradient_op(grad_node, input_node, axis, idx, all_nodes=None, ctx=None):
    return ConcatGradientOp(grad_node, input_node, all_nodes or [input_node], idx, axis, ctx=ctx)


class PadOp(Op):
    def __init__(self, node, paddings, mode='CONSTANT', constant_values=0, ctx=None):
        super().__init__(PadOp, [node], ctx)
        self.paddings, self.mode, self.constant_values = [list(p) for p in paddings], mode.lower(), constant_values

    def _torch_pad(self):
        pads = []
        for p in reversed(self.paddings):
            pads += [p[0], p[1]]
        return pads

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        nd = x.dim()
        padl = [[0, 0]] * (nd - len(self.paddings)) + self.paddings
        pads = []
        for p in reversed(padl):
            pads += [p[0], p[1]]
        if self.mode == 'constant':
            if _gpu(x) or _cpu(x):
                return KT.pad_constant(x, padl, self.constant_values)
            return F.pad(x, pads, 'constant', self.constant_values)
        _fallback('pad_' + self.mode, x)
        return F.pad(x, pads, self.mode)

    def gradient(self, output_grad):
        return [pad_gradient_op(output_grad, self.paddings, self.mode, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        off = len(s) - len(self.paddings)
        for i, p in enumerate(self.paddings):
            s[off + i] += p[0] + p[1]
        return tuple(s)


class PadGradientOp(Op):
    def __init__(self, grad, paddings, mode='CONSTANT', ctx=None):
        super().__init__(PadGradientOp, [grad], ctx)
        self.paddings = [list(p) for p in paddings]

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g = input_vals[0]
        off = g.dim() - len(self.paddings)
        if _gpu(g) or _cpu(g):
            return KT.unpad(g, [[0, 0]] * off + self.paddings)
        sl = [slice(None)] * off + [slice(p[0], g.shape[off + i] - p[1]) for i, p in enumerate(self.paddings)]
        return g[tuple(sl)]

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        off = len(s) - len(self.paddings)
        for i, p in enumerate(self.paddings):
            s[off + i] -= p[0] + p[1]
        return tuple(s)


def pad_op(node_A, paddings, mode='CONSTANT', constant_values=0, ctx=None):
    return PadOp(node_A, paddings, mode, constant_values, ctx=ctx)


def pad_gradient_op(node_A, paddings, mode='CONSTANT', ctx=None):
    return PadGradientOp(node_A, paddings, mode, ctx=ctx)


class RepeatOp(Op):
    def __init__(self, node, reps, ctx=None):
        super().__init__(RepeatOp, [node], ctx)
        self.reps = tuple(reps)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if _gpu(input_vals[0]) or _cpu(input_vals[0]):
            return KT.repeat(input_vals[0], self.reps)
        return input_vals[0].repeat(*self.reps)

    def gradient(self, output_grad):
        return [repeat_gradient_op(self.inputs[0], output_grad, self.reps, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        s = [1] * (len(self.reps) - len(s)) + s
        return tuple(a * b for a, b in zip(s, self.reps))


class RepeatGradientOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, ref, grad, reps, ctx=None):
        super().__init__(RepeatGradientOp, [ref, grad], ctx)
        self.reps = tuple(reps)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        shape, g = input_vals
        shape = tuple(shape)
        full = (1,) * (len(self.reps) - len(shape)) + shape
        inter = []
        for r, s in zip(self.reps, full):
            inter += [r, s]
        if _gpu(g) or _cpu(g):
            # sum over the tile axes: the interleaved [r0, s0, r1, s1, ...] view reduced
            # over the r axes by the native column reduction
            from ..kernels import reduce as KR
            r = KR.reduce_sum(g.reshape(inter), tuple(range(0, 2 * len(full), 2)))
            return r.reshape(shape).to(g.dtype)
        r = g.reshape(inter).float().sum(dim=tuple(range(0, 2 * len(full), 2)))
        return r.reshape(shape).to(g.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def repeat_op(node, reps, ctx=None):
    return RepeatOp(node, reps, ctx=ctx)


def repeat_gradient_op(node_input, node_grad, reps=None, ctx=None):
    return RepeatGradientOp(node_input, node_grad, reps, ctx=ctx)


class RollOp(Op):
    def __init__(self, node, shift=0, axis=None, ctx=None):
        super().__init__(RollOp, [node], ctx)
        self.shift, self.axis = shift, axis

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if _gpu(x):
            if self.axis is None:
                return KT.roll(x.reshape(-1), [self.shift], [0]).reshape(x.shape)
            sh = list(self.shift) if isinstance(self.shift, (list, tuple)) else [self.shift]
            ax = list(self.axis) if isinstance(self.axis, (list, tuple)) else [self.axis]
            return KT.roll(x, sh, ax)
        return torch.roll(x, self.shift, self.axis)

    def gradient(self, output_grad):
        neg = [-s for s in self.shift] if isinstance(self.shift, (list, tuple)) else -self.shift
        return [RollOp(output_grad, neg, self.axis, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def roll_op(node, shift=0, axis=None, ctx=None):
    return RollOp(node, shift, axis, ctx=ctx)


class InterpolateOp(Op):
    def __init__(self, node, size=None, scale_factor=None, mode='bicubic', align_corners=False, ctx=None):
        super().__init__(InterpolateOp, [node], ctx)
        self.size, self.scale_factor, self.mode, self.align_corners = size, scale_factor, mode, align_corners

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if _gpu(x) and self.mode == 'bicubic' and x.dtype in (torch.float32, torch.bfloat16):
            oh, ow = self.infer_shape([tuple(x.shape)])[2:]
            return KT.bicubic(x, oh, ow, self.align_corners, None if self.size is not None else self.scale_factor)
        if _gpu(x):
            _record_fallback('interpolate_' + str(self.mode))
        return F.interpolate(x.float(), size=self.size, scale_factor=self.scale_factor, mode=self.mode,
                             align_corners=self.align_corners).to(x.dtype)

    def gradient(self, output_grad):
        return [interpolate_grad_op(output_grad, self.inputs[0], self.mode, self.align_corners,
                                    scale_factor=None if self.size is not None else self.scale_factor,
                                    ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        n, c, h, w = input_shapes[0]
        if self.size is not None:
            return (n, c) + tuple(self.size)
        return (n, c, int(h * self.scale_factor), int(w * self.scale_factor))


class InterpolateGradOp(Op):
    shape_only_inputs = (1,)

    def __init__(self, grad, ref, mode='bicubic', align_corners=False, scale_factor=None, ctx=None):
        super().__init__(InterpolateGradOp, [grad, ref], ctx)
        self.mode, self.align_corners, self.scale_factor = mode, align_corners, scale_factor

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        if _gpu(g) and self.mode == 'bicubic' and g.dtype in (torch.float32, torch.bfloat16):
            return KT.bicubic_grad(g, tuple(shape), self.align_corners, self.scale_factor)
        if _gpu(g):
            _record_fallback('interpolate_grad_' + str(self.mode))
        xs = _NA.zeros(tuple(shape), dtype=torch.float32, device=g.device, requires_grad=True)
        sf = self.scale_factor
        with torch.enable_grad():
            y = F.interpolate(xs, size=None if sf else tuple(g.shape[2:]), scale_factor=sf, mode=self.mode,
                              align_corners=self.align_corners)
            (gx,) = torch.autograd.grad(y, xs, g.float())
        return gx.to(g.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def interpolate_op(input, size=None, scale_factor=None, mode='bicubic', align_corners=False, ctx=None):
    return InterpolateOp(input, size, scale_factor, mode, align_corners, ctx=ctx)


def interpolate_grad_op(grad, input, mode='bicubic', align_corners=False, scale_factor=None, ctx=None):
    return InterpolateGradOp(grad, input, mode, align_corners, scale_factor, ctx=ctx)


class GatherOp(Op):
    def __init__(self, node, dim, index, ctx=None):
        super().__init__(GatherOp, [node, index], ctx)
        self.dim = dim

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, idx = input_vals
        if _gpu(x) and x.dtype in (torch.float32, torch.bfloat16):
            return KT.gather(x, self.dim, idx)
        return torch.gather(x, self.dim, idx.long())

    def gradient(self, output_grad):
        return [gather_gradient_op(self.inputs[0], output_grad, self.dim, self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


class GatherGradientOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, ref, grad, dim, index, ctx=None):
        super().__init__(GatherGradientOp, [ref, grad, index], ctx)
        self.dim = dim

    def compute(self, input_vals, output_val=None, stream_handle=None):
        shape, g, idx = input_vals
        if _gpu(g) and g.dtype in (torch.float32, torch.bfloat16):
            return KT.scatter_add(g, self.dim, idx, tuple(shape)).to(g.dtype)
        out = _NA.zeros(tuple(shape), dtype=torch.float32, device=g.device)
        out.scatter_add_(self.dim, idx.long(), g.float())
        return out.to(g.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def gather_op(node, dim, index, ctx=None):
    return GatherOp(node, dim, index, ctx=ctx)


def gather_gradient_op(input, grad, dim, index, ctx=None):
    return GatherGradientOp(input, grad, dim, index, ctx=ctx)


class IndexingOp(Op):
    """out[i, :] = input[index[i], :] (reference Indexing.cu:3-9)."""

    def __init__(self, inp, index, ctx=None):
        super().__init__(IndexingOp, [inp, index], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import sparse as KS
        return KS.gather_rows(input_vals[0].contiguous(), input_vals[1])

    def gradient(self, output_grad):
        return [indexing_grad_op(output_grad, self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class IndexingGradOp(Op):
    def __init__(self, grad, index, ctx=None):
        super().__init__(IndexingGradOp, [grad, index], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, idx = input_vals
        out = _NA.zeros_like(g)
        out[idx.long().reshape(-1)] = g
        return out

    def gradient(self, output_grad):
        # scatter by a permutation: its adjoint is the gather with the same index
        return [indexing_op(output_grad, self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def indexing_op(input_mat, index_mat, ctx=None):
    return IndexingOp(input_mat, index_mat, ctx=ctx)


def indexing_grad_op(output_grad, index, ctx=None):
    return IndexingGradOp(output_grad, index, ctx=ctx)


class ScatterOp(Op):
    """target[r][index[r][c]] = src[r][c] (reference Scatter.cu)."""

    def __init__(self, target, index, src, ctx=None):
        super().__init__(ScatterOp, [target, index, src], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        t, idx, src = input_vals
        return t.scatter(1, idx.long(), src.to(t.dtype))

    def gradient(self, output_grad):
        return [None, None, None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def scatter_op(node1, node2, node3, ctx=None):
    return ScatterOp(node1, node2, node3, ctx=ctx)


class Scatter1DOp(Op):
    """out[index[i]] = in[i]."""

    def __init__(self, inp, index, ctx=None):
        super().__init__(Scatter1DOp, [inp, index], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, idx = input_vals
        out = _NA.zeros_like(x)
        out[idx.long()] = x
        return out

    def gradient(self, output_grad):
        return [scatter1d_grad_op(output_grad, self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Scatter1DGradOp(Op):
    def __init__(self, grad, index, ctx=None):
        super().__init__(Scatter1DGradOp, [grad, index], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, idx = input_vals
        return g[idx.long()]

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def scatter1d_op(input_mat, index_mat, ctx=None):
    return Scatter1DOp(input_mat, index_mat, ctx=ctx)


def scatter1d_grad_op(output_grad_mat, index_mat, ctx=None):
    return Scatter1DGradOp(output_grad_mat, index_mat, ctx=ctx)


class Conv2d_BroadcastToOp(Op):
    """bias [C] -> NCHW shape of B."""
    shape_only_inputs = (1,)

    def __init__(self, a, b, ctx=None):
        super().__init__(Conv2d_BroadcastToOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        bias, shape = input_vals
        n, c, h, w = tuple(shape)
        return bias.reshape(1, c, 1, 1).expand(n, c, h, w)

    def gradient(self, output_grad):
        return [conv2d_reducesum_op(output_grad, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


class Conv2d_ReduceSumOp(Op):
    """NCHW -> [C] (bias gradient)."""

    def __init__(self, node, ctx=None):
        super().__init__(Conv2d_ReduceSumOp, [node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        n, c, h, w = x.shape
        if x.is_contiguous(memory_format=torch.channels_last):
            return KR.reduce_mid(x.permute(0, 2, 3, 1).reshape(1, n * h * w, c), out_dtype=torch.float32).reshape(c)
        return x.float().sum((0, 2, 3))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return (input_shapes[0][1],)


def conv2d_broadcastto_op(node_A, node_B, ctx=None):
    return Conv2d_BroadcastToOp(node_A, node_B, ctx=ctx)


def conv2d_reducesum_op(node, ctx=None):
    return Conv2d_ReduceSumOp(node, ctx=ctx)
