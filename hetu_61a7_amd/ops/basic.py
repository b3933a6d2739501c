"""Elementwise, constant and fill operators.

Parity: reference gpu_ops Abs.py, Opposite.py, Exp.py, LogElewise.py, Floor.py,
Sqrt.py, Sin.py, Tanh.py, Sigmoid.py, Relu.py, LeakyRelu.py, Gelu.py, Pow.py,
ConstPow.py, Clamp.py, Bool.py, MaskedFill.py, OneHot.py, Where.py,
AddElewise.py, AddConst.py, MinusElewise.py, MinusByConst.py,
MultiplyElewise.py, MultiplyConst.py, Division.py, MatrixDot.py, Max.py,
Min.py, OnesLike.py, ZerosLike.py, Full.py, Rand.py, Arange.py (SURVEY §2.4
rows "Unary elementwise", "Binary / const", "Fill / init / iota").

GPU execution goes through the vectorised HIP elementwise family
(``kernels.elementwise``); broadcasting follows numpy rules and gradients are
reduced back with ``reduce_to_shape_op``.
"""
from __future__ import annotations

import numpy as np
import torch
from .. import native_array as _NA

from .node import Op
from ..kernels import elementwise as K
from ..kernels import reduce as KR


def _shape_bcast(a, b):
    return tuple(np.broadcast_shapes(tuple(a), tuple(b)))


def _dt(a, b):
    """Result dtype: the dtype of the larger operand (keeps bf16 activations
    bf16 when a fp32 bias/scale is broadcast against them)."""
    if not b.dtype.is_floating_point:
        return a.dtype
    if not a.dtype.is_floating_point:
        return b.dtype
    return a.dtype if a.numel() >= b.numel() else b.dtype


class ReduceToShapeOp(Op):
    """Sum a (broadcast) gradient down to the shape of ``ref`` (shape-only input)."""
    shape_only_inputs = (1,)

    def __init__(self, grad, ref, ctx=None):
        super().__init__(ReduceToShapeOp, [grad, ref], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        return KR.sum_to_shape(g, shape)

    def gradient(self, output_grad):
        from .shape import broadcastto_op
        return [broadcastto_op(output_grad, self.inputs[0]), None]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def reduce_to_shape_op(grad, ref, ctx=None):
    return ReduceToShapeOp(grad, ref, ctx=ctx)


# ---------------------------------------------------------------------------
# unary ops
class UnaryOp(Op):
    kop = None

    def __init__(self, node, ctx=None, c=0.0, c2=0.0):
        super().__init__(type(self), [node], ctx)
        self.c, self.c2 = c, c2

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.unary(self.kop, input_vals[0], self.c, self.c2)

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class AbsOp(UnaryOp):
    kop = 'abs'

    def gradient(self, output_grad):
        return [abs_gradient_op(self.inputs[0], output_grad, ctx=self.raw_ctx)]


class AbsGradientOp(Op):
    def __init__(self, node, grad, ctx=None):
        super().__init__(AbsGradientOp, [node, grad], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('abs_grad', input_vals[0], input_vals[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def abs_op(node, ctx=None):
    return AbsOp(node, ctx=ctx)


def abs_gradient_op(node, grad, ctx=None):
    return AbsGradientOp(node, grad, ctx=ctx)


class OppositeOp(UnaryOp):
    kop = 'neg'

    def gradient(self, output_grad):
        return [opposite_op(output_grad, ctx=self.raw_ctx)]


def opposite_op(node, ctx=None):
    return OppositeOp(node, ctx=ctx)


class ExpOp(UnaryOp):
    kop = 'exp'

    def gradient(self, output_grad):
        return [mul_op(output_grad, self, ctx=self.raw_ctx)]


def exp_op(node, ctx=None):
    return ExpOp(node, ctx=ctx)


class LogOp(UnaryOp):
    kop = 'log'

    def gradient(self, output_grad):
        return [log_grad_op(output_grad, self.inputs[0], ctx=self.raw_ctx)]


class LogGradOp(Op):
    def __init__(self, grad, node, ctx=None):
        super().__init__(LogGradOp, [grad, node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('log_grad', input_vals[1], input_vals[0])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def log_op(node, ctx=None):
    return LogOp(node, ctx=ctx)


def log_grad_op(grad, node, ctx=None):
    return LogGradOp(grad, node, ctx=ctx)


class FloorOp(UnaryOp):
    kop = 'floor'

    def gradient(self, output_grad):
        return [zeroslike_op(self.inputs[0], ctx=self.raw_ctx)]


def floor_op(node, ctx=None):
    return FloorOp(node, ctx=ctx)


class SqrtOp(UnaryOp):
    kop = 'sqrt'

    def gradient(self, output_grad):
        return [SqrtGradOp(self, output_grad, ctx=self.raw_ctx)]


class SqrtGradOp(Op):
    def __init__(self, y, g, ctx=None):
        super().__init__(SqrtGradOp, [y, g], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('sqrt_grad', input_vals[0], input_vals[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class ReciprocalSqrtOp(UnaryOp):
    kop = 'rsqrt'

    def gradient(self, output_grad):
        # d/dx x^-1/2 = -0.5 x^-3/2 = -0.5 * y^3
        y3 = const_pow_like(self, 3.0)
        return [mul_byconst_op(mul_op(output_grad, y3, ctx=self.raw_ctx), -0.5, ctx=self.raw_ctx)]


def sqrt_op(node, ctx=None):
    return SqrtOp(node, ctx=ctx)


def rsqrt_op(node, ctx=None):
    return ReciprocalSqrtOp(node, ctx=ctx)


class SinOp(UnaryOp):
    kop = 'sin'

    def gradient(self, output_grad):
        return [mul_op(output_grad, cos_op(self.inputs[0], ctx=self.raw_ctx), ctx=self.raw_ctx)]


class CosOp(UnaryOp):
    kop = 'cos'

    def gradient(self, output_grad):
        return [opposite_op(mul_op(output_grad, sin_op(self.inputs[0], ctx=self.raw_ctx),
                                   ctx=self.raw_ctx), ctx=self.raw_ctx)]


def sin_op(node, ctx=None):
    return SinOp(node, ctx=ctx)


def cos_op(node, ctx=None):
    return CosOp(node, ctx=ctx)


class TanhOp(UnaryOp):
    kop = 'tanh'

    def gradient(self, output_grad):
        return [tanh_gradient_op(self, output_grad, ctx=self.raw_ctx)]


class TanhGradientOp(Op):
    def __init__(self, y, g, ctx=None):
        super().__init__(TanhGradientOp, [y, g], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('tanh_grad', input_vals[0], input_vals[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def tanh_op(node, ctx=None):
    return TanhOp(node, ctx=ctx)


def tanh_gradient_op(node, grad, ctx=None):
    return TanhGradientOp(node, grad, ctx=ctx)


class SigmoidOp(UnaryOp):
    kop = 'sigmoid'

    def gradient(self, output_grad):
        return [SigmoidGradientOp(self, output_grad, ctx=self.raw_ctx)]


class SigmoidGradientOp(Op):
    def __init__(self, y, g, ctx=None):
        super().__init__(SigmoidGradientOp, [y, g], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('sigmoid_grad', input_vals[0], input_vals[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def sigmoid_op(node, ctx=None):
    return SigmoidOp(node, ctx=ctx)


class ReluOp(UnaryOp):
    kop = 'relu'

    def gradient(self, output_grad):
        # mask from the OUTPUT (y > 0 <=> x > 0): keeps x dead after the forward
        return [relu_gradient_op(self, output_grad, ctx=self.raw_ctx)]


class ReluGradientOp(Op):
    def __init__(self, node, grad, ctx=None):
        super().__init__(ReluGradientOp, [node, grad], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, g = input_vals
        if g.dim() == 4 and x.dim() == 4:
            cl = torch.channels_last
            if x.is_contiguous(memory_format=cl) and not x.is_contiguous():
                g = g.contiguous(memory_format=cl)
                return K.binary('relu_grad', x.permute(0, 2, 3, 1), g.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return K.binary('relu_grad', x.contiguous(), g.contiguous())

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def relu_op(node, ctx=None):
    return ReluOp(node, ctx=ctx)


def relu_gradient_op(node, grad, ctx=None):
    return ReluGradientOp(node, grad, ctx=ctx)


class LeakyReluOp(UnaryOp):
    kop = 'leaky_relu'

    def gradient(self, output_grad):
        return [leaky_relu_gradient_op(self.inputs[0], output_grad, self.c, ctx=self.raw_ctx)]


class LeakyReluGradientOp(Op):
    def __init__(self, node, grad, alpha, ctx=None):
        super().__init__(LeakyReluGradientOp, [node, grad], ctx)
        self.alpha = alpha

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('leaky_relu_grad', input_vals[0].contiguous(), input_vals[1].contiguous(), self.alpha)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def leaky_relu_op(node, alpha, ctx=None):
    return LeakyReluOp(node, ctx=ctx, c=alpha)


def leaky_relu_gradient_op(node_A, node_B, alpha, ctx=None):
    return LeakyReluGradientOp(node_A, node_B, alpha, ctx=ctx)


class GeluOp(UnaryOp):
    kop = 'gelu'

    def gradient(self, output_grad):
        return [gelu_gradient_op(self.inputs[0], output_grad, ctx=self.raw_ctx)]


class GeluGradientOp(Op):
    def __init__(self, node, grad, ctx=None):
        super().__init__(GeluGradientOp, [node, grad], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('gelu_grad', input_vals[0].contiguous(), input_vals[1].contiguous())

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def gelu_op(node, ctx=None):
    return GeluOp(node, ctx=ctx)


def gelu_gradient_op(node_A, node_B, ctx=None):
    return GeluGradientOp(node_A, node_B, ctx=ctx)


class PowOp(UnaryOp):
    """x ** eps (reference Pow.py)."""
    kop = 'pow_c'

    def gradient(self, output_grad):
        return [pow_gradient_op(self.inputs[0], output_grad, self.c, ctx=self.raw_ctx)]


class PowGradientOp(Op):
    def __init__(self, node, grad, eps, ctx=None):
        super().__init__(PowGradientOp, [node, grad], ctx)
        self.eps = eps

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, g = input_vals
        return K.binary('mul', K.unary('pow_c', x, self.eps - 1.0), g) * self.eps

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def pow_op(node, eps, ctx=None):
    return PowOp(node, ctx=ctx, c=eps)


def pow_gradient_op(node_A, node_B, eps, ctx=None):
    return PowGradientOp(node_A, node_B, eps, ctx=ctx)


def const_pow_like(node, p):
    return PowOp(node, c=p)


class ConstPowOp(UnaryOp):
    """val ** x (reference ConstPow.cu:3-8)."""
    kop = 'cpow'

    def gradient(self, output_grad):
        return [const_pow_gradient_op(self, output_grad, self.c, ctx=self.raw_ctx)]


class ConstPowGradientOp(Op):
    def __init__(self, y, grad, val, ctx=None):
        super().__init__(ConstPowGradientOp, [y, grad], ctx)
        self.val = val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('mul', input_vals[0], input_vals[1]) * float(np.log(self.val))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def const_pow_op(node, val, ctx=None):
    return ConstPowOp(node, ctx=ctx, c=val)


def const_pow_gradient_op(input_node, grad_node, val, ctx=None):
    return ConstPowGradientOp(input_node, grad_node, val, ctx=ctx)


class ClampOp(Op):
    def __init__(self, node, min_mat=None, max_mat=None, mmin=None, mmax=None, ctx=None):
        inputs = [node] + [n for n in (min_mat, max_mat) if n is not None]
        super().__init__(ClampOp, inputs, ctx)
        self.has_min_mat, self.has_max_mat = min_mat is not None, max_mat is not None
        self.mmin, self.mmax = mmin, mmax

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        i = 1
        lo = hi = None
        if self.has_min_mat:
            lo = input_vals[i]
            i += 1
        if self.has_max_mat:
            hi = input_vals[i]
        if lo is None and hi is None:
            return K.unary('clamp', x.contiguous(), -np.inf if self.mmin is None else self.mmin,
                           np.inf if self.mmax is None else self.mmax)
        r = x
        if lo is not None:
            r = torch.maximum(r, lo.to(r.dtype))
        elif self.mmin is not None:
            r = torch.clamp(r, min=self.mmin)
        if hi is not None:
            r = torch.minimum(r, hi.to(r.dtype))
        elif self.mmax is not None:
            r = torch.clamp(r, max=self.mmax)
        return r

    def gradient(self, output_grad):
        mask = ClampMaskOp(self.inputs[0], self.mmin, self.mmax, ctx=self.raw_ctx)
        return [mul_op(output_grad, mask, ctx=self.raw_ctx)] + [None] * (len(self.inputs) - 1)

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class ClampMaskOp(Op):
    def __init__(self, node, mmin, mmax, ctx=None):
        super().__init__(ClampMaskOp, [node], ctx)
        self.mmin, self.mmax = mmin, mmax

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        m = torch.ones_like(x, dtype=torch.bool)
        if self.mmin is not None:
            m &= x >= self.mmin
        if self.mmax is not None:
            m &= x <= self.mmax
        return m.to(x.dtype)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def clamp_op(node_A, min_mat=None, max_mat=None, min=None, max=None, ctx=None):
    return ClampOp(node_A, min_mat, max_mat, min, max, ctx=ctx)


_CMP = {0: torch.eq, 1: torch.lt, 2: torch.gt, 3: torch.le, 4: torch.ge}


class BoolOp(Op):
    """Comparisons producing float {0,1} (reference Bool.py cond codes
    0 ==, 1 <, 2 >, 3 <=, 4 >=)."""

    def __init__(self, node, other=None, val=None, cond=0, ctx=None):
        super().__init__(BoolOp, [node] + ([other] if other is not None else []), ctx)
        self.val, self.cond, self.has_other = val, cond, other is not None

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if self.has_other:
            r = _CMP[self.cond](x, input_vals[1])
        elif self.val is not None:
            r = _CMP[self.cond](x, self.val)
        else:
            r = x != 0
        dt = x.dtype if x.dtype.is_floating_point else torch.float32
        return r.to(dt)

    def gradient(self, output_grad):
        return [None] * len(self.inputs)

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def bool_op(node, input=None, val=None, cond=0, ctx=None):
    return BoolOp(node, input, val, cond, ctx=ctx)


class MaskedFillOp(Op):
    def __init__(self, node, mask, val, ctx=None):
        super().__init__(MaskedFillOp, [node, mask], ctx)
        self.val = val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, m = input_vals
        return x.masked_fill(m.bool() if m.dtype != torch.bool else m, self.val)

    def gradient(self, output_grad):
        return [MaskedFillOp(output_grad, self.inputs[1], 0.0, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def masked_fill_op(input, mask, val, ctx=None):
    return MaskedFillOp(input, mask, val, ctx=ctx)


class OneHotOp(Op):
    def __init__(self, node, num_classes, ctx=None):
        super().__init__(OneHotOp, [node], ctx)
        self.num_classes = num_classes

    def compute(self, input_vals, output_val=None, stream_handle=None):
        idx = input_vals[0]
        if idx.is_cuda and idx.dtype in (torch.int64, torch.int32, torch.float32):
            from ..kernels import tensor as KT
            return KT.one_hot(idx, self.num_classes)
        return torch.nn.functional.one_hot(idx.long(), self.num_classes).float()

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0]) + (self.num_classes,)


def one_hot_op(node, num_classes, ctx=None):
    return OneHotOp(node, num_classes, ctx=ctx)


class WhereOp(Op):
    def __init__(self, cond, a, b, ctx=None):
        super().__init__(WhereOp, [cond, a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        c, a, b = input_vals
        return torch.where(c.bool(), a, b.to(a.dtype))

    def gradient(self, output_grad):
        z = zeroslike_op(output_grad, ctx=self.raw_ctx)
        return [None,
                reduce_to_shape_op(where_op(self.inputs[0], output_grad, z, ctx=self.raw_ctx), self.inputs[1]),
                reduce_to_shape_op(where_op(self.inputs[0], z, output_grad, ctx=self.raw_ctx), self.inputs[2])]

    def infer_shape(self, input_shapes):
        return _shape_bcast(_shape_bcast(input_shapes[0], input_shapes[1]), input_shapes[2])


class WhereConstOp(Op):
    def __init__(self, cond, a, const_attr, ctx=None):
        super().__init__(WhereConstOp, [cond, a], ctx)
        self.const_attr = const_attr

    def compute(self, input_vals, output_val=None, stream_handle=None):
        c, a = input_vals
        return torch.where(c.bool(), a, torch.full_like(a, self.const_attr))

    def gradient(self, output_grad):
        return [None, WhereConstOp(self.inputs[0], output_grad, 0.0, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def where_op(cond, node_A, node_B, ctx=None):
    return WhereOp(cond, node_A, node_B, ctx=ctx)


def where_const_op(cond, node_A, const_attr, ctx=None):
    return WhereConstOp(cond, node_A, const_attr, ctx=ctx)


# ---------------------------------------------------------------------------
# binary ops
class AddOp(Op):
    def __init__(self, a, b, ctx=None):
        super().__init__(AddOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        if a.numel() < b.numel():
            a, b = b, a
        if a.dim() == 4 and b.dim() == 4 and a.shape == b.shape and not a.is_contiguous():
            cl = torch.channels_last
            if a.is_contiguous(memory_format=cl):
                b = b.contiguous(memory_format=cl)
                return K.binary('add', a.permute(0, 2, 3, 1), b.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        if a.shape == b.shape or b.numel() == 1 or (a.dim() >= b.dim() and tuple(a.shape[a.dim()-b.dim():]) == tuple(b.shape)):
            return K.binary('add', a.contiguous(), b.contiguous())
        return (a + b).to(_dt(a, b))

    def gradient(self, output_grad):
        return [reduce_to_shape_op(output_grad, self.inputs[0], ctx=self.raw_ctx),
                reduce_to_shape_op(output_grad, self.inputs[1], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return _shape_bcast(input_shapes[0], input_shapes[1])


def add_op(node_A, node_B, ctx=None):
    return AddOp(node_A, node_B, ctx=ctx)


class AddByConstOp(Op):
    def __init__(self, node, const_val, ctx=None):
        super().__init__(AddByConstOp, [node], ctx)
        self.const_attr = const_val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.unary('add_c', input_vals[0].contiguous(), self.const_attr)

    def gradient(self, output_grad):
        return [output_grad]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def addbyconst_op(node, const_val, ctx=None):
    return AddByConstOp(node, const_val, ctx=ctx)


class MinusOp(Op):
    def __init__(self, a, b, ctx=None):
        super().__init__(MinusOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        if a.shape == b.shape or b.numel() == 1:
            return K.binary('sub', a.contiguous(), b.contiguous())
        return (a - b).to(_dt(a, b))

    def gradient(self, output_grad):
        return [reduce_to_shape_op(output_grad, self.inputs[0], ctx=self.raw_ctx),
                reduce_to_shape_op(opposite_op(output_grad, ctx=self.raw_ctx), self.inputs[1], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return _shape_bcast(input_shapes[0], input_shapes[1])


def minus_op(node_A, node_B, ctx=None):
    return MinusOp(node_A, node_B, ctx=ctx)


class MinusByConstOp(Op):
    """const - x (reference MinusByConst.cu)."""

    def __init__(self, node, const_val, ctx=None):
        super().__init__(MinusByConstOp, [node], ctx)
        self.const_attr = const_val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.unary('rsub_c', input_vals[0].contiguous(), self.const_attr)

    def gradient(self, output_grad):
        return [opposite_op(output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def minus_byconst_op(node, const_val, ctx=None):
    return MinusByConstOp(node, const_val, ctx=ctx)


class MulOp(Op):
    def __init__(self, a, b, ctx=None):
        super().__init__(MulOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        if a.numel() < b.numel():
            a, b = b, a
        if a.shape == b.shape or b.numel() == 1 or (a.dim() >= b.dim() and tuple(a.shape[a.dim()-b.dim():]) == tuple(b.shape)):
            return K.binary('mul', a.contiguous(), b.contiguous())
        return (a * b).to(_dt(a, b))

    def gradient(self, output_grad):
        return [reduce_to_shape_op(mul_op(output_grad, self.inputs[1], ctx=self.raw_ctx), self.inputs[0], ctx=self.raw_ctx),
                reduce_to_shape_op(mul_op(output_grad, self.inputs[0], ctx=self.raw_ctx), self.inputs[1], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return _shape_bcast(input_shapes[0], input_shapes[1])


def mul_op(node_A, node_B, ctx=None):
    return MulOp(node_A, node_B, ctx=ctx)


class MulByConstOp(Op):
    def __init__(self, node, const_val, ctx=None):
        super().__init__(MulByConstOp, [node], ctx)
        self.const_attr = const_val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.unary('mul_c', input_vals[0].contiguous(), self.const_attr)

    def gradient(self, output_grad):
        return [mul_byconst_op(output_grad, self.const_attr, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def mul_byconst_op(node, const_val, ctx=None):
    return MulByConstOp(node, const_val, ctx=ctx)


class DivOp(Op):
    def __init__(self, a, b, ctx=None):
        super().__init__(DivOp, [a, b], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        if a.shape == b.shape or b.numel() == 1:
            return K.binary('div', a.contiguous(), b.contiguous())
        return (a / b).to(_dt(a, b))

    def gradient(self, output_grad):
        ga = div_op(output_grad, self.inputs[1], ctx=self.raw_ctx)
        gb = opposite_op(div_op(mul_op(output_grad, self, ctx=self.raw_ctx), self.inputs[1], ctx=self.raw_ctx), ctx=self.raw_ctx)
        return [reduce_to_shape_op(ga, self.inputs[0], ctx=self.raw_ctx),
                reduce_to_shape_op(gb, self.inputs[1], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return _shape_bcast(input_shapes[0], input_shapes[1])


class DivConstOp(Op):
    """const / x (reference DivideConst.cu:3-8)."""

    def __init__(self, const_val, node, ctx=None):
        super().__init__(DivConstOp, [node], ctx)
        self.const_attr = const_val

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.unary('rdiv_c', input_vals[0].contiguous(), self.const_attr)

    def gradient(self, output_grad):
        # d(c/x) = -c/x^2 = -y/x
        return [opposite_op(div_op(mul_op(output_grad, self, ctx=self.raw_ctx), self.inputs[0], ctx=self.raw_ctx), ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def div_op(node_A, node_B, ctx=None):
    return DivOp(node_A, node_B, ctx=ctx)


def div_const_op(const_val, node_A, ctx=None):
    return DivConstOp(const_val, node_A, ctx=ctx)


class MatrixDotOp(Op):
    """Row-broadcast multiply a[i, j] * b[j] (reference Dot.cu:3-8)."""

    def __init__(self, a, b, axes=0, ctx=None):
        super().__init__(MatrixDotOp, [a, b], ctx)
        self.axes = axes

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return K.binary('mul', input_vals[0].contiguous(), input_vals[1].contiguous())

    def gradient(self, output_grad):
        return [matrix_dot_op(output_grad, self.inputs[1], ctx=self.raw_ctx),
                reduce_to_shape_op(mul_op(output_grad, self.inputs[0], ctx=self.raw_ctx), self.inputs[1], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def matrix_dot_op(node_A, node_B, axes=0, ctx=None):
    return MatrixDotOp(node_A, node_B, axes, ctx=ctx)


class MaxMinOp(Op):
    """max/min: elementwise with two inputs, reduction over ``dim`` with one."""

    def __init__(self, is_max, a, b=None, dim=0, keepdim=False, ctx=None):
        super().__init__('MaxOp' if is_max else 'MinOp', [a] + ([b] if b is not None else []), ctx)
        self.is_max, self.dim, self.keepdim = is_max, dim, keepdim

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if len(input_vals) == 2:
            return K.binary('max' if self.is_max else 'min', input_vals[0].contiguous(), input_vals[1].contiguous())
        x = input_vals[0]
        r = torch.amax(x, self.dim, self.keepdim) if self.is_max else torch.amin(x, self.dim, self.keepdim)
        return r

    def gradient(self, output_grad):
        if len(self.inputs) == 2:
            m = BoolOp(self.inputs[0], self.inputs[1], cond=4 if self.is_max else 3, ctx=self.raw_ctx)
            return [mul_op(output_grad, m, ctx=self.raw_ctx),
                    mul_op(output_grad, minus_byconst_op(m, 1.0, ctx=self.raw_ctx), ctx=self.raw_ctx)]
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        if len(self.inputs) == 2:
            return input_shapes[0]
        s = list(input_shapes[0])
        if self.keepdim:
            s[self.dim] = 1
        else:
            s.pop(self.dim)
        return tuple(s)


def max_op(node_A, node_B=None, dim=0, keepdim=False, ctx=None):
    return MaxMinOp(True, node_A, node_B, dim, keepdim, ctx=ctx)


def min_op(node_A, node_B=None, dim=0, keepdim=False, ctx=None):
    return MaxMinOp(False, node_A, node_B, dim, keepdim, ctx=ctx)


# ---------------------------------------------------------------------------
# fills
class OnesLikeOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, node, ctx=None):
        super().__init__(OnesLikeOp, [node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.tensor import fill_
        return fill_(_NA.empty(tuple(input_vals[0]), dtype=torch.float32, device=self.device), 1.0)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class ZerosLikeOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, node, ctx=None):
        super().__init__(ZerosLikeOp, [node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if self.device.type == 'cuda':
            from ..kernels.tensor import zeros
            return zeros(tuple(input_vals[0]), torch.float32, self.device)
        return _NA.zeros(tuple(input_vals[0]), dtype=torch.float32, device=self.device)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def oneslike_op(node, ctx=None):
    return OnesLikeOp(node, ctx=ctx)


def zeroslike_op(node, ctx=None):
    return ZerosLikeOp(node, ctx=ctx)


class FullOp(Op):
    def __init__(self, size, fill_value, ctx=None):
        super().__init__(FullOp, [], ctx)
        self.size, self.fill_value = tuple(size), fill_value

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return _full(self.size, self.fill_value, self.device)

    def gradient(self, output_grad):
        return []

    def infer_shape(self, input_shapes):
        return self.size


class FullLikeOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, node, fill_value, ctx=None):
        super().__init__(FullLikeOp, [node], ctx)
        self.fill_value = fill_value

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return _full(tuple(input_vals[0]), self.fill_value, self.device)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def _full(size, value, device):
    """fp32 constant tensor: the native fill kernel on the GPU (reference ArraySet.cu)"""
    if device.type == 'cuda':
        from .. import native_array as _NA
        from ..kernels.tensor import fill_
        return fill_(_NA.empty(tuple(size), dtype=torch.float32, device=device), float(value))
    return torch.full(tuple(size), value, dtype=torch.float32, device=device)


def full_op(size, fill_value, ctx=None):
    return FullOp(size, fill_value, ctx=ctx)


def full_like_op(node, fill_value, ctx=None):
    return FullLikeOp(node, fill_value, ctx=ctx)


class RandOp(Op):
    def __init__(self, size, ctx=None):
        super().__init__(RandOp, [], ctx)
        self.size = tuple(size)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import rng
        dev = self.device
        seed = rng.next_seed(self.id, on_gpu=dev.type == 'cuda')
        if dev.type == 'cuda':
            # Philox uniform kernel (random.hip; reference Initializers.cu uniform fill)
            from .. import native_array as _NA
            return rng.uniform_(_NA.empty(self.size, dtype=torch.float32, device=dev), 0.0, 1.0, seed=seed)
        g = torch.Generator()
        g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
        return torch.rand(self.size, generator=g)

    def gradient(self, output_grad):
        return []

    def infer_shape(self, input_shapes):
        return self.size


def rand_op(size, ctx=None):
    return RandOp(size, ctx=ctx)


class ArangeOp(Op):
    def __init__(self, start, end, step=1.0, ctx=None):
        super().__init__(ArangeOp, [], ctx)
        self.start, self.end, self.step = start, end, step

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if self.device.type == 'cuda':
            from ..kernels import rng
            return rng.arange(self.infer_shape(None)[0], self.start, self.step, device=self.device)
        return torch.arange(self.start, self.end, self.step, dtype=torch.float32, device=self.device)

    def gradient(self, output_grad):
        return []

    def infer_shape(self, input_shapes):
        return (int(np.ceil((self.end - self.start) / self.step)),)


def arange_op(start, end, step=1.0, ctx=None):
    return ArangeOp(start, end, step, ctx=ctx)


# Op.device: torch device of the op's resolved context (set by forward_hook)
def _device(self):
    from .. import ndarray
    c = self.ctx
    if isinstance(c, ndarray.DLContext):
        return c.torch_device
    return torch.device('cpu')


Op.device = property(_device)
