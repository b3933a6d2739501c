"""Softmax and loss operators (reference Softmax.py, SoftmaxCrossEntropy.py,
SoftmaxCrossEntropySparse.py, CrossEntropy.py, CrossEntropySparse.py,
BinaryCrossEntropy.py, NllLoss.py; SURVEY §2.4 "Softmax / losses").

Softmax and the fused softmax-cross-entropy run on the wave-per-row HIP
kernels; losses are produced in fp32 regardless of the logits dtype.
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

from .node import Op
from .nn import AuxResult
from ..kernels import softmax as KS


def softmax_func(y):
    """numpy softmax helper (reference Softmax.py:10)."""
    import numpy as np
    b = y - np.max(y, axis=-1, keepdims=True)
    e = np.exp(b)
    return e / np.sum(e, axis=-1, keepdims=True)


from ..kernels import native as _native
from ..kernels import tensor as KT


def _gpu(t):
    return isinstance(t, torch.Tensor) and _native(t) and t.dtype in (torch.float32, torch.bfloat16)


class SoftmaxOp(Op):
    def __init__(self, x, ctx=None):
        super().__init__(SoftmaxOp, [x], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return KS.softmax(input_vals[0])

    def gradient(self, output_grad):
        return [softmax_gradient_op(self, output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class SoftmaxGradientOp(Op):
    def __init__(self, y, g, ctx=None):
        super().__init__(SoftmaxGradientOp, [y, g], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, g = input_vals
        if g.dtype != y.dtype and g.is_cuda:
            from ..kernels.elementwise import cast
            g = cast(g.contiguous(), y.dtype)
        return KS.softmax_backward(y, g.to(y.dtype))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def softmax_op(node, ctx=None):
    return SoftmaxOp(node, ctx=ctx)


def softmax_gradient_op(node_y, grad, ctx=None):
    return SoftmaxGradientOp(node_y, grad, ctx=ctx)


class SoftmaxCrossEntropyOp(Op):
    """Per-row -sum(y_ * log softmax(x)); output shape x.shape[:-1]."""

    def __init__(self, x, y_, use_cudnn=True, ctx=None):
        super().__init__(SoftmaxCrossEntropyOp, [x, y_], ctx)
        self.use_cudnn = use_cudnn

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, lab = input_vals
        loss, lse = KS.softmax_ce(x, lab)
        return AuxResult(loss, lse)

    def gradient(self, output_grad):
        return [softmaxcrossentropy_gradient_op(self.inputs[0], self.inputs[1], output_grad, fwd=self, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][:-1])


class SoftmaxCrossEntropyGradientOp(Op):
    def __init__(self, x, y_, g, fwd=None, ctx=None):
        super().__init__(SoftmaxCrossEntropyGradientOp, [x, y_, g] + ([fwd] if fwd is not None else []), ctx)
        if fwd is not None:
            self.aux_inputs = (3,)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, lab, g = input_vals[:3]
        lse = input_vals[3] if len(input_vals) > 3 else None
        return KS.softmax_ce_backward(x, lab, g, lse)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def softmaxcrossentropy_op(node_A, node_B, use_cudnn=True, ctx=None):
    return SoftmaxCrossEntropyOp(node_A, node_B, use_cudnn, ctx=ctx)


def softmaxcrossentropy_gradient_op(node_A, node_B, node_C, use_cudnn=True, fwd=None, ctx=None):
    return SoftmaxCrossEntropyGradientOp(node_A, node_B, node_C, fwd=fwd, ctx=ctx)


def _label_feed(node):
    """class-index targets fed as fp32 stay fp32 under mixed precision: bf16 holds integers
    exactly only up to 256, so the feed cast would move vocabulary / token ids"""
    node.keep_fp32 = True


class SoftmaxCrossEntropySparseOp(Op):
    def __init__(self, x, y_, ignored_index=-1, ctx=None):
        super().__init__(SoftmaxCrossEntropySparseOp, [x, y_], ctx)
        _label_feed(y_)
        self.ignored_index = ignored_index

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, lab = input_vals
        loss, lse = KS.softmax_ce_sparse(x, lab, self.ignored_index)
        return AuxResult(loss, lse)

    def gradient(self, output_grad):
        return [SoftmaxCrossEntropySparseGradientOp(self.inputs[0], self.inputs[1], output_grad, self.ignored_index, fwd=self, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][:-1])


class SoftmaxCrossEntropySparseGradientOp(Op):
    def __init__(self, x, y_, g, ignored_index, fwd=None, ctx=None):
        super().__init__(SoftmaxCrossEntropySparseGradientOp, [x, y_, g] + ([fwd] if fwd is not None else []), ctx)
        self.ignored_index = ignored_index
        if fwd is not None:
            self.aux_inputs = (3,)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, lab, g = input_vals[:3]
        lse = input_vals[3] if len(input_vals) > 3 else None
        return KS.softmax_ce_sparse_backward(x, lab, g, lse, self.ignored_index)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def softmaxcrossentropy_sparse_op(node_A, node_B, ignored_index=-1, ctx=None):
    return SoftmaxCrossEntropySparseOp(node_A, node_B, ignored_index, ctx=ctx)


def softmaxcrossentropy_sparse_gradient_op(node_A, node_B, node_C, ignored_index=-1, ctx=None):
    return SoftmaxCrossEntropySparseGradientOp(node_A, node_B, node_C, ignored_index, ctx=ctx)


class CrossEntropyOp(Op):
    """-sum(y_ * log(y)) over the last axis (y already a distribution)."""

    def __init__(self, y, y_, ctx=None):
        super().__init__(CrossEntropyOp, [y, y_], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, lab = input_vals
        if _gpu(y):
            return KT.ce_dense(y, lab)
        return -(lab.float() * torch.log(y.float())).sum(-1)

    def gradient(self, output_grad):
        return [crossentropy_gradient_op(output_grad, self.inputs[0], self.inputs[1], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][:-1])


class CrossEntropyGradientOp(Op):
    def __init__(self, g, y, y_, ctx=None):
        super().__init__(CrossEntropyGradientOp, [g, y, y_], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, y, lab = input_vals
        if _gpu(y):
            return KT.ce_dense_grad(g, y, lab)
        gg = g.float().unsqueeze(-1) if g.numel() > 1 else g.float()
        return (-gg * lab.float() / y.float()).to(y.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def crossentropy_op(node_y, node_y_, ctx=None):
    return CrossEntropyOp(node_y, node_y_, ctx=ctx)


def crossentropy_gradient_op(node_grad, node_y, node_y_, ctx=None):
    return CrossEntropyGradientOp(node_grad, node_y, node_y_, ctx=ctx)


class CrossEntropySparseOp(Op):
    def __init__(self, y, y_, ignored_index=-1, ctx=None):
        super().__init__(CrossEntropySparseOp, [y, y_], ctx)
        _label_feed(y_)
        self.ignored_index = ignored_index

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, lab = input_vals
        if _gpu(y):
            return KT.ce_sparse(y, lab, self.ignored_index)
        lab = lab.long().reshape(y.shape[:-1])
        valid = lab != self.ignored_index
        safe = torch.where(valid, lab, _NA.zeros_like(lab))
        p = torch.gather(y.float(), -1, safe.unsqueeze(-1)).squeeze(-1)
        return torch.where(valid, -torch.log(p), _NA.zeros_like(p))

    def gradient(self, output_grad):
        return [crossentropy_sparse_gradient_op(output_grad, self.inputs[0], self.inputs[1], self.ignored_index, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][:-1])


class CrossEntropySparseGradientOp(Op):
    def __init__(self, g, y, y_, ignored_index, ctx=None):
        super().__init__(CrossEntropySparseGradientOp, [g, y, y_], ctx)
        self.ignored_index = ignored_index

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, y, lab = input_vals
        if _gpu(y):
            return KT.ce_sparse_grad(g, y, lab, self.ignored_index)
        lab = lab.long().reshape(y.shape[:-1])
        valid = lab != self.ignored_index
        safe = torch.where(valid, lab, _NA.zeros_like(lab))
        out = _NA.zeros(y.shape, dtype=torch.float32, device=y.device)
        p = torch.gather(y.float(), -1, safe.unsqueeze(-1)).squeeze(-1)
        gg = g.float() if g.numel() > 1 else g.float().expand(p.shape)
        val = torch.where(valid, -gg / p, _NA.zeros_like(p))
        out.scatter_(-1, safe.unsqueeze(-1), val.unsqueeze(-1))
        return out.to(y.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def crossentropy_sparse_op(node_y, node_y_, ignored_index=-1, ctx=None):
    return CrossEntropySparseOp(node_y, node_y_, ignored_index, ctx=ctx)


def crossentropy_sparse_gradient_op(node_grad, node_y, node_y_, ignored_index=-1, ctx=None):
    return CrossEntropySparseGradientOp(node_grad, node_y, node_y_, ignored_index, ctx=ctx)


class BinaryCrossEntropyOp(Op):
    """-y_ log(y) - (1-y_) log(1-y), elementwise (reference BinaryCrossEntropy.py)."""

    def __init__(self, pred, label, ctx=None):
        super().__init__(BinaryCrossEntropyOp, [pred, label], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, lab = input_vals
        if _gpu(y) and lab.shape == y.shape:
            return KT.bce(y, lab)
        yf = y.float().clamp(1e-12, 1 - 1e-7)
        lf = lab.float()
        return -lf * torch.log(yf) - (1 - lf) * torch.log(1 - yf)

    def gradient(self, output_grad):
        return [binarycrossentropy_gradient_op(self.inputs[0], self.inputs[1], output_grad, ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class BinaryCrossEntropyGradientOp(Op):
    def __init__(self, pred, label, g, ctx=None):
        super().__init__(BinaryCrossEntropyGradientOp, [pred, label, g], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, lab, g = input_vals
        if _gpu(y) and lab.shape == y.shape:
            return KT.bce_grad(y, lab, g)
        yf = y.float().clamp(1e-12, 1 - 1e-7)
        lf = lab.float()
        return (g.float() * (-lf / yf + (1 - lf) / (1 - yf))).to(y.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def binarycrossentropy_op(node_A, node_B, ctx=None):
    return BinaryCrossEntropyOp(node_A, node_B, ctx=ctx)


def binarycrossentropy_gradient_op(node_A, node_B, node_C, ctx=None):
    return BinaryCrossEntropyGradientOp(node_A, node_B, node_C, ctx=ctx)


class NllLossOp(Op):
    """mean over rows of -input[r, target[r]] (reference NllLoss.cu)."""

    def __init__(self, inp, target, cols, ctx=None):
        super().__init__(NllLossOp, [inp, target], ctx)
        _label_feed(target)
        self.cols = cols

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, t = input_vals
        if _gpu(x):
            return KT.nll(x, t, self.cols)
        picked = torch.gather(x.float().reshape(-1, self.cols), 1, t.long().reshape(-1, 1))
        return -picked.mean().reshape(1)

    def gradient(self, output_grad):
        return [nll_loss_grad_op(output_grad, self.inputs[1], self.cols, ref=self.inputs[0], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        return (1,)


class NllLossGradOp(Op):
    def __init__(self, g, target, cols, ref=None, ctx=None):
        super().__init__(NllLossGradOp, [g, target], ctx)
        self.cols = cols

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, t = input_vals
        if _gpu(g):
            return KT.nll_grad(g, t, self.cols)
        t = t.long().reshape(-1)
        out = _NA.zeros((t.numel(), self.cols), dtype=torch.float32, device=t.device)
        out.scatter_(1, t.reshape(-1, 1), -(g.float().reshape(1, 1).expand(t.numel(), 1)) / t.numel())
        return out

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def nll_loss_op(input, target, cols, ctx=None):
    return NllLossOp(input, target, cols, ctx=ctx)


def nll_loss_grad_op(output_grad, target, cols, ref=None, ctx=None):
    return NllLossGradOp(output_grad, target, cols, ref, ctx=ctx)
