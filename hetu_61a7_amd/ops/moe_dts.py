"""Ops for the Dense-To-Sparse MoE gate: annealed Gumbel-softmax and the
gate-weight threshold mask."""
from __future__ import annotations

import torch

from .node import Op
from .nn import AuxResult


class GumbelSoftmaxOp(Op):
    """softmax((logits + g) / tau), g ~ Gumbel(0,1); tau from an annealing
    schedule object read at every step (``temperature.value``)."""

    def __init__(self, logits, temperature, ctx=None):
        super().__init__(GumbelSoftmaxOp, [logits], ctx)
        self.temperature = temperature
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0].float()
        tau = float(self.temperature.value)
        if not self.inference:
            from .nn import _next_seed
            g = torch.Generator(device=x.device)
            g.manual_seed(_next_seed() & 0x7FFFFFFFFFFF)
            u = torch.rand(x.shape, generator=g, device=x.device).clamp_(1e-9, 1 - 1e-9)
            x = x - torch.log(-torch.log(u))
        y = torch.softmax(x / tau, -1)
        return AuxResult(y, tau)

    def gradient(self, output_grad):
        return [GumbelSoftmaxGradOp(self, output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class GumbelSoftmaxGradOp(Op):
    value_and_aux_inputs = (0,)

    def __init__(self, fwd, grad, ctx=None):
        super().__init__(GumbelSoftmaxGradOp, [fwd, grad], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        (y, tau), g = input_vals
        g = g.float()
        return y * (g - (g * y).sum(-1, keepdim=True)) / tau

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def gumbel_softmax_op(logits, temperature, ctx=None):
    return GumbelSoftmaxOp(logits, temperature, ctx=ctx)


class ThresholdMaskOp(Op):
    """x * (x >= threshold): drops experts whose gate weight is negligible."""

    def __init__(self, x, threshold, ctx=None):
        super().__init__(ThresholdMaskOp, [x], ctx)
        self.threshold = threshold

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        return torch.where(x >= self.threshold, x, torch.zeros_like(x))

    def gradient(self, output_grad):
        return [ThresholdMaskGradOp(output_grad, self.inputs[0], self.threshold, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class ThresholdMaskGradOp(Op):
    def __init__(self, g, x, threshold, ctx=None):
        super().__init__(ThresholdMaskGradOp, [g, x], ctx)
        self.threshold = threshold

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, x = input_vals
        g = g.reshape(x.shape)
        return torch.where(x >= self.threshold, g, torch.zeros_like(g))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def threshold_mask_op(x, threshold, ctx=None):
    return ThresholdMaskOp(x, threshold, ctx=ctx)
