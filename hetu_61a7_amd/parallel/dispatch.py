"""Model-parallel split descriptors and the ``dispatch`` op (reference
gpu_ops/Dispatch.py:11-65, Variable.py:83-125).  The lowering pass that turns
``dispatch`` annotations into per-device sub-graphs with RCCL collectives (the
piece missing from the reference) lives in ``parallel.lowering``.
"""
from __future__ import annotations

import torch

from ..ops.node import Op


class MPSplit(object):
    """Which shard of a global tensor this rank owns: ``parts = {axis: nparts}``,
    ``cur_part = {axis: index}``."""

    def __init__(self, cur_part, parts):
        self.cur_part = dict(cur_part) if not isinstance(cur_part, dict) else cur_part
        self.parts = dict(parts) if not isinstance(parts, dict) else parts

    def local_shape(self, shape):
        s = list(shape)
        for ax, n in self.parts.items():
            s[ax] = s[ax] // n
        return tuple(s)

    def slices(self, shape):
        sl = []
        for ax, d in enumerate(shape):
            if ax in self.parts:
                part = d // self.parts[ax]
                st = part * self.cur_part[ax]
                sl.append(slice(st, st + part))
            else:
                sl.append(slice(None))
        return tuple(sl)

    def slice_tensor(self, t):
        return t[self.slices(t.shape)].contiguous()


class DispatchOp(Op):
    """Declares a split of its input: ``parts`` maps axis -> number of parts.
    Consumed by the lowering pass; executing it un-lowered is an identity."""

    def __init__(self, node, parts, ctx=None):
        super().__init__(DispatchOp, [node], ctx)
        self.parts = parts

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0]

    def gradient(self, output_grad):
        return [DispatchGradientOp(output_grad, self.inputs[0], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class DispatchGradientOp(Op):
    def __init__(self, node, forward_input, ctx=None):
        super().__init__(DispatchGradientOp, [node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0]

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def dispatch(node, parts=None, ctx=None):
    if parts is None:
        parts = {}
    if isinstance(parts, (list, tuple)):
        parts = {i: p for i, p in enumerate(parts) if p > 1}
    return DispatchOp(node, parts, ctx=ctx)


def apply_model_parallel_cnn(node_list, settings):
    from .lowering import model_parallel_cnn
    return model_parallel_cnn(node_list, settings)


def apply_model_parallel_lm(node_list, settings):
    from .lowering import model_parallel_lm
    return model_parallel_lm(node_list, settings)


def apply_one_weird_trick(node_list, settings):
    from .lowering import one_weird_trick
    return one_weird_trick(node_list, settings)
