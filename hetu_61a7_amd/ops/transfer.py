"""Host<->device transfer ops (reference gpu_ops/DataTransfer.py:7-157).

H2D copies are issued asynchronously from pinned host memory on the
executor's dedicated H2D stream; the consumer stream waits on an event
(``hipStreamWaitEvent``), never on the host.
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

from .node import Op
from .. import ndarray


class DataH2DOp(Op):
    def __init__(self, node, ctx=None):
        super().__init__(DataH2DOp, [node], ctx)
        self.stream_kind = 'h2d'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        v = input_vals[0]
        dev = self.ctx.torch_device
        if isinstance(v, ndarray.IndexedSlices):
            return ndarray.IndexedSlices(v._t(v.indices).to(dev, non_blocking=True),
                                         v._t(v.values).to(dev, non_blocking=True), v.dense_shape)
        if not v.is_pinned() and not v.is_cuda and torch.cuda.is_available():
            v = v.pin_memory()
        return v.to(dev, non_blocking=True)

    def gradient(self, output_grad):
        return [datad2h_op(output_grad)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class DataD2HOp(Op):
    def __init__(self, node, ctx=None):
        super().__init__(DataD2HOp, [node], ctx)
        self.stream_kind = 'd2h'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        v = input_vals[0]
        if isinstance(v, ndarray.IndexedSlices):
            return v.cpu()
        out = _NA.empty(v.shape, dtype=v.dtype, pin_memory=torch.cuda.is_available())
        out.copy_(v, non_blocking=True)
        return out

    def gradient(self, output_grad):
        return [datah2d_op(output_grad, self.inputs[0].ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def datah2d_op(node, ctx=None):
    return DataH2DOp(node, ctx=ctx)


def datad2h_op(node, ctx=None):
    return DataD2HOp(node, ctx=ctx)


def datah2d_sparse_op(node, ctx=None):
    op = DataH2DOp(node, ctx=ctx)
    op.use_indexed_slices = True
    return op


def datad2h_sparse_op(node, ctx=None):
    op = DataD2HOp(node, ctx=ctx)
    op.use_indexed_slices = True
    return op
