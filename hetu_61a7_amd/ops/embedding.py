"""Embedding lookup with row-sparse gradients (reference EmbeddingLookUp.py:11-149).

Forward: wave-per-row vectorised HIP gather.  Backward: an ``IndexedSlices``
(ids, grad rows) that the optimizer applies as a row-sparse update after a
device-side de-duplication -- the dense table gradient is never materialised.
When the table is PS/HET-cache managed the lookup is served by the PS op
(``ops.ps``) instead.
"""
from __future__ import annotations

import torch

from .node import Op
from .. import ndarray
from ..kernels import sparse as KS


class EmbeddingLookUp(Op):
    def __init__(self, embedding, index, ctx=None):
        super().__init__(EmbeddingLookUp, [embedding, index], ctx)
        embedding.is_embed = True
        self.grad_node = None
        self.out_dtype = None  # set to bf16 under mixed precision

    def forward_hook(self, config):
        Op.forward_hook(self, config)
        if config.mixed_precision and ndarray.is_gpu_ctx(self.ctx):
            self.out_dtype = torch.bfloat16
        if getattr(self.inputs[0], 'ps_managed', False):
            # ids are consumed on the host by the PS / HET cache
            self.inputs[1].host_feed = True

    def compute(self, input_vals, output_val=None, stream_handle=None):
        table, idx = input_vals
        if not isinstance(table, torch.Tensor):  # PS / HET-cache managed table
            return table.lookup(idx, self.out_dtype)
        out = KS.gather_rows(table, idx)
        if self.out_dtype is not None and out.dtype != self.out_dtype:
            from ..kernels.elementwise import cast
            out = cast(out, self.out_dtype)
        return out

    def gradient(self, output_grad):
        self.grad_node = embedding_lookup_gradient_op(output_grad, self.inputs[1], self.inputs[0], ctx=self.raw_ctx)
        return [self.grad_node, None]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[1]) + (input_shapes[0][-1],)


def _rows(t, width):
    """t as [-1] / [-1, width]: a view when the layout allows, else a native copy (a strided
    gradient -- e.g. of a broadcast / transposed consumer -- would otherwise go through
    torch's copy kernel on the device)"""
    shape = (-1,) if width is None else (-1, width)
    try:
        return t.view(*shape)
    except RuntimeError:
        if t.is_cuda:
            from .. import native_array as _NA
            from ..kernels.tensor import copy_into
            t = copy_into(_NA.empty(tuple(t.shape), dtype=t.dtype, device=t.device), t)
        return t.reshape(*shape)


class EmbeddingLookUp_Gradient(Op):
    shape_only_inputs = (2,)

    def __init__(self, vectors, index, embed_ref, ctx=None):
        super().__init__(EmbeddingLookUp_Gradient, [vectors, index, embed_ref], ctx)
        self.use_indexed_slices = True

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, idx, shape = input_vals
        width = tuple(shape)[-1]
        return ndarray.IndexedSlices(_rows(idx, None), _rows(g, width), tuple(shape))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def embedding_lookup_op(embedding, index, ctx=None):
    return EmbeddingLookUp(embedding, index, ctx=ctx)


def embedding_lookup_gradient_op(vectors, index, embed_shape, ctx=None):
    return EmbeddingLookUp_Gradient(vectors, index, embed_shape, ctx=ctx)
