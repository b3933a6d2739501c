"""Variables / placeholders (reference ``gpu_ops/Variable.py:8-140``)."""
from __future__ import annotations

import numpy as np
import torch

from .node import Op
from .. import ndarray


def Variable(name, value=None, initializer=None, trainable=True, dtype=np.float32, ctx=None):
    """Trainable parameter (``trainable=True`` with a value/initializer) or a fed
    placeholder (no value)."""
    return placeholder_op(name, value, initializer, trainable, dtype, ctx)


class PlaceholderOp(Op):
    def __init__(self, name, value=None, initializer=None, trainable=True, dtype=np.float32, ctx=None):
        super().__init__(PlaceholderOp, [], ctx)
        if name is not None:
            self.name = name
        self.is_embed = False
        self.shape = None
        if value is None and initializer is None:
            trainable = False
        elif value is not None:
            assert initializer is None, 'Value already specified, initializer should be None.'
            if isinstance(value, ndarray.NDArray):
                value = value.asnumpy()
            if isinstance(value, torch.Tensor):
                value = value.detach().cpu().numpy()
            assert isinstance(value, np.ndarray), 'Value data type %s not valid.' % type(value)
            self.shape = tuple(value.shape)
        else:
            self.shape = tuple(initializer.shape)
        self.tensor_value = value
        self.initializer = initializer
        self.trainable = trainable
        self.dtype = dtype
        self.reshaped = False
        self.embedding_offsets = None
        # set by parallel lowering: (axis -> parts, index) slicing of a global tensor
        self.mp_split = None

    def compute(self, input_vals, output_val=None, stream_handle=None):
        raise AssertionError('placeholder %s: value provided by the executor' % self.name)

    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        assert self.shape, 'placeholder %s shape provided by feed_shape' % self.name
        return self.shape

    def forward_hook(self, config):
        if self.ctx is None or not isinstance(self.ctx, ndarray.DLContext):
            Op.forward_hook(self, config)
        self.on_gpu = ndarray.is_gpu_ctx(self.ctx)
        self.on_cpu = not self.on_gpu

    def backward_hook(self, config):
        pass

    # ---- value materialisation (called by the executor) ----------------------
    @property
    def is_param(self) -> bool:
        return self.tensor_value is not None or self.initializer is not None

    def initial_value(self, seed: int, device) -> torch.Tensor:
        if self.tensor_value is not None:
            t = torch.from_numpy(np.ascontiguousarray(self.tensor_value))
            if t.dtype == torch.float64:
                t = t.float()
            t = t.to(device)
        else:
            # a parameter tied to another (``tied_to``: the pipeline-stage copy of a shared
            # weight) draws exactly its source's initial values (seed + source id)
            src = getattr(self, 'tied_to', None)
            t = self.initializer(src if src is not None else self, seed, device=device)
        if self.mp_split is not None:
            t = self.mp_split.slice_tensor(t)
        return t

    def reshape_in_mp(self, cur_part, parts):
        """Keep only this model-parallel shard (reference Variable.py:83-125)."""
        from ..parallel.dispatch import MPSplit
        self.mp_split = MPSplit(cur_part, parts)
        if self.shape is not None:
            self.shape = self.mp_split.local_shape(self.shape)
        self.reshaped = True


def placeholder_op(name, value=None, initializer=None, trainable=True, dtype=np.float32, ctx=None):
    return PlaceholderOp(name, value, initializer, trainable, dtype, ctx)
