"""Graph IR node (reference ``python/hetu/gpu_ops/Node.py:18-220``).

Every operator is an ``Op`` with ``inputs``, a placement (``raw_ctx`` /
``ctx``) and three methods:

* ``compute(input_vals, output_val=None, stream_handle=None)`` -- produce the
  output tensor.  Unlike the reference (which writes into a buffer pre-planned by
  a Python memory pool), compute is *functional*: it returns a new tensor (or a
  zero-copy view) and the executor frees every value right after its last use, so
  memory is planned by liveness on top of the HIP stream-ordered caching
  allocator.  ``output_val`` is accepted for API compatibility; when given, the
  result is copied into it.
* ``gradient(output_grad)`` -- build gradient sub-graph nodes, one per input.
* ``infer_shape(input_shapes)`` -- static shape inference (used by the planner,
  profiler and pipeline partitioner).

``shape_only_inputs`` lists input indices whose *value* is never read (only its
shape, e.g. the reference operand of a broadcast-gradient reduction); the
executor passes a ``torch.Size`` for them and does not keep the producer's
tensor alive for them.
"""
from __future__ import annotations

from copy import copy, deepcopy
from typing import List, Optional

from ..context import DeviceGroup, get_current_context
from .. import ndarray

G_NODE_ID = 0


_SHADOW_DEPTH = [0]


def _next_id():
    global G_NODE_ID, G_SHADOW_ID
    if _SHADOW_DEPTH[0]:
        i = G_SHADOW_ID
        G_SHADOW_ID += 1
        return i
    i = G_NODE_ID
    G_NODE_ID += 1
    return i


class shadow_ids(object):
    """``with shadow_ids():`` nodes created inside take ids from the shadow range:
    placement-only additions (per-stage copies of a tied weight or of a mask
    computation) then leave the ids of the rest of the graph as in the unplaced model."""

    def __enter__(self):
        _SHADOW_DEPTH[0] += 1
        return self

    def __exit__(self, *a):
        _SHADOW_DEPTH[0] -= 1


# ids of "shadow" nodes (the pipeline-stage copy of a tied weight): a separate range
# below the PS key space (< 2^20) that does not advance the main counter, so adding
# such a copy leaves every other node's id -- and with it its ``seed + id`` initial
# value (reference initializers.py:13-16) -- unchanged
G_SHADOW_ID = 900000


def reassign_shadow_id(node):
    """Move ``node`` (just created) out of the main id sequence."""
    global G_NODE_ID, G_SHADOW_ID
    if node.id == G_NODE_ID - 1:
        G_NODE_ID -= 1
    node.id = G_SHADOW_ID
    G_SHADOW_ID += 1
    return node


class Op(object):
    """Basic unit of the computation graph."""

    shape_only_inputs = ()
    # number of outputs; >1 means compute returns a tuple and consumers pick
    # through ``OutputSelectOp``.
    num_outputs = 1

    def __init__(self, op_type, inputs: List['Op'], ctx=None):
        self.inputs: List[Op] = list(inputs)
        self.raw_ctx = get_current_context() if ctx is None else (
            ctx if isinstance(ctx, DeviceGroup) else DeviceGroup(ctx))
        self.ctx = ctx
        self.const_attr = None
        self.dtype = None
        self.inplace = False
        self.lazy_execution = False
        self.event = None
        self.use_indexed_slices = False
        self.op_type = op_type.__name__ if isinstance(op_type, type) else str(op_type)
        self.id = _next_id()
        self.name = self.op_type + str(self.id)

    @property
    def desc(self) -> str:
        return self.name + '(' + ', '.join(inp.name for inp in self.inputs) + ')'

    # operator sugar (reference Node.py:48-75) ---------------------------------
    def __add__(self, other):
        from .basic import add_op, addbyconst_op
        return add_op(self, other) if isinstance(other, Op) else addbyconst_op(self, other)

    def __mul__(self, other):
        from .basic import mul_op, mul_byconst_op
        return mul_op(self, other) if isinstance(other, Op) else mul_byconst_op(self, other)

    def __sub__(self, other):
        from .basic import minus_op, addbyconst_op
        return minus_op(self, other) if isinstance(other, Op) else addbyconst_op(self, -other)

    def __rsub__(self, other):
        from .basic import minus_byconst_op
        return minus_byconst_op(self, other)

    def __neg__(self):
        from .basic import opposite_op
        return opposite_op(self)

    def __truediv__(self, other):
        from .basic import div_op, mul_byconst_op
        return div_op(self, other) if isinstance(other, Op) else mul_byconst_op(self, 1.0 / other)

    def __rtruediv__(self, other):
        from .basic import div_const_op
        return div_const_op(other, self)

    __radd__ = __add__
    __rmul__ = __mul__

    def __str__(self):
        return self.name

    def __repr__(self):
        return self.name

    def __hash__(self):
        return self.id

    def __eq__(self, other):
        return self is other

    def __deepcopy__(self, memo):
        if id(self) not in memo:
            new_op = copy(self)
            memo[id(self)] = new_op
            new_op.id = _next_id()
            for k, v in self.__dict__.items():
                if k in ('inputs', 'grad_nodes'):
                    new_op.__dict__[k] = [deepcopy(n, memo) for n in v]
                elif k in ('grad_node', 'forward_node', 'optimizer'):
                    new_op.__dict__[k] = deepcopy(v, memo)
        return memo[id(self)]

    # the three op methods ------------------------------------------------------
    def compute(self, input_vals, output_val=None, stream_handle=None):
        raise NotImplementedError(self.op_type)

    def gradient(self, output_grad):
        raise NotImplementedError(self.op_type)

    def infer_shape(self, input_shapes):
        raise NotImplementedError(self.op_type)

    def naive_infer_shape(self, input_shapes):
        return self.infer_shape(input_shapes)

    # hooks (reference Node.py:192-213) ------------------------------------------
    def forward_hook(self, config):
        if getattr(config, 'pipeline', None) is not None or getattr(config, 'spmd', False) or \
                (getattr(config, 'cpu_only', False) and not isinstance(self.ctx, ndarray.DLContext)):
            # pipeline: each process computes only its own stage, on its own
            # device; cross-stage edges are p2p messages, not transfer ops
            self.ctx = config.context
            self.on_gpu = ndarray.is_gpu_ctx(self.ctx)
            self.on_cpu = not self.on_gpu
            return
        if self.ctx is None:
            self.ctx = config.context
        elif isinstance(self.ctx, DeviceGroup):
            self.ctx = config.resolve_ctx(self.ctx)
        elif not isinstance(self.ctx, ndarray.DLContext):
            self.ctx = config.resolve_ctx(DeviceGroup(self.ctx))
        for i, n in enumerate(self.inputs):
            self.inputs[i] = self.add_transfer_op(n, self.ctx, config.h2d_ops, config.d2h_ops)
        self.on_gpu = ndarray.is_gpu_ctx(self.ctx)
        self.on_cpu = not self.on_gpu

    def backward_hook(self, config):
        pass

    def reset_status(self):
        pass

    def add_transfer_op(self, src_node, dst_ctx, h2d_ops, d2h_ops):
        """Insert H2D/D2H ops across a host/device edge (ref ``Node.py:153-190``)."""
        from .transfer import datah2d_op, datad2h_op
        src_ctx = src_node.ctx
        if src_ctx is None or dst_ctx is None or src_ctx == dst_ctx:
            return src_node
        if not isinstance(src_ctx, ndarray.DLContext) or not isinstance(dst_ctx, ndarray.DLContext):
            return src_node
        if ndarray.is_gpu_ctx(dst_ctx):
            if ndarray.is_gpu_ctx(src_ctx):
                # GPU->GPU edges belong to the parallel lowering (RCCL send/recv)
                return src_node
            key = (src_node, dst_ctx)
            if key not in h2d_ops:
                h2d_ops[key] = datah2d_op(src_node, dst_ctx)
                h2d_ops[key].ctx = dst_ctx
                h2d_ops[key].on_gpu, h2d_ops[key].on_cpu = True, False
            return h2d_ops[key]
        key = src_node
        if key not in d2h_ops:
            d2h_ops[key] = datad2h_op(src_node)
            d2h_ops[key].ctx = dst_ctx
            d2h_ops[key].on_gpu, d2h_ops[key].on_cpu = False, True
        return d2h_ops[key]


class OutputSelectOp(Op):
    """Select output ``index`` of a multi-output op."""

    def __init__(self, node, index, ctx=None):
        super().__init__(OutputSelectOp, [node], ctx)
        self.index = index

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0][self.index]

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0][self.index]


def select_output(node, index, ctx=None):
    return OutputSelectOp(node, index, ctx)
