"""Collective-communication graph ops (reference AllReduceCommunicate.py,
AllGatherCommunicate.py, ReduceScatterCommunicate.py, BroadcastCommunicate.py,
ReduceCommunicate.py, AllToAll.py, HAllToAll.py, PipelineSend.py,
PipelineReceive.py).

All run RCCL collectives through ``parallel.comm.Communicator`` on the
stream the executor assigns to communication (``stream_kind = 'comm'``).
Dense gradient all-reduce inside the optimizer is *bucketed* and overlapped
with backward (see ``optimizer.OptimizerOp``); these standalone ops are the
user-visible primitives.
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

from .node import Op
from .. import ndarray
from ..parallel import comm as C


def _comm(c):
    return c if c is not None else C.init_process_group()


class AllReduceCommunicateOp(Op):
    """SUM all-reduce; IndexedSlices are all-gathered (indices and values)."""

    def __init__(self, node, comm=None, op='sum', ctx=None):
        super().__init__(AllReduceCommunicateOp, [node], ctx)
        self.comm, self.reduce_op = comm, op
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        v = input_vals[0]
        comm = _comm(self.comm)
        if isinstance(v, ndarray.IndexedSlices):
            idx = v._t(v.indices).reshape(-1).contiguous()
            val = v._t(v.values).reshape(idx.numel(), -1).contiguous()
            oi = _NA.empty((idx.numel() * comm.nrank,), dtype=idx.dtype, device=idx.device)
            ov = _NA.empty((val.shape[0] * comm.nrank, val.shape[1]), dtype=val.dtype, device=val.device)
            comm.all_gather(oi, idx)
            comm.all_gather(ov, val)
            return ndarray.IndexedSlices(oi, ov, v.dense_shape)
        out = v.clone() if not v.is_contiguous() or True else v
        comm.all_reduce(out, self.reduce_op)
        return out

    def gradient(self, output_grad):
        return [allreduceCommunicate_op(output_grad, self.comm, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def allreduceCommunicate_op(node, comm=None, ctx=None):
    return AllReduceCommunicateOp(node, comm, ctx=ctx)


def allreduceCommunicatep2p_op(node, comm=None, ctx=None):
    return AllReduceCommunicateOp(node, comm, ctx=ctx)


def groupallreduceCommunicate_op(node, group_comm, ctx=None):
    return AllReduceCommunicateOp(node, group_comm, ctx=ctx)


class AllGatherCommunicateOp(Op):
    def __init__(self, node, comm=None, ctx=None):
        super().__init__(AllGatherCommunicateOp, [node], ctx)
        self.comm = comm
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0].contiguous()
        comm = _comm(self.comm)
        out = _NA.empty((x.shape[0] * comm.nrank,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        comm.all_gather(out, x)
        return out

    def gradient(self, output_grad):
        return [reducescatterCommunicate_op(output_grad, self.comm, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        s[0] *= _comm(self.comm).nrank
        return tuple(s)


def allgatherCommunicate_op(node, comm=None, ctx=None):
    return AllGatherCommunicateOp(node, comm, ctx=ctx)


class ReduceScatterCommunicateOp(Op):
    def __init__(self, node, comm=None, ctx=None):
        super().__init__(ReduceScatterCommunicateOp, [node], ctx)
        self.comm = comm
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0].contiguous()
        comm = _comm(self.comm)
        out = _NA.empty((x.shape[0] // comm.nrank,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        comm.reduce_scatter(out, x)
        return out

    def gradient(self, output_grad):
        return [allgatherCommunicate_op(output_grad, self.comm, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        s[0] //= _comm(self.comm).nrank
        return tuple(s)


def reducescatterCommunicate_op(node, comm=None, ctx=None):
    return ReduceScatterCommunicateOp(node, comm, ctx=ctx)


class BroadcastCommunicateOp(Op):
    def __init__(self, node, comm=None, root=0, ctx=None):
        super().__init__(BroadcastCommunicateOp, [node], ctx)
        self.comm, self.root = comm, root
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        comm = _comm(self.comm)
        x = input_vals[0]
        # shape header first (reference broadcasts the shape in infer_shape)
        hdr = _NA.zeros(8, dtype=torch.int64, device=x.device)
        if comm.rank == self.root:
            hdr[0] = x.dim()
            hdr[1:1 + x.dim()] = torch.tensor(x.shape, dtype=torch.int64)
        comm.broadcast(hdr, self.root)
        shape = tuple(int(v) for v in hdr[1:1 + int(hdr[0])].tolist())
        out = x.contiguous().clone() if comm.rank == self.root else _NA.empty(shape, dtype=x.dtype, device=x.device)
        comm.broadcast(out, self.root)
        return out

    def gradient(self, output_grad):
        return [reduceCommunicate_op(output_grad, self.comm, self.root, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def broadcastCommunicate_op(node, comm=None, root=0, ctx=None):
    return BroadcastCommunicateOp(node, comm, root, ctx=ctx)


class ReduceCommunicateOp(Op):
    def __init__(self, node, comm=None, root=0, ctx=None):
        super().__init__(ReduceCommunicateOp, [node], ctx)
        self.comm, self.root = comm, root
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        comm = _comm(self.comm)
        out = input_vals[0].contiguous().clone()
        comm.reduce(out, self.root)
        return out

    def gradient(self, output_grad):
        return [broadcastCommunicate_op(output_grad, self.comm, self.root, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def reduceCommunicate_op(node, comm=None, root=0, ctx=None):
    return ReduceCommunicateOp(node, comm, root, ctx=ctx)


class AllToAllOp(Op):
    def __init__(self, node, comm=None, ctx=None):
        super().__init__(AllToAllOp, [node], ctx)
        self.comm = comm
        self.stream_kind = 'comm'

    def compute(self, input_vals, output_val=None, stream_handle=None):
        comm = _comm(self.comm)
        x = input_vals[0].contiguous()
        if comm.nrank == 1:
            return x
        out = _NA.empty_like(x)
        comm.all_to_all(out, x)
        return out

    def gradient(self, output_grad):
        return [alltoall_op(output_grad, self.comm, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def alltoall_op(node, comm=None, ctx=None):
    return AllToAllOp(node, comm, ctx=ctx)


class HAllToAllOp(AllToAllOp):
    """Hierarchical all-to-all (reference HAllToAll.py:24-59).  On a single
    MI355X node every GPU is one xGMI hop from every other, so the two-level
    (intra-node gather -> inter-node A2A -> scatter) schedule degenerates to the
    direct mesh all-to-all; multi-node runs route through the same RCCL call,
    which is topology aware."""

    def __init__(self, node, num_nodes=1, num_local_gpus=8, comm=None, ctx=None):
        super().__init__(node, comm, ctx)
        self.op_type = 'HAllToAllOp'
        self.num_nodes, self.num_local_gpus = num_nodes, num_local_gpus

    def gradient(self, output_grad):
        return [halltoall_op(output_grad, self.num_nodes, self.num_local_gpus, self.comm, ctx=self.raw_ctx)]


def halltoall_op(node, num_nodes=1, num_local_gpus=8, comm=None, ctx=None):
    return HAllToAllOp(node, num_nodes, num_local_gpus, comm, ctx=ctx)


class PipelineSendOp(Op):
    """Send to a pipeline peer; the shape header travels once per channel (static shapes,
    as the reference), or with every message when ``dynamic_shapes``."""

    def __init__(self, node, destination, comm=None, ctx=None, dynamic_shapes=False):
        super().__init__(PipelineSendOp, [node], ctx)
        self.const_attr = destination
        self.comm = comm
        self.stream_kind = 'p2p'
        self.dynamic_shapes = dynamic_shapes
        self._chan = {'dynamic': dynamic_shapes}

    def compute(self, input_vals, output_val=None, stream_handle=None, group_call=False):
        from ..parallel import pipeline as PP
        PP.send_tensor(_comm(self.comm), input_vals[0], self.const_attr, None if self.dynamic_shapes else self._chan)
        return None

    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        return None


class PipelineReceiveOp(Op):
    def __init__(self, source, comm=None, ctx=None, dynamic_shapes=False):
        super().__init__(PipelineReceiveOp, [], ctx)
        self.const_attr = source
        self.comm = comm
        self.stream_kind = 'p2p'
        self.dynamic_shapes = dynamic_shapes
        self._chan = {}

    def compute(self, input_vals, output_val=None, stream_handle=None, group_call=False):
        from ..parallel import pipeline as PP
        return PP.recv_tensor(_comm(self.comm), self.const_attr, self.device,
                              None if self.dynamic_shapes else self._chan)

    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        return None


def pipeline_send_op(node, destination, comm=None, ctx=None, dynamic_shapes=False):
    return PipelineSendOp(node, destination, comm, ctx=ctx, dynamic_shapes=dynamic_shapes)


def pipeline_receive_op(source, comm=None, ctx=None, dynamic_shapes=False):
    return PipelineReceiveOp(source, comm, ctx=ctx, dynamic_shapes=dynamic_shapes)
