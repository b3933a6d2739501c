"""1.5-D distributed GCN layer (reference ``gpu_ops/DistGCN_15d.py:9-156``;
SURVEY §2.3 S12).

``P`` processes, replication factor ``c`` (``P % c**2 == 0``):

* the node set is split into ``P/c`` row blocks; process ``r`` owns row block
  ``r // c`` of the features ``H`` and the rows of the adjacency ``A`` for that
  block, restricted to the node columns of its *column group* ``r % c``
  (column indices relative to the start of that column range);
* forward, per stage ``i`` of ``P/c**2``: the owner ``q`` of the next H block
  broadcasts it inside the column group (RCCL over xGMI), every member does a
  windowed CSR SpMM ``A[:, window_i] @ H_q`` into its accumulator; finally the
  ``c`` replicas of a row block all-reduce (row group) -> ``(A @ H)[block]``;
* ``Z = (A @ H) @ W`` (or ``A @ (H @ W)`` when W narrows the features, which
  shrinks the broadcast payload);
* backward: ``dH = (A @ dZ) @ W^T`` (A is the symmetric normalised adjacency, so
  ``A^T = A``), ``dW = H^T (A @ dZ)`` summed over the column group.
"""
from __future__ import annotations

import math

import torch
from .. import native_array as _NA

from .node import Op
from ..kernels import spmm as KSP


def row_num(node_count, rank, size):
    """Rows of block ``rank`` when ``node_count`` rows are split in ``size``
    near-equal blocks (reference DistGCN_15d.py:9-16)."""
    n_per_proc = math.ceil(float(node_count) / size)
    if node_count % size == 0:
        return node_count // size
    return int(n_per_proc) if rank < size - 1 else int(node_count % n_per_proc)


def make_15d_groups(size, replication):
    """(row_groups, col_groups): row group ``k`` = the c replicas of row block k,
    column group ``j`` = ranks ``r`` with ``r % c == j``.  Every rank must call
    this (group creation is collective)."""
    from ..parallel.comm import new_group_comm
    c = replication
    row_groups = [new_group_comm(list(range(k * c, (k + 1) * c))) if c > 1 else None
                  for k in range(size // c)]
    col_groups = [new_group_comm([r for r in range(size) if r % c == j]) for j in range(c)]
    return row_groups, col_groups


def broad_func(node_count, adj, inputs, rank, size, replication, row_groups, col_groups, comm):
    """Distributed ``(A @ H)[own row block]`` (reference DistGCN_15d.py:19-70)."""
    c = replication
    assert size % (c * c) == 0, 'size must be a multiple of replication^2'
    n_per_proc = math.ceil(float(node_count) / (size // c))
    rank_c, rank_col = rank // c, rank % c
    proc_rows = row_num(node_count, rank_c, size // c)
    feat = inputs.shape[1]
    z = _NA.zeros((proc_rows, feat), dtype=inputs.dtype, device=inputs.device)
    stages = size // (c * c)
    node_count_col = stages * n_per_proc
    if rank_col == c - 1:
        stages = (size // c) - (c - 1) * stages
        node_count_col = node_count - (c - 1) * node_count_col
    starts = list(range(0, int(node_count_col), int(n_per_proc)))
    ends = starts[1:] + [int(node_count_col)]
    group = col_groups[rank_col] if c > 1 else comm
    for i in range(stages):
        q = (rank_col * (size // (c * c)) + i) * c + rank_col
        q_c = q // c
        rows_q = row_num(node_count, q_c, size // c)
        if q == rank:
            buf = inputs.contiguous().clone()
        else:
            buf = _NA.empty((rows_q, feat), dtype=inputs.dtype, device=inputs.device)
        root = q // c if c > 1 else q  # group-local index of q inside its column group
        group.broadcast(buf, root)
        KSP.csrmm(adj, buf, col_window=(starts[i], ends[i]), out=z, accumulate=True)
    if c > 1:
        row_groups[rank_c].all_reduce(z, 'sum')
    return z


class DistGCN_15dOp(Op):
    def __init__(self, node_A, node_B, node_C, node_Count_Self, node_Count_All, size, replication,
                 device_id=None, comm=None, comm_groups=(None, None), need_W=True, ctx=None):
        super().__init__(DistGCN_15dOp, [node_A, node_B, node_C], ctx)
        self.need_W = need_W
        self.node_Count_Self, self.node_Count_All = node_Count_Self, node_Count_All
        self.replication, self.size = replication, size
        self.comm, self.comm_groups = comm, list(comm_groups)
        self.device_id = device_id
        self.stream_kind = 'comm'

    def _comm(self):
        from ..parallel import comm as C
        return self.comm if self.comm is not None else C.init_process_group()

    def compute(self, input_vals, output_val=None, stream_handle=None):
        adj, H, W = input_vals
        comm = self._comm()
        rank = comm.rank
        rg, cg = self.comm_groups[0], self.comm_groups[1]
        if self.need_W and W.shape[1] < H.shape[1]:
            return broad_func(self.node_Count_All, adj, H @ W.to(H.dtype), rank, self.size,
                              self.replication, rg, cg, comm)
        AH = broad_func(self.node_Count_All, adj, H, rank, self.size, self.replication, rg, cg, comm)
        return AH @ W.to(AH.dtype) if self.need_W else AH

    def gradient(self, output_grad):
        from .linalg import matmul_op
        from .comm import groupallreduceCommunicate_op
        adj, H, W = self.inputs
        ag = distgcn_15d_op(adj, output_grad, W, self.node_Count_Self, self.node_Count_All, self.size,
                            self.replication, self.device_id, self.comm, self.comm_groups,
                            need_W=False, ctx=self.raw_ctx)
        grad_H = matmul_op(ag, W, trans_B=True, ctx=self.raw_ctx)
        grad_weight = matmul_op(H, ag, trans_A=True, ctx=self.raw_ctx)
        if self.replication > 1:
            groups = self.comm_groups[2] if len(self.comm_groups) == 3 else self.comm_groups[1]
            rank = self._comm().rank
            grad_W = groupallreduceCommunicate_op(grad_weight, groups[rank % self.replication],
                                                  ctx=self.raw_ctx)
        else:
            grad_W = groupallreduceCommunicate_op(grad_weight, self.comm, ctx=self.raw_ctx)
        return [None, grad_H, grad_W]

    def infer_shape(self, input_shapes):
        H, W = input_shapes[1], input_shapes[2]
        return (self.node_Count_Self, W[1] if self.need_W else H[1])


def distgcn_15d_op(node_A, node_B, node_C, node_Count_Self, node_Count_All, size, replication,
                   device_id=None, comm=None, comm_groups=(None, None), need_W=True, ctx=None):
    return DistGCN_15dOp(node_A, node_B, node_C, node_Count_Self, node_Count_All, size, replication,
                         device_id, comm, comm_groups, need_W=need_W, ctx=ctx)


def partition_15d(adj_dense_or_csr, node_count, rank, size, replication):
    """Host helper: the CSR block process ``rank`` holds -- rows of its row block,
    columns of its column group, column indices relative to the group start."""
    import numpy as np
    import scipy.sparse
    from ..ndarray import ND_Sparse_Array, array
    c = replication
    A = scipy.sparse.csr_matrix(adj_dense_or_csr)
    n_per_proc = math.ceil(float(node_count) / (size // c))
    rank_c, rank_col = rank // c, rank % c
    r0 = rank_c * n_per_proc
    r1 = r0 + row_num(node_count, rank_c, size // c)
    stages = size // (c * c)
    col0 = rank_col * stages * n_per_proc
    col1 = col0 + stages * n_per_proc if rank_col < c - 1 else node_count
    blk = A[r0:r1, col0:col1].tocsr()
    return ND_Sparse_Array(array(blk.data.astype(np.float32)), array(blk.indptr, dtype=np.int32),
                           array(blk.indices, dtype=np.int32), blk.shape[0], blk.shape[1]), (r0, r1)
