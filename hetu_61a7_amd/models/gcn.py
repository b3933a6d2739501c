"""Graph convolutional networks (reference examples/gnn/gnn_model/*,
tests/test_DistGCN/test_model_distGCN15d.py).

``gcn``: two-layer GCN on one device, ``softmax(A relu(A X W1) W2)`` with the
normalised adjacency ``A`` fed as a CSR ``ND_Sparse_Array`` (hand-written
wave-per-row SpMM on the GPU).  ``dist_gcn_15d``: the same network with every
propagation distributed 1.5-D over P processes (``ops.distgcn``).  GraphMix
sampling (an empty submodule in the reference) is not part of this build; the
graph is an in-memory CSR.
"""
from __future__ import annotations

from .. import initializers as init
from ..ops import (csrmm_op, matmul_op, relu_op, softmaxcrossentropy_op, reduce_mean_op,
                   distgcn_15d_op)


def gcn(adj, x, y_, in_dim, hidden=16, num_classes=7):
    w1 = init.xavier_uniform((in_dim, hidden), name='gcn_w1')
    w2 = init.xavier_uniform((hidden, num_classes), name='gcn_w2')
    h = relu_op(csrmm_op(adj, matmul_op(x, w1)))
    logits = csrmm_op(adj, matmul_op(h, w2))
    loss = reduce_mean_op(softmaxcrossentropy_op(logits, y_), [0])
    return loss, logits


def dist_gcn_15d(adj_block, x_block, y_block, rows_self, node_count, size, replication, comm,
                 comm_groups, in_dim, hidden=16, num_classes=7):
    w1 = init.xavier_uniform((in_dim, hidden), name='gcn_w1')
    w2 = init.xavier_uniform((hidden, num_classes), name='gcn_w2')
    h = relu_op(distgcn_15d_op(adj_block, x_block, w1, rows_self, node_count, size, replication,
                               comm=comm, comm_groups=comm_groups))
    logits = distgcn_15d_op(adj_block, h, w2, rows_self, node_count, size, replication, comm=comm,
                            comm_groups=comm_groups)
    loss = reduce_mean_op(softmaxcrossentropy_op(logits, y_block), [0])
    return loss, logits
