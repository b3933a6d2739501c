"""DistGCN-1.5D layer vs a dense single-process reference (reference pattern:
tests/test_DistGCN/test_model_distGCN15d.py compares against one GPU).  Runs
P processes on CPU (gloo) for (P, c) in {(2, 1), (4, 2), (4, 1)}."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n=11, f=6, k=4, seed=0):
    rng = np.random.RandomState(seed)
    A = (rng.rand(n, n) < 0.3).astype(np.float32)
    A = np.maximum(A, A.T) + np.eye(n, dtype=np.float32)
    d = 1.0 / np.sqrt(A.sum(1))
    A = (A * d[:, None] * d[None, :]).astype(np.float32)  # symmetric normalised adjacency
    H = rng.randn(n, f).astype(np.float32)
    W = rng.randn(f, k).astype(np.float32)
    R = rng.randn(n, k).astype(np.float32)
    return A, H, W, R


def _worker(rank, size, c, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.parallel import comm as C
    world = C.init_process_group(use_gpu=False)
    A, H, W, R = _problem()
    n = A.shape[0]
    groups = ht.make_15d_groups(size, c)
    blkA, (r0, r1) = ht.partition_15d(A, n, rank, size, c)
    a_node = ht.Variable(name='A', trainable=False)
    h = ht.Variable(name='H', value=H[r0:r1])
    w = ht.Variable(name='W', value=W)
    r_node = ht.Variable(name='R', trainable=False)
    z = ht.distgcn_15d_op(a_node, h, w, r1 - r0, n, size, c, comm=world, comm_groups=groups)
    loss = ht.reduce_sum_op(ht.mul_op(z, r_node), [0, 1])
    gh, gw = ht.gradients(loss, [h, w])
    ex = ht.Executor({'t': [z, gh, gw]}, ctx=ht.cpu(0))
    zv, ghv, gwv = ex.run('t', feed_dict={a_node: blkA, r_node: R[r0:r1]}, convert_to_numpy_ret_vals=True)
    q.put((rank, r0, r1, zv, ghv, gwv))
    C.destroy()


@pytest.mark.parametrize('size,c', [(2, 1), (4, 2), (4, 1)])
def test_distgcn_15d_matches_dense(size, c):
    A, H, W, R = _problem()
    Z = A @ H @ W
    dH = A @ R @ W.T
    dW = H.T @ A @ R
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, size, c, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, r0, r1, zv, ghv, gwv in res:
        np.testing.assert_allclose(zv, Z[r0:r1], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(ghv, dH[r0:r1], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(gwv, dW, rtol=1e-4, atol=1e-4)


def test_gcn_single_device_trains():
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models.gcn import gcn
    A, H, _, _ = _problem(n=40, f=12)
    rng = np.random.RandomState(1)
    Y = np.eye(3, dtype=np.float32)[rng.randint(0, 3, 40)]
    a = ht.sparse_array(A[A != 0], np.nonzero(A), A.shape)
    adj, x, y_ = ht.Variable(name='adj', trainable=False), ht.Variable(name='x', trainable=False), \
        ht.Variable(name='y', trainable=False)
    loss, _ = gcn(adj, x, y_, 12, hidden=16, num_classes=3)
    train = ht.optim.AdamOptimizer(0.05).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=3)
    ls = [float(ex.run('train', feed_dict={adj: a, x: H, y_: Y}, convert_to_numpy_ret_vals=True)[0])
          for _ in range(60)]
    assert ls[-1] < 0.85 * ls[0]
