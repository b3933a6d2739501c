"""Multi-process data-parallel tests on CPU (gloo, world_size 2).

Parallel-equivalence pattern of the reference (examples/runner/parallel/
validate_results.py): DP with SUM all-reduce and lr/N must reproduce the
single-process baseline on the concatenated batch.  The ZeRO-1 variant
(reduce-scatter, sharded optimizer state, all-gather of the weights) must
reproduce it too.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mlp_losses(X, Y, lr, steps, dp=False, bucket_mb=32, opt='momentum', zero=0):
    import hetu_61a7_amd as ht
    rng = np.random.RandomState(11)
    w1 = (rng.randn(20, 32) * 0.3).astype(np.float32)
    w2 = (rng.randn(32, 4) * 0.3).astype(np.float32)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W1 = ht.Variable(name='w1', value=w1)
    B1 = ht.Variable(name='b1', value=np.zeros(32, np.float32))
    W2 = ht.Variable(name='w2', value=w2)
    h = ht.relu_op(ht.linear_op(x, W1, B1))
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, W2), y_), [0])
    o = ht.optim.MomentumOptimizer(lr, 0.9) if opt == 'momentum' else ht.optim.AdamOptimizer(lr)
    train = o.minimize(loss)
    kw = dict(bucket_mb=bucket_mb)
    if zero:
        kw['zero'] = zero
    if dp:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), **kw)
    out = []
    for _ in range(steps):
        out.append(float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]))
    params = {n.name: v.numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items() if n.trainable}
    info = {}
    if train.flat is not None:
        info = dict(zero=train.zero, padded=train.flat.padded,
                    state=train.flat.s1.numel() if train.flat.s1 is not None else 0, buckets=len(train.buckets))
    return out, params, info


def _worker(rank, world, port, X, Y, q, opt, zero):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HETU_USE_CONFIG='0')
    n = X.shape[0] // world
    sl = slice(rank * n, (rank + 1) * n)
    lr = 0.1 / world if opt == 'momentum' else 0.01
    # tiny bucket so several buckets are exercised
    losses, params, info = _mlp_losses(X[sl], Y[sl], lr, 5, dp=True, bucket_mb=0.001, opt=opt, zero=zero)
    q.put((rank, losses, params, info))
    from hetu_61a7_amd.parallel import comm
    comm.destroy()


def _run_dp(X, Y, opt, zero, world=2):
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, X, Y, q, opt, zero)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    return res


def _data():
    rng = np.random.RandomState(0)
    X = rng.randn(32, 20).astype(np.float32)
    Y = np.eye(4, dtype=np.float32)[rng.randint(0, 4, 32)]
    return X, Y


def test_dp_allreduce_matches_single_process():
    X, Y = _data()
    # baseline: one process on the full batch (mean loss), lr 0.1
    _, base_params, _ = _mlp_losses(X, Y, 0.1, 5)
    res = _run_dp(X, Y, 'momentum', 0)
    # SUM all-reduce of per-shard mean-loss grads with lr/N == full-batch mean with lr
    for name, v in base_params.items():
        np.testing.assert_allclose(res[0][2][name], v, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(res[1][2][name], v, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('opt', ['momentum', 'adam'])
def test_zero1_matches_single_process(opt):
    X, Y = _data()
    # Adam is invariant to the gradient scale (SUM of 2 shard means = 2 x full mean)
    _, base_params, _ = _mlp_losses(X, Y, 0.1 if opt == 'momentum' else 0.01, 5, opt=opt)
    res = _run_dp(X, Y, opt, 1)
    for rank, _, params, info in res:
        assert info['zero'] and info['buckets'] > 1
        if opt == 'adam':
            assert info['state'] == info['padded'] // 2     # optimizer state sharded over 2 ranks
        for name, v in base_params.items():
            np.testing.assert_allclose(params[name], v, rtol=2e-4, atol=2e-5)


def _resnet_worker(rank, world, port, q):
    """bench.py's ResNet-50 data-parallel path (DataParallel('allreduce'), bucketed
    SUM all-reduce, momentum SGD with lr/N) on gloo, 1 image per rank."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HETU_USE_CONFIG='0')
    torch.set_num_threads(2)
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models import resnet50_imagenet
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    loss, _ = resnet50_imagenet(x, y_, 10)
    train = ht.optim.MomentumOptimizer(learning_rate=0.1 / world, momentum=0.9).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'),
                     mixed_precision='bf16', bucket_mb=8, seed=1234)
    rng = np.random.RandomState(100 + rank)
    X = rng.randn(1, 3, 224, 224).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 1)]
    losses = [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0])
              for _ in range(2)]
    params = {n.name: v.numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items()
              if n.trainable and ('fc' in n.name or n.name.startswith('stem'))}
    q.put((rank, losses, params, len(train.buckets)))
    from hetu_61a7_amd.parallel import comm
    comm.destroy()


def test_resnet50_dp_bench_path_keeps_replicas_identical():
    """Rehearsal of the driver's N-GPU bench: every rank must hold identical weights
    after each all-reduced step (per-rank data differs)."""
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_resnet_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, l0, p0, nb0), (_, l1, p1, nb1) = res
    assert np.all(np.isfinite(l0 + l1)) and l0 != l1        # different data per rank
    assert nb0 == nb1 and nb0 > 1                            # several buckets exercised
    assert p0.keys() == p1.keys() and len(p0) >= 3
    for k in p0:
        np.testing.assert_array_equal(p0[k], p1[k])


def _trace_worker(rank, world, port, q, order):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port), HETU_USE_CONFIG='0', HETU_COMM_TRACE='1', HETU_GRAD_ORDER=order)
    import hetu_61a7_amd as ht
    rng = np.random.RandomState(3)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    h = x
    dims = [64, 256, 256, 256, 256, 8]
    for i in range(len(dims) - 1):
        W = ht.Variable(name='w%d' % i, value=(rng.randn(dims[i], dims[i + 1]) * 0.1).astype(np.float32))
        h = ht.matmul_op(h, W)
        if i < len(dims) - 2:
            h = ht.relu_op(h)
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(h, y_), [0])
    train = ht.optim.SGDOptimizer(0.01).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), bucket_mb=0.25)
    X = rng.randn(64, 64).astype(np.float32)
    Y = np.eye(8, dtype=np.float32)[rng.randint(0, 8, 64)]
    for _ in range(2):
        ex.run('train', feed_dict={x: X, y_: Y})
    q.put((rank, train.comm_trace()))
    from hetu_61a7_amd.parallel import comm
    comm.destroy()


@pytest.mark.parametrize('order', ['forward', 'reverse'])
def test_buckets_launch_before_backward_ends(order):
    """Overlap of the bucketed all-reduce with the backward pass:
    every bucket but the last is launched while gradients are still being
    produced, i.e. before the optimizer step that closes the backward."""
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_trace_worker, args=(r, 2, port, q, order)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, tr in res:
        assert len(tr) >= 3, tr
        early = [b for b in tr if b['launch_host_ms'] < 0]
        assert len(early) >= len(tr) - 1, tr


def _forced_dp_worker(port, X, Y, q):
    os.environ.update(RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      HETU_USE_CONFIG='0', HETU_FORCE_DP='1')
    losses, params, info = _mlp_losses(X, Y, 0.1, 5, dp=True, bucket_mb=0.001)
    from hetu_61a7_amd.parallel import comm
    backend = comm.world().backend if comm.world() is not None else None
    comm.destroy()
    q.put((losses, params, info, backend))


def test_forced_single_rank_dp_matches_baseline():
    """HETU_FORCE_DP=1 runs the bucketed all-reduce path with one rank (the one-GPU
    rehearsal of the multi-GPU path, tests/test_rccl_gpu.py): same losses and weights
    as the plain single-process run."""
    rng = np.random.RandomState(3)
    X = rng.randn(16, 20).astype(np.float32)
    Y = np.eye(4, dtype=np.float32)[rng.randint(0, 4, 16)]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_forced_dp_worker, args=(_free_port(), X, Y, q))
    p.start()
    losses, params, info, backend = q.get(timeout=120)
    p.join(60)
    assert p.exitcode == 0
    assert backend == 'gloo' and info['buckets'] >= 2, (backend, info)
    base, bparams, _ = _mlp_losses(X, Y, 0.1, 5)
    np.testing.assert_allclose(losses, base, rtol=1e-5, atol=1e-6)
    for k in bparams:
        np.testing.assert_allclose(params[k], bparams[k], rtol=1e-5, atol=1e-6)
