"""MLP through heturun (reference examples/runner/run_mlp.py): one script for
local, AllReduce, PS and Hybrid training, the mode chosen by --comm-mode.

    python examples/runner/run_mlp.py --gpu -1                       # local CPU
    python bin/heturun -w 8 python examples/runner/run_mlp.py --comm-mode AllReduce
    python bin/heturun -w 4 -s 1 python examples/runner/run_mlp.py --comm-mode PS

Synthetic MNIST-shaped data (784 features, 10 classes).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--comm-mode', default=None, help='None, AllReduce, PS, Hybrid')
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--batch-size', type=int, default=128)
    p.add_argument('--learning-rate', type=float, default=0.1)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU (local mode)')
    a = p.parse_args(argv)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W1 = ht.init.xavier_normal((784, 256), name='W1')
    b1 = ht.init.zeros((256,), name='b1')
    W2 = ht.init.xavier_normal((256, 10), name='W2')
    h = ht.relu_op(ht.linear_op(x, W1, b1))
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, W2), y_), [0])
    train = ht.optim.SGDOptimizer(a.learning_rate).minimize(loss)
    if a.comm_mode:
        ex = ht.Executor({'train': [loss, train]}, comm_mode=a.comm_mode)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu))
    rng = np.random.RandomState(getattr(ex.config, 'rank', 0))
    centers = np.random.RandomState(0).randn(10, 784).astype(np.float32)
    losses = []
    for s in range(a.steps):
        lab = rng.randint(0, 10, a.batch_size)
        X = centers[lab] + rng.randn(a.batch_size, 784).astype(np.float32)
        Y = np.eye(10, dtype=np.float32)[lab]
        losses.append(float(np.mean(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0])))
    print('rank %s loss %.4f -> %.4f' % (getattr(ex.config, 'rank', 0), losses[0], losses[-1]), flush=True)
    if a.comm_mode and a.comm_mode.lower() in ('ps', 'hybrid'):
        from hetu_61a7_amd.ps import worker
        ex.config.ps_comm.BarrierWorker()
        worker.worker_finish()
    return losses


if __name__ == '__main__':
    main()
