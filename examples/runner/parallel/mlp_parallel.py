"""Parallel-equivalence MLP (reference examples/runner/parallel/test_mlp_base.py,
test_mlp_pp.py, test_mlp_mp.py, test_mlp_mp_pp.py, simple_pipeline_mlp.py).

One script, the layout chosen by ``--mode``:

    base   one process, the whole MLP                       (heturun -w 1)
    pp     one pipeline stage per process, GPipe or 1F1B    (heturun -w N, --schedule)
    mp     the middle layer split over all processes with ``ht.dispatch``
           (--split left | right | middle)                    (heturun -w 2 / 4)
    dp_pp  pipeline stages each replicated over R ranks     (heturun -w S*R, --replicas R)

Every mode trains from the same fixed weights and batch and saves its per-step
losses to ``results/<mode>[_<split>].npy`` (rank holding the loss); with
``validate_results.py`` every layout must reproduce ``results/base.npy``.  The
reference could not run its context-annotated PP/MP examples (no dispatch
lowering pass); here they lower to RCCL (GPU) / gloo (CPU)
collectives and send/recv.  Synthetic MNIST-shaped data.

    python bin/heturun -w 1 python examples/runner/parallel/mlp_parallel.py --mode base
    python bin/heturun -w 4 python examples/runner/parallel/mlp_parallel.py --mode pp --schedule pipedream_flush
    python bin/heturun -w 2 python examples/runner/parallel/mlp_parallel.py --mode mp --split middle
    python examples/runner/parallel/validate_results.py
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402

SPLITS = {'left': ((2, 1), (1, 1)), 'right': ((1, 1), (1, 2)), 'middle': ((1, 2), (2, 1))}
DIMS = [784, 256, 256, 256, 10]


def weights():
    rng = np.random.RandomState(42)
    return [(rng.randn(a, b) * (2.0 / a) ** 0.5).astype(np.float32) for a, b in zip(DIMS[:-1], DIMS[1:])]


def batch(n):
    rng = np.random.RandomState(7)
    lab = rng.randint(0, 10, n)
    centers = np.random.RandomState(0).randn(10, 784).astype(np.float32)
    return centers[lab] + rng.randn(n, 784).astype(np.float32), np.eye(10, dtype=np.float32)[lab]


def dev(a, i):
    return ht.cpu(0) if a.cpu and a.mode == 'base' else ht.gpu(i)


def build(a, world):
    ws = weights()
    nl = len(ws)
    x = y_ = None

    def layer(h, i):
        W = ht.Variable(name='w%d' % i, value=ws[i])
        if i == 1:      # the layer the mp mode splits: no bias (a split bias would
            h = ht.matmul_op(h, W)          # need its own dispatch), in every mode
        else:
            b = ht.Variable(name='b%d' % i, value=np.zeros(ws[i].shape[1], np.float32))
            h = ht.linear_op(h, W, b)
        return ht.relu_op(h) if i < nl - 1 else h

    if a.mode in ('pp', 'dp_pp'):
        rep = a.replicas if a.mode == 'dp_pp' else 1
        S = world // rep
        per = [list(range(nl))[s * nl // S:(s + 1) * nl // S] for s in range(S)]
        h = None
        for s in range(S):
            ctx = [ht.gpu(s * rep + r) for r in range(rep)] if rep > 1 else ht.gpu(s)
            with ht.context(ctx):
                if s == 0:
                    x = ht.Variable(name='x', trainable=False)
                    h = x
                for i in per[s]:
                    h = layer(h, i)
                if s == S - 1:
                    y_ = ht.Variable(name='y_', trainable=False)
                    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(h, y_), [0])
                    train = ht.optim.SGDOptimizer(a.lr).minimize(loss)
        return x, y_, loss, train
    with ht.context(dev(a, 0)):
        x = ht.Variable(name='x', trainable=False)
        h = layer(x, 0)
    if a.mode == 'mp':
        with ht.context(tuple(ht.gpu(i) for i in range(world))):
            pa, pb = SPLITS[a.split]
            W = ht.Variable(name='w1', value=ws[1])
            h = ht.relu_op(ht.matmul_op(ht.dispatch(h, pa), ht.dispatch(W, pb)))
        last = ht.gpu(min(1, world - 1))
    else:
        with ht.context(dev(a, 0)):
            h = layer(h, 1)
        last = dev(a, 0)
    with ht.context(last):
        if a.mode == 'mp':
            h = ht.dispatch(h, (1, 1))
        for i in range(2, nl):
            h = layer(h, i)
        y_ = ht.Variable(name='y_', trainable=False)
        loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(h, y_), [0])
        train = ht.optim.SGDOptimizer(a.lr).minimize(loss)
    return x, y_, loss, train


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--mode', default='base', choices=['base', 'pp', 'mp', 'dp_pp'])
    p.add_argument('--split', default='middle', choices=sorted(SPLITS))
    p.add_argument('--schedule', default='gpipe', choices=['gpipe', 'pipedream', 'pipedream_flush', 'hetpipe'],
                   help='hetpipe: 1F1B with each stage\'s weights synced through the PS (heturun -s 1)')
    p.add_argument('--micro-batches', type=int, default=4)
    p.add_argument('--replicas', type=int, default=2)
    p.add_argument('--batch-size', type=int, default=64)
    p.add_argument('--steps', type=int, default=5)
    p.add_argument('--lr', type=float, default=0.05)
    p.add_argument('--cpu', action='store_true', help='base mode on the CPU backend')
    p.add_argument('--out', default=os.path.join(os.path.dirname(os.path.abspath(__file__)), 'results'))
    a = p.parse_args(argv)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    x, y_, loss, train = build(a, world)
    X, Y = batch(a.batch_size)
    losses = []
    if a.mode in ('pp', 'dp_pp'):
        # pipelines sum the micro-batch mean gradients (and the replicas' sums):
        # scale the lr so the update equals the full-batch mean-loss step
        M = a.micro_batches
        rep = a.replicas if a.mode == 'dp_pp' else 1
        train.optimizer.learning_rate = a.lr / (M * rep)
        # HetPipe in BSP mode (bsp=0): replicas push, barrier, pull -> same weights everywhere
        kw = {'comm_mode': 'PS', 'bsp': 0} if a.schedule == 'hetpipe' else {}
        ex = ht.Executor({'train': [loss, train]}, pipeline=a.schedule, **kw)
        r = ex.subexecutor['train'].replica
        n = a.batch_size // rep
        sl = slice(r * n, (r + 1) * n)
        for _ in range(a.steps):
            res = ex.run('train', feed_dict={x: X[sl], y_: Y[sl]}, batch_num=M, convert_to_numpy_ret_vals=True)
            mb = [float(np.mean(v[0])) for v in res if v is not None and v[0] is not None]
            if mb:
                losses.append(float(np.mean(mb)))
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=dev(a, 0) if a.mode == 'base' else None)
        for _ in range(a.steps):
            out = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]
            if out is not None:
                losses.append(float(np.mean(out)))
    if losses:
        os.makedirs(a.out, exist_ok=True)
        tag = a.mode + ('_' + a.split if a.mode == 'mp' else '') + \
            ('_' + a.schedule if a.mode in ('pp', 'dp_pp') else '')
        path = os.path.join(a.out, '%s_rank%d.npy' % (tag, rank) if a.mode != 'base' else 'base.npy')
        np.save(path, np.asarray(losses, np.float64))
        print('rank %d %s losses %s -> %s' % (rank, tag, ' '.join('%.5f' % v for v in losses), path), flush=True)
    if world > 1:
        from hetu_61a7_amd.parallel import comm
        comm.destroy()
    return losses


if __name__ == '__main__':
    main()
