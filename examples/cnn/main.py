"""CNN / MLP / RNN training entry (reference examples/cnn/main.py): same CLI.

    python examples/cnn/main.py --model mlp --dataset cifar10 --gpu 0 --timing
    python -m torch.distributed.run --nproc-per-node 8 examples/cnn/main.py \
        --model resnet18 --dataset cifar10 --comm-mode allreduce

Datasets load from ``datasets/`` when present (MNIST pickle, CIFAR python
batches); otherwise synthetic data of the same shape is used (no network).
"""
import argparse
import logging
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models import cnn as M_cnn, resnet as M_resnet  # noqa: E402

logging.basicConfig(level=logging.INFO, format='%(asctime)s - %(levelname)s - %(message)s')
log = logging.getLogger('cnn')

MODELS = {'logreg': M_cnn.logreg, 'mlp': M_cnn.mlp, 'cnn_3_layers': M_cnn.cnn_3_layers, 'lenet': M_cnn.lenet,
          'alexnet': M_cnn.alexnet, 'vgg16': M_cnn.vgg16, 'vgg19': M_cnn.vgg19, 'rnn': M_cnn.rnn,
          'lstm': M_cnn.lstm, 'resnet18': M_resnet.resnet18, 'resnet34': M_resnet.resnet34}


def optimizer(name, lr):
    return {'sgd': lambda: ht.optim.SGDOptimizer(learning_rate=lr),
            'momentum': lambda: ht.optim.MomentumOptimizer(learning_rate=lr),
            'nesterov': lambda: ht.optim.MomentumOptimizer(learning_rate=lr, nesterov=True),
            'adagrad': lambda: ht.optim.AdaGradOptimizer(learning_rate=lr, initial_accumulator_value=0.1),
            'adam': lambda: ht.optim.AdamOptimizer(learning_rate=lr)}[name]()


def load(dataset, model, synthetic):
    if dataset == 'mnist':
        (tx, ty), (vx, vy), _ = ht.data.mnist(synthetic=synthetic)
        if model in ('lenet', 'cnn_3_layers'):
            tx, vx = tx.reshape(-1, 1, 28, 28), vx.reshape(-1, 1, 28, 28)
        return tx, ty, vx, vy
    ncls = 100 if dataset == 'cifar100' else 10
    tx, ty, vx, vy = ht.data.normalize_cifar(num_class=ncls, synthetic=synthetic)
    if model in ('mlp', 'logreg'):
        tx, vx = tx.reshape(tx.shape[0], -1), vx.reshape(vx.shape[0], -1)
    return tx, ty, vx, vy


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--model', required=True)
    p.add_argument('--dataset', required=True)
    p.add_argument('--batch-size', type=int, default=128)
    p.add_argument('--learning-rate', type=float, default=0.1)
    p.add_argument('--opt', default='sgd')
    p.add_argument('--num-epochs', type=int, default=10)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU')
    p.add_argument('--validate', action='store_true')
    p.add_argument('--timing', action='store_true')
    p.add_argument('--comm-mode', default=None)
    p.add_argument('--synthetic', action='store_true', help='force synthetic data')
    p.add_argument('--max-steps', type=int, default=0, help='stop each epoch after N steps (smoke runs)')
    a = p.parse_args(argv)
    model = MODELS[a.model.lower()]
    tx, ty, vx, vy = load(a.dataset.lower(), a.model.lower(), a.synthetic)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    if a.model.lower() == 'mlp' and a.dataset.lower() == 'mnist':
        loss, y = model(x, y_, in_dim=784)
    elif a.model.lower() in ('resnet18', 'resnet34', 'vgg16', 'vgg19', 'alexnet'):
        loss, y = model(x, y_, ty.shape[1]) if a.model.lower().startswith('resnet') else model(x, y_)
    else:
        loss, y = model(x, y_)
    train = optimizer(a.opt.lower(), a.learning_rate).minimize(loss)
    nodes = {'train': [loss, y, train], 'validate': [loss, y]}
    if a.comm_mode:
        ex = ht.Executor(nodes, comm_mode={'allreduce': 'AllReduce', 'ps': 'PS', 'hybrid': 'Hybrid'}[a.comm_mode.lower()])
        rank, world = ex.config.rank, ex.config.nrank
    else:
        ex = ht.Executor(nodes, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu))
        rank, world = 0, 1
    B = a.batch_size
    nb = tx.shape[0] // B
    for ep in range(a.num_epochs):
        t0 = time.time()
        losses, acc = [], []
        steps = nb if not a.max_steps else min(nb, a.max_steps)
        for i in range(steps):
            sl = slice(i * B, (i + 1) * B)
            lv, yv, _ = ex.run('train', feed_dict={x: tx[sl], y_: ty[sl]}, convert_to_numpy_ret_vals=True)
            losses.append(float(np.mean(lv)))
            acc.append(float(np.mean(np.argmax(yv, 1) == np.argmax(ty[sl], 1))))
        dt = time.time() - t0
        if rank == 0:
            log.info('epoch %d train loss %.4f acc %.4f%s', ep, np.mean(losses), np.mean(acc),
                     (' time %.3fs (%.1f samples/s)' % (dt, steps * B * world / dt)) if a.timing else '')
        if a.validate:
            vl, va = [], []
            for i in range(min(vx.shape[0] // B, steps)):
                sl = slice(i * B, (i + 1) * B)
                lv, yv = ex.run('validate', feed_dict={x: vx[sl], y_: vy[sl]}, convert_to_numpy_ret_vals=True)
                vl.append(float(np.mean(lv)))
                va.append(float(np.mean(np.argmax(yv, 1) == np.argmax(vy[sl], 1))))
            if rank == 0:
                log.info('epoch %d validate loss %.4f acc %.4f', ep, np.mean(vl), np.mean(va))
    return float(np.mean(losses))


if __name__ == '__main__':
    main()
