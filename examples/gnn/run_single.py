"""GCN training entry (reference examples/gnn/run_single.py; the GraphMix
sampling submodule is empty in the reference, so the graph is a synthetic
random graph of the requested size, normalised with self loops).

    python examples/gnn/run_single.py --nodes 20000 --feat 128 --hidden 128 --classes 16
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.gcn import gcn  # noqa: E402


def random_graph(n, avg_deg, seed=0):
    import scipy.sparse as sp
    rng = np.random.RandomState(seed)
    m = n * avg_deg
    a = sp.coo_matrix((np.ones(m, np.float32), (rng.randint(0, n, m), rng.randint(0, n, m))), shape=(n, n))
    a = ((a + a.T) > 0).astype(np.float32) + sp.eye(n, dtype=np.float32)
    d = np.asarray(a.sum(1)).reshape(-1)
    dinv = sp.diags(1.0 / np.sqrt(d))
    return (dinv @ a @ dinv).tocsr().astype(np.float32)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--nodes', type=int, default=20000)
    p.add_argument('--degree', type=int, default=10)
    p.add_argument('--feat', type=int, default=128)
    p.add_argument('--hidden', type=int, default=128)
    p.add_argument('--classes', type=int, default=16)
    p.add_argument('--epochs', type=int, default=20)
    p.add_argument('--lr', type=float, default=0.1)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU')
    a = p.parse_args(argv)
    A = random_graph(a.nodes, a.degree)
    rng = np.random.RandomState(1)
    X = rng.randn(a.nodes, a.feat).astype(np.float32)
    Y = np.eye(a.classes, dtype=np.float32)[rng.randint(0, a.classes, a.nodes)]
    x, y_ = ht.Variable(name='x', trainable=False), ht.Variable(name='y_', trainable=False)
    adj = ht.Variable(name='adj', trainable=False)
    loss, y = gcn(adj, x, y_, a.feat, hidden=a.hidden, num_classes=a.classes)
    train = ht.optim.SGDOptimizer(learning_rate=a.lr).minimize(loss)
    ex = ht.Executor({'train': [loss, y, train]}, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu))
    C = A.tocoo()
    sparse_adj = ht.sparse_array(C.data, (C.row, C.col), A.shape)
    for ep in range(a.epochs):
        t0 = time.time()
        lv, yv, _ = ex.run('train', feed_dict={x: X, y_: Y, adj: sparse_adj}, convert_to_numpy_ret_vals=True)
        acc = float(np.mean(np.argmax(yv, 1) == np.argmax(Y, 1)))
        print('epoch %d loss %.4f train acc %.4f time %.4fs' % (ep, float(np.mean(lv)), acc, time.time() - t0),
              flush=True)
    return float(np.mean(lv))


if __name__ == '__main__':
    main()
