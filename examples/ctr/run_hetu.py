"""CTR training entry (reference examples/ctr/run_hetu.py): same CLI.

    python examples/ctr/run_hetu.py --model wdl_criteo --nepoch 2
    # PS / Hybrid with the HET cache (one server, N workers on this node):
    python bin/heturun -s 1 -w 4 python examples/ctr/run_hetu.py --model wdl_criteo \
        --comm Hybrid --cache lfuopt --bound 3

Criteo is not downloadable here: a Criteo-shaped synthetic stream is used
(``--rows`` embedding rows, Zipf-skewed ids; ``models.ctr.synthetic_criteo``).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models import ctr as M  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--model', required=True, help='wdl_criteo | dfm_criteo | dcn_criteo | dc_criteo | wdl_adult')
    p.add_argument('--val', action='store_true')
    p.add_argument('--comm', default=None, help='None, AllReduce, PS, Hybrid')
    p.add_argument('--bsp', type=int, default=-1, help='bsp 0, asp -1, ssp > 0')
    p.add_argument('--cache', default=None, help='lru | lfu | lfuopt')
    p.add_argument('--bound', type=int, default=100)
    p.add_argument('--nepoch', type=int, default=2)
    p.add_argument('--batch-size', type=int, default=128)
    p.add_argument('--rows', type=int, default=100000, help='embedding rows of the synthetic stream')
    p.add_argument('--steps', type=int, default=50, help='steps per epoch')
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU (local mode)')
    a = p.parse_args(argv)
    model = getattr(M, a.model)
    xd, xs, y_ = ht.Variable(name='dense_input'), ht.Variable(name='sparse_input'), ht.Variable(name='y_')
    loss, y, y_, train = model(xd, xs, y_, feature_dimension=a.rows) if 'criteo' in a.model else model(xd, xs, y_)
    kw = {}
    if a.comm:
        kw.update(comm_mode={'allreduce': 'AllReduce', 'ps': 'PS', 'hybrid': 'Hybrid'}[a.comm.lower()], bsp=a.bsp)
        if a.cache:
            kw.update(cstable_policy=a.cache, cache_bound=a.bound)
    else:
        kw.update(ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu))
    ex = ht.Executor({'train': [loss, y, y_, train], 'validate': [loss, y, y_]}, **kw)
    B = a.batch_size
    dense, sparse, labels = M.synthetic_criteo(B * a.steps, a.rows, seed=7 + getattr(ex.config, 'rank', 0))
    start = None
    for ep in range(a.nepoch):
        if ep == min(5, a.nepoch - 1):
            start = time.time()
        t0 = time.time()
        losses, accs = [], []
        for i in range(a.steps):
            sl = slice(i * B, (i + 1) * B)
            lv, yv, yt, _ = ex.run('train', feed_dict={xd: dense[sl], xs: sparse[sl], y_: labels[sl]},
                                   convert_to_numpy_ret_vals=True)
            losses.append(float(np.mean(lv)))
            accs.append(float(np.mean((yv > 0.5) == (yt > 0.5))))
        msg = 'epoch %d train_loss: %.4f, train_acc: %.4f, train_time: %.4f' % (ep, np.mean(losses), np.mean(accs),
                                                                                time.time() - t0)
        if a.val:
            yv, _, yt = ex.run('validate', feed_dict={xd: dense[:B], xs: sparse[:B], y_: labels[:B]},
                               convert_to_numpy_ret_vals=True)[1:] + [None]
            msg += ', val_auc: %.4f' % ht.metrics.roc_auc_score(labels[:B].reshape(-1), np.asarray(yv).reshape(-1))
        print(msg, flush=True)
    print('all time:', time.time() - start)
    if a.comm and a.comm.lower() in ('ps', 'hybrid'):
        from hetu_61a7_amd.ps import worker
        ex.config.ps_comm.BarrierWorker()
        worker.worker_finish()
    return float(np.mean(losses))


if __name__ == '__main__':
    main()
