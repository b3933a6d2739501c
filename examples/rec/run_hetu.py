"""NCF training entry (reference examples/rec/run_hetu.py, hetu_ncf.py): same CLI.

    python examples/rec/run_hetu.py --val
    # PS / Hybrid (reference ps_ncf.sh / hybrid_ncf.sh): embedding tables on the server
    python bin/heturun -s 1 -w 4 python examples/rec/run_hetu.py --comm Hybrid --cache lfuopt --bound 3

MovieLens is not downloadable here: a MovieLens-shaped synthetic stream is used
(user / item ids, 1 positive + ``--num-ng`` negatives per interaction).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.ncf import neural_mf  # noqa: E402


def synthetic_movielens(n, num_users, num_items, num_ng, seed):
    """Interactions with a planted user/item affinity so the model can learn it."""
    rng = np.random.RandomState(seed)
    users = rng.randint(0, num_users, n)
    items = (users * 7 + rng.randint(0, 5, n)) % num_items           # positives near 7*u
    u = np.concatenate([users] + [users] * num_ng)
    i = np.concatenate([items] + [rng.randint(0, num_items, n) for _ in range(num_ng)])
    y = np.concatenate([np.ones(n)] + [np.zeros(n)] * num_ng).astype(np.float32)
    p = rng.permutation(len(u))
    return u[p].astype(np.float32), i[p].astype(np.float32), y[p].reshape(-1, 1)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--val', action='store_true')
    p.add_argument('--comm', default=None, help='None, AllReduce, PS, Hybrid')
    p.add_argument('--bsp', type=int, default=-1)
    p.add_argument('--cache', default=None, help='lru | lfu | lfuopt')
    p.add_argument('--bound', type=int, default=100)
    p.add_argument('--nepoch', type=int, default=3)
    p.add_argument('--batch-size', type=int, default=1024)
    p.add_argument('--num-users', type=int, default=6040)
    p.add_argument('--num-items', type=int, default=3706)
    p.add_argument('--num-ng', type=int, default=4)
    p.add_argument('--steps', type=int, default=20, help='steps per epoch')
    p.add_argument('--learning-rate', type=float, default=0.01)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU (local mode)')
    a = p.parse_args(argv)
    uid, iid, y_ = ht.Variable(name='user_input'), ht.Variable(name='item_input'), ht.Variable(name='y_')
    loss, y, train = neural_mf(uid, iid, y_, a.num_users, a.num_items, learning_rate=a.learning_rate)
    kw = {}
    if a.comm:
        kw.update(comm_mode={'allreduce': 'AllReduce', 'ps': 'PS', 'hybrid': 'Hybrid'}[a.comm.lower()], bsp=a.bsp)
        if a.cache:
            kw.update(cstable_policy=a.cache, cache_bound=a.bound)
    else:
        kw.update(ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu))
    ex = ht.Executor({'train': [loss, y, train], 'validate': [loss, y]}, **kw)
    B = a.batch_size
    U, I, Y = synthetic_movielens(B * a.steps // (a.num_ng + 1) + 1, a.num_users, a.num_items, a.num_ng,
                                  seed=3 + getattr(ex.config, 'rank', 0))
    t_all = time.time()
    for ep in range(a.nepoch):
        t0 = time.time()
        losses = []
        for s in range(a.steps):
            sl = slice(s * B, (s + 1) * B)
            lv, _, _ = ex.run('train', feed_dict={uid: U[sl], iid: I[sl], y_: Y[sl]}, convert_to_numpy_ret_vals=True)
            losses.append(float(np.mean(lv)))
        msg = 'epoch %d train_loss: %.4f, train_time: %.4f' % (ep, np.mean(losses), time.time() - t0)
        if a.val:
            _, yv = ex.run('validate', feed_dict={uid: U[:B], iid: I[:B], y_: Y[:B]}, convert_to_numpy_ret_vals=True)
            msg += ', val_auc: %.4f' % ht.metrics.roc_auc_score(Y[:B].reshape(-1), np.asarray(yv).reshape(-1))
        print(msg, flush=True)
    print('all time:', time.time() - t_all)
    if a.comm and a.comm.lower() in ('ps', 'hybrid'):
        from hetu_61a7_amd.ps import worker
        ex.config.ps_comm.BarrierWorker()
        worker.worker_finish()
    return float(np.mean(losses))


if __name__ == '__main__':
    main()
