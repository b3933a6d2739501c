"""Wide&Deep on Adult through heturun (reference examples/runner/run_wdl.py):
dataloader-fed inputs (12 deep columns, the wide one-hot block and the
labels, with 'train' / 'validate' splits), the model built inside a device
context whose string picks the mode:

    --config local  'gpu:0'                        one device
    --config lps    'cpu:0,gpu:0,...,gpu:N-1'      every parameter on the PS (cpu:0 = server)
    --config lhy    'cpu:0,gpu:0,...'  + dense 'gpu:0,...'   Hybrid: embeddings on the
                    PS, dense weights all-reduced over RCCL

    python examples/runner/run_wdl.py --config local --nepoch 2
    python bin/heturun -s 1 -w 2 python examples/runner/run_wdl.py --config lps --val
    python bin/heturun -s 1 -w 2 python examples/runner/run_wdl.py --config lhy --cache lfuopt

The Adult files are not available offline: the data is synthetic with the
Adult shape (8 categorical fields of 50 values, 4 continuous, an 809-wide
one-hot wide block), labels a noisy function of two fields.
"""
import argparse
import contextlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.ctr import wdl_adult  # noqa: E402


def synthetic_adult(n, seed=0):
    rng = np.random.RandomState(seed)
    cat = rng.randint(0, 50, (n, 8))
    cont = rng.randn(n, 4).astype(np.float32)
    wide = np.zeros((n, 809), np.float32)
    wide[np.arange(n)[:, None], (cat * 101 // 50)[:, :8] + np.arange(8) * 101] = 1.0
    logit = (cat[:, 0] % 2) * 2.0 - 1.0 + cont[:, 0] + 0.3 * rng.randn(n)
    y = np.eye(2, dtype=np.float32)[(logit > 0).astype(np.int64)]
    deep = [cat[:, i].astype(np.float32) for i in range(8)] + [cont[:, i] for i in range(4)]
    return deep, wide, y


def worker(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    import torch
    gpus = ['gpu:%d' % i for i in range(world)]
    # in a context string 'cpu:0' is the PS server, so local CPU runs go without one
    local_cpu = args.config == 'local' and not torch.cuda.is_available()
    ctx = {'local': None if local_cpu else gpus[0],
           'lps': ','.join(['cpu:0'] + gpus), 'lhy': ','.join(['cpu:0'] + gpus)}[args.config]
    batch_size = args.batch_size
    n_train, n_test = batch_size * args.batches, batch_size * 4
    deep_tr, wide_tr, y_tr = synthetic_adult(n_train, seed=1 + rank)
    deep_te, wide_te, y_te = synthetic_adult(n_test, seed=1000)
    with (ht.context(ctx) if ctx is not None else contextlib.nullcontext()):
        dense_input = [ht.dataloader_op([[deep_tr[i], batch_size, 'train'], [deep_te[i], batch_size, 'validate']])
                       for i in range(12)]
        sparse_input = ht.dataloader_op([[wide_tr, batch_size, 'train'], [wide_te, batch_size, 'validate']])
        y_ = ht.dataloader_op([[y_tr, batch_size, 'train'], [y_te, batch_size, 'validate']])
        if args.config == 'lhy':
            # dense weights in a GPU-only context -> all-reduced; embeddings stay on the PS
            with ht.context(','.join(gpus)):
                loss, prediction, y_, train_op = wdl_adult(dense_input, sparse_input, y_)
        else:
            loss, prediction, y_, train_op = wdl_adult(dense_input, sparse_input, y_)
        eval_nodes = {'train': [loss, prediction, y_, train_op]}
        if args.val:
            eval_nodes['validate'] = [loss, prediction, y_]
        executor = ht.Executor(eval_nodes, cstable_policy=args.cache, bsp=args.bsp, cache_bound=args.bound,
                               seed=123, **({'ctx': ht.cpu(0)} if local_cpu else {}))
    start = time.time()
    results = []
    for ep in range(args.nepoch):
        if ep == 5:
            start = time.time()
        t0 = time.time()
        losses, accs = [], []
        for _ in range(executor.get_batch_num('train')):
            lv, pv, yv, _ = executor.run('train', convert_to_numpy_ret_vals=True)
            losses.append(float(np.mean(lv)))
            accs.append(float(np.mean(np.argmax(yv, 1) == np.argmax(pv, 1))))
        msg = 'epoch %d train_loss: %.4f, train_acc: %.4f, train_time: %.4f' % (
            ep, np.mean(losses), np.mean(accs), time.time() - t0)
        if args.val:
            vl, va, vauc = [], [], []
            for _ in range(executor.get_batch_num('validate')):
                lv, pv, yv = executor.run('validate', convert_to_numpy_ret_vals=True)
                vl.append(float(np.mean(lv)))
                va.append(float(np.mean(np.argmax(yv, 1) == np.argmax(pv, 1))))
                vauc.append(ht.metrics.roc_auc_score(yv[:, 1], pv[:, 1] - pv[:, 0]))
            msg += ', test_loss: %.4f, test_acc: %.4f, test_auc: %.4f' % (np.mean(vl), np.mean(va), np.mean(vauc))
        results.append(float(np.mean(accs)))
        print(msg, flush=True)
    print('all time:', time.time() - start, flush=True)
    if args.config in ('lps', 'lhy'):
        from hetu_61a7_amd.ps import worker as psw
        executor.config.ps_comm.BarrierWorker()
        psw.worker_finish()
    return results


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--config', default='local', choices=['local', 'lps', 'lhy'])
    p.add_argument('--val', action='store_true')
    p.add_argument('--bsp', type=int, default=-1, help='bsp 0, asp -1, ssp > 0')
    p.add_argument('--cache', default=None, help='cache policy: lru | lfu | lfuopt')
    p.add_argument('--bound', type=int, default=100)
    p.add_argument('--nepoch', type=int, default=10)
    p.add_argument('--batch-size', type=int, default=128)
    p.add_argument('--batches', type=int, default=20, help='training batches per epoch (synthetic)')
    return worker(p.parse_args(argv))


if __name__ == '__main__':
    main()
