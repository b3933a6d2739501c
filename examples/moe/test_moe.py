"""MoE benchmark entry (reference examples/moe/test_moe_{top,ktop1,hash,sam,base}.py).

    python examples/moe/test_moe.py --gate top --top 2
    python -m torch.distributed.run --nproc-per-node 8 examples/moe/test_moe.py --gate dts

One MoE layer (``--num_local_experts`` experts per rank, expert parallel over
all ranks through RCCL all-to-all), reduce-sum -> softmax -> NLL over tokens,
plus the balance loss; prints the average synced step time like the reference.
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.moe import moe_top  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--batch_size', type=int, default=16)
    p.add_argument('--num_tokens', type=int, default=1024)
    p.add_argument('--model_dim', type=int, default=2048)
    p.add_argument('--hidden_size', type=int, default=2048)
    p.add_argument('--num_local_experts', type=int, default=2)
    p.add_argument('--top', type=int, default=2)
    p.add_argument('--gate', default='top', help='top | ktop1 | hash | sam | base | dts')
    p.add_argument('--num_steps', type=int, default=30)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU')
    p.add_argument('--fp32', action='store_true')
    a = p.parse_args(argv)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    x = ht.Variable(name='x', trainable=False)
    y_ = ht.Variable(name='y_', trainable=False)
    h = ht.Variable(name='hash_ids', trainable=False) if a.gate == 'hash' else None
    gate = {'top': 'topk'}.get(a.gate, a.gate)
    loss, y = moe_top(x, y_, a.batch_size, a.num_tokens, a.model_dim, a.hidden_size, a.num_local_experts,
                      world, rank, top=a.top, gate=gate, hash_ids=h)
    train = ht.optim.SGDOptimizer(learning_rate=0.125).minimize(loss)
    kw = dict(seed=1234)
    if a.gpu >= 0 and not a.fp32:
        kw['mixed_precision'] = 'bf16'
    if world > 1:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(int(os.environ.get('LOCAL_RANK', '0'))),
                         comm_mode='AllReduce', **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu), **kw)
    rng = np.random.RandomState(rank)
    fd = {x: rng.normal(size=(a.batch_size, a.num_tokens, a.model_dim)).astype(np.float32),
          y_: np.zeros((a.batch_size,), np.float32)}
    if h is not None:
        E = a.num_local_experts * world
        fd[h] = (np.arange(a.batch_size * a.num_tokens) % E).astype(np.float32).reshape(-1, 1)
    times = []
    for i in range(a.num_steps):
        t0 = time.time()
        lv = ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]
        times.append(time.time() - t0)
        if rank == 0 and i % 10 == 0:
            print('Step %d  Train loss = %f' % (i, float(np.asarray(lv).reshape(-1)[0])), flush=True)
    tail = times[len(times) // 2:]
    if rank == 0:
        print('Average synced step_time=%s sec.' % (sum(tail) / len(tail)), flush=True)
    return times


if __name__ == '__main__':
    main()
