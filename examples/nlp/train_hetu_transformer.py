"""Encoder-decoder Transformer training entry (reference
examples/nlp/train_hetu_transformer.py + hparams.py: IWSLT de-en, d_model 512,
6 blocks, 8 heads, maxlen 100, label smoothing 0.1).

    python examples/nlp/train_hetu_transformer.py --steps 100
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        examples/nlp/train_hetu_transformer.py --dp

IWSLT is not downloadable here: a synthetic padded batch of the same shape is
used (``models.transformer.synthetic_batch``).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.transformer import Transformer, TransformerConfig, synthetic_batch  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--batch_size', type=int, default=32)
    p.add_argument('--lr', type=float, default=3e-4)
    p.add_argument('--vocab_size', type=int, default=32000)
    p.add_argument('--d_model', type=int, default=512)
    p.add_argument('--d_ff', type=int, default=2048)
    p.add_argument('--num_blocks', type=int, default=6)
    p.add_argument('--num_heads', type=int, default=8)
    p.add_argument('--maxlen1', type=int, default=100)
    p.add_argument('--maxlen2', type=int, default=100)
    p.add_argument('--dropout_rate', type=float, default=0.3)
    p.add_argument('--smoothing', type=float, default=0.1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU')
    p.add_argument('--dp', action='store_true', help='RCCL data parallel over all launched ranks')
    p.add_argument('--fp32', action='store_true', help='fp32 compute (default bf16 on GPU)')
    a = p.parse_args(argv)
    hp = TransformerConfig(a.vocab_size, a.d_model, a.d_ff, a.num_blocks, a.num_heads, a.maxlen1, a.maxlen2,
                           a.dropout_rate, a.smoothing, a.batch_size)
    names = ('xs', 'src_mask', 'ys', 'tgt_mask', 'labels')
    ph = {n: ht.Variable(name=n, trainable=False) for n in names}
    loss, _ = Transformer(hp).train(*(ph[n] for n in names))
    train = ht.optim.AdamOptimizer(a.lr, 0.9, 0.98, 1e-8).minimize(loss)
    kw = dict(seed=123)
    if a.gpu >= 0 and not a.fp32:
        kw['mixed_precision'] = 'bf16'
    if a.dp:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu), **kw)
    b = synthetic_batch(hp, seed=getattr(ex.config, 'rank', 0))
    feed = {ph[n]: b[n] for n in names}
    t0, losses = time.time(), []
    for s in range(a.steps):
        lv = ex.run('train', feed_dict=feed, convert_to_numpy_ret_vals=True)[0]
        losses.append(float(np.mean(lv)))
        if s % 10 == 0 or s == a.steps - 1:
            print('step %d loss %.4f' % (s, losses[-1]), flush=True)
    dt = time.time() - t0
    print('%.1f sentences/s' % (a.steps * a.batch_size / dt))
    return losses


if __name__ == '__main__':
    main()
