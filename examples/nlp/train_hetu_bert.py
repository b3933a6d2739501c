"""BERT pretraining entry (reference examples/nlp/bert/train_hetu_bert{,_dp}.py):
same flags.  Single GPU, or data parallel under torch.distributed.run /
heturun (``--dp``), or planner-chosen DP x PP (``--galvatron``).

    python examples/nlp/train_hetu_bert.py --train_batch_size 64 --seq_length 128 -e 1
    python -m torch.distributed.run --nproc-per-node 8 examples/nlp/train_hetu_bert.py --dp

The pretraining corpus is not downloadable here: synthetic token ids of the
configured vocabulary are used (``models.bert.synthetic_bert_batch``).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--train_batch_size', type=int, default=64)
    p.add_argument('--dataset', default='synthetic')
    p.add_argument('--vocab_size', type=int, default=30522)
    p.add_argument('--hidden_size', type=int, default=768)
    p.add_argument('--num_hidden_layers', type=int, default=12)
    p.add_argument('--num_attention_heads', type=int, default=12)
    p.add_argument('--seq_length', type=int, default=128)
    p.add_argument('-e', '--epochs', type=int, default=1)
    p.add_argument('--lr', type=float, default=1e-5)
    p.add_argument('--adam_weight_decay', type=float, default=0.01)
    p.add_argument('--hidden_act', default='gelu')
    p.add_argument('--dropout_prob', type=float, default=0.1)
    p.add_argument('--steps', type=int, default=20, help='steps per epoch')
    p.add_argument('--gpu', type=int, default=0, help='-1 = CPU')
    p.add_argument('--dp', action='store_true', help='data parallel over all ranks (RCCL)')
    p.add_argument('--ps', action='store_true', help='data parallel through the parameter server '
                   '(DataParallel(aggregate="PS"); launch with heturun -s 1 -w N)')
    p.add_argument('--galvatron', action='store_true', help='DP x PP layout from the planner')
    p.add_argument('--fp32', action='store_true')
    a = p.parse_args(argv)
    cfg = BertConfig(vocab_size=a.vocab_size, hidden_size=a.hidden_size, num_hidden_layers=a.num_hidden_layers,
                     num_attention_heads=a.num_attention_heads, intermediate_size=4 * a.hidden_size,
                     hidden_act=a.hidden_act, hidden_dropout_prob=a.dropout_prob,
                     attention_probs_dropout_prob=a.dropout_prob, batch_size=a.train_batch_size,
                     seq_len=a.seq_length, max_position_embeddings=max(512, a.seq_length))
    opt = ht.optim.AdamWOptimizer(learning_rate=a.lr, weight_decay=a.adam_weight_decay)
    plan = None
    kw = dict(seed=1234)
    if a.gpu >= 0 and not a.fp32:
        kw['mixed_precision'] = 'bf16'
    if a.galvatron:
        from hetu_61a7_amd.parallel.galvatron import GalvatronPlanner, Hardware, bert_layers
        world = int(os.environ.get('WORLD_SIZE', '1'))
        plan = GalvatronPlanner(bert_layers(a.hidden_size, a.num_hidden_layers, a.seq_length, a.vocab_size),
                                hw=Hardware(gpus=world)).search(a.train_batch_size * world)
        print(plan.describe(), flush=True)
    feeds, loss, train = bert_pretrain_graph(cfg, optimizer=opt, plan=plan)
    if plan is not None and plan.pp > 1:
        ex = ht.Executor({'train': [loss, train]}, pipeline='gpipe', **kw)
    elif a.ps:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel(aggregate='PS'), **kw)
    elif a.dp or plan is not None:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0) if a.gpu < 0 else ht.gpu(a.gpu), **kw)
    rank = getattr(ex.config, 'rank', 0)
    for ep in range(a.epochs):
        t0 = time.time()
        ls = []
        for i in range(a.steps):
            fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1000 * ep + i + 97 * rank).items()}
            out = ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)
            if out and out[0] is not None:
                ls.append(float(np.asarray(out[0]).reshape(-1)[0]))
        dt = time.time() - t0
        if rank == 0:
            print('epoch %d loss %.4f  %.3f s  %.1f samples/s' % (ep, np.mean(ls) if ls else float('nan'), dt,
                                                                  a.steps * a.train_batch_size / dt), flush=True)
    return ls


if __name__ == '__main__':
    main()
