"""Distributed GCN over the parameter server (reference examples/gnn/run_dist.py):
every worker trains on its own sampled subgraphs; the node-embedding table is
PS-held (sparse push/pull, optional HET cache), the GCN weights are PS-held
dense parameters (``comm_mode='PS'``).  ``run_dist_hybrid.py`` keeps the GCN
weights on RCCL all-reduce instead (Hybrid).

    python bin/heturun -s 1 -w 2 python examples/gnn/run_dist.py --num_epoch 2
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..'))
sys.path.insert(0, HERE)
import hetu_61a7_amd as ht  # noqa: E402
from gnn_model import sparse_model, SyntheticGraph, get_norm_adj  # noqa: E402


def train_main(args, comm_mode='PS'):
    rank = int(os.environ.get('RANK', '0'))
    nrank = int(os.environ.get('WORLD_SIZE', '1'))
    import torch
    gpu = torch.cuda.is_available() and not args.cpu
    ctx = ht.gpu(rank % args.num_local_worker) if gpu else ht.cpu(0)
    G = SyntheticGraph(nodes=args.nodes, int_feature=args.int_feature, idx_max=args.idx_max, classes=args.classes)
    [loss, y, train_op], [mask_, norm_adj_] = sparse_model(
        args.int_feature, args.hidden_size, G.idx_max, args.hidden_size, G.classes, args.learning_rate)
    rng = np.random.RandomState(100 + rank)
    graph = G.sample(args.batch_size, rng)
    ht.GNNDataLoaderOp.step(graph)
    ht.GNNDataLoaderOp.step(graph)
    ex = ht.Executor([loss, y, train_op], ctx=ctx, comm_mode=comm_mode, use_sparse_pull=False,
                     cstable_policy=args.cache)
    nbatches = max(args.nodes // (args.batch_size * nrank), 1) if args.steps <= 0 else args.steps
    accs = []
    for epoch in range(args.num_epoch):
        t0 = time.time()
        correct = total = 0
        for _ in range(nbatches):
            graph_nxt = G.sample(args.batch_size, rng)
            ht.GNNDataLoaderOp.step(graph_nxt)          # sampled now, trained on next step
            lv, yv, _ = ex.run(feed_dict={norm_adj_: get_norm_adj(graph, ctx), mask_: graph.train_mask},
                               convert_to_numpy_ret_vals=True)
            pred = np.asarray(yv).argmax(1)
            correct += int(np.sum((pred == graph.label) * graph.train_mask))
            total += int(graph.train_mask.sum())
            graph = graph_nxt
        accs.append(correct / max(total, 1))
        print('rank %d epoch %d loss %.4f train acc %.4f time %.3fs' %
              (rank, epoch, float(np.mean(lv)), accs[-1], time.time() - t0), flush=True)
    return accs


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--num_epoch', type=int, default=10)
    p.add_argument('--hidden_size', type=int, default=64)
    p.add_argument('--learning_rate', type=float, default=0.5)
    p.add_argument('--batch_size', type=int, default=256, help='seed nodes per sampled subgraph')
    p.add_argument('--steps', type=int, default=0, help='subgraphs per epoch (0: nodes / (batch * workers))')
    p.add_argument('--nodes', type=int, default=20000)
    p.add_argument('--int_feature', type=int, default=4)
    p.add_argument('--idx_max', type=int, default=5000)
    p.add_argument('--classes', type=int, default=8)
    p.add_argument('--cache', default=None, help='HET cache policy: lru | lfu | lfuopt')
    p.add_argument('--num_local_worker', type=int, default=8)
    p.add_argument('--cpu', action='store_true')
    return p.parse_args(argv)


if __name__ == '__main__':
    train_main(parse())
