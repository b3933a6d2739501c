"""Distributed GCN, Hybrid mode (reference examples/gnn/run_dist_hybrid.py): the
node-embedding table stays on the parameter server (sparse push/pull, optional
HET cache) while the dense GCN weights are all-reduced over RCCL.

    python bin/heturun -s 1 -w 2 python examples/gnn/run_dist_hybrid.py --num_epoch 2
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from run_dist import train_main, parse  # noqa: E402

if __name__ == '__main__':
    train_main(parse(), comm_mode='Hybrid')
