"""GPU diagnostic: ResNet-50 first-step loss on GPU vs CPU for a tiny batch.

Usage: python scripts/diag_smoke.py [batch] [mp]   (mp: bf16 | none)
Prints the first three losses and the max |logit| per step.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import hetu_61a7_amd as ht
from hetu_61a7_amd.models import resnet50_imagenet

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
mp = sys.argv[2] if len(sys.argv) > 2 else 'bf16'
x = ht.Variable(name='x'); y_ = ht.Variable(name='y_')
loss, logits = resnet50_imagenet(x, y_, 1000)
train_op = ht.optim.MomentumOptimizer(0.01, 0.9).minimize(loss)
kw = {} if mp == 'none' else {'mixed_precision': mp}
ex = ht.Executor({'train': [loss, logits, train_op]}, ctx=ht.gpu(0), **kw)
rng = np.random.RandomState(0)
X = rng.randn(bs, 3, 224, 224).astype(np.float32)
Y = np.eye(1000, dtype=np.float32)[rng.randint(0, 1000, bs)]
for i in range(3):
    l, lg, _ = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)
    print('bs', bs, 'mp', mp, 'conv', os.environ.get('HETU_CONV', 'auto'), 'step', i,
          'loss', float(np.asarray(l).reshape(-1)[0]), 'max|logit|', float(np.abs(lg).max()), flush=True)
