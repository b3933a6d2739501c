"""GPU diagnostic: per-layer fp32 vs bf16 ResNet-50 training-mode forward.
Usage: python scripts/diag_layers.py [batch] [fused]   (fused: only loss/logits
requested, so every BN/ReLU/add fusion applies; HETU_FUSE=0 disables fusion)
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import hetu_61a7_amd as ht
from hetu_61a7_amd.models import resnet as R
from hetu_61a7_amd.ops import node as _node

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
fused = len(sys.argv) > 2 and sys.argv[2] == 'fused'
rng = np.random.RandomState(0)
X = rng.randn(bs, 3, 224, 224).astype(np.float32)
Y = np.eye(1000, dtype=np.float32)[rng.randint(0, 1000, bs)]
outs = {}
for mp in ('none', 'bf16'):
    _node.G_NODE_ID = 0
    rec = []
    orig = R.bn
    def bn_rec(x, c, name, relu=False, **kw):
        y = orig(x, c, name, relu=relu, **kw)
        rec.append((name, y))
        return y
    R.bn = bn_rec
    x = ht.Variable(name='x'); y_ = ht.Variable(name='y_')
    loss, logits = R.resnet50_imagenet(x, y_, 1000)
    R.bn = orig
    nodes = [n for _, n in rec]
    train = ht.optim.MomentumOptimizer(0.0, 0.0).minimize(loss)   # training-mode BN, no update
    ev = [loss, logits, train] + ([] if fused else nodes)
    kw = {} if mp == 'none' else {'mixed_precision': 'bf16'}
    ex = ht.Executor({'f': ev}, ctx=ht.gpu(0), seed=11, **kw)
    res = ex.run('f', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)
    names = ['loss', 'logits', 'train'] + ([nm for nm, _ in rec] if not fused else [])
    outs[mp] = {nm: (np.asarray(v, dtype=np.float32) if v is not None else None) for nm, v in zip(names, res)}
a, b = outs['none'], outs['bf16']
for k in a:
    if a[k] is None or b[k] is None:
        continue
    d = np.abs(a[k] - b[k]).max()
    s = np.abs(a[k]).max()
    print('%-20s shape %-22s max|fp32| %11.4g  max|diff| %11.4g  rel %9.3g' % (k, a[k].shape, s, d, d / max(s, 1e-12)), flush=True)
