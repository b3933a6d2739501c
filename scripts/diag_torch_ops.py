"""List the aten ops (i.e. everything NOT launched through our own HIP kernels)
that one steady-state training step (ResNet-50 / BERT / MoE bench) issues, grouped by op + the
framework source line that called it.  Finds stray layout copies / casts.

    python scripts/diag_torch_ops.py [batch|0] [resnet50|bert|moe]
"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.utils._python_dispatch import TorchDispatchMode

import hetu_61a7_amd as ht
from hetu_61a7_amd.models import resnet50_imagenet

B = int(sys.argv[1]) if len(sys.argv) > 1 else 0
PKG = os.sep + 'hetu_61a7_amd' + os.sep
SKIP = {'aten.empty.memory_format', 'aten.empty_strided.default', 'aten.view.default', 'aten.t.default',
        'aten.permute.default', 'aten.reshape.default', 'aten._unsafe_view.default', 'aten.as_strided.default',
        'aten.slice.Tensor', 'aten.select.int', 'aten.detach.default', 'aten.expand.default',
        'aten.unsqueeze.default', 'aten.squeeze.dim', 'aten.transpose.int', 'aten.alias.default',
        'aten.empty_like.default', 'aten.new_empty.default', 'aten.split.Tensor', 'aten.narrow.default'}


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if PKG in fr.filename:
            return '%s:%d %s' % (fr.filename.split(PKG)[1], fr.lineno, fr.name)
    return '?'


def _desc(t):
    if isinstance(t, torch.Tensor):
        cl = t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)
        return '%s%s%s' % (str(t.dtype).replace('torch.', ''), list(t.shape), '/CL' if cl else '')
    return ''


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()
        self.example = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if name not in SKIP:
            key = (name, _site())
            self.rows[key] += 1
            if key not in self.example:
                ins = ' '.join(_desc(a) for a in args if isinstance(a, torch.Tensor))
                self.example[key] = ins + ' -> ' + (_desc(out) if isinstance(out, torch.Tensor) else type(out).__name__)
        return out


MODEL = sys.argv[2] if len(sys.argv) > 2 else 'resnet50'
if MODEL == 'resnet50':
    x = ht.Variable(name='x')
    y_ = ht.Variable(name='y_')
    loss, _ = resnet50_imagenet(x, y_, 1000)
    opt = ht.optim.MomentumOptimizer(learning_rate=0.1, momentum=0.9)
    train_op = opt.minimize(loss)
    ex = ht.Executor({'train': [loss, train_op]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=1234)
    B = B or 256
    X = torch.randn((B, 3, 224, 224), device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    Y = torch.nn.functional.one_hot(torch.randint(0, 1000, (B,), device='cuda'), 1000).bfloat16()

    def step():
        ex.run('train', feed_dict={x: X, y_: Y})
else:   # the bench.py step of another model (its default batch unless given)
    import bench
    sys.argv = ['bench.py', '--model', MODEL] + (['--batch', str(B)] if B else [])
    if MODEL == 'bert':
        from hetu_61a7_amd.models.bert import bert_bench as build
    else:
        from hetu_61a7_amd.models.moe import moe_top_bench as build
    step, *_ = build(bench.parse(), 1, 0, 0)
for _ in range(4):
    step()
torch.cuda.synchronize()
log = Log()
with log:
    step()
torch.cuda.synchronize()
print('aten ops in one steady-state step (count, op, call site, first example):')
for (name, site), n in sorted(log.rows.items(), key=lambda kv: -kv[1]):
    print('%4d  %-36s %-55s %s' % (n, name, site, log.example[(name, site)]))
