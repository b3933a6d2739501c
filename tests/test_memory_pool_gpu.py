"""BFC allocator on the GPU: pinned-DRAM pool tensors and the process-wide
device allocator hook (HETU_ALLOCATOR=bfc) under a real training loop."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r'''
import json, sys
import numpy as np, torch
import hetu_61a7_amd as ht
from hetu_61a7_amd import memory_pool as MP
from hetu_61a7_amd.models import mlp
from hetu_61a7_amd.ops import node as _node
_node.G_NODE_ID = 0
rng = np.random.RandomState(2)
X = rng.randn(64, 3072).astype(np.float32)
Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 64)]
x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
loss, _ = mlp(x, y_)
train = ht.optim.AdamOptimizer(1e-3).minimize(loss)
ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3)
ls = [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(6)]
st = MP.device_stats(0) if MP.torch_bfc_enabled() else {}
print(json.dumps({'losses': ls, 'stats': st}))
'''


def _run(env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    r = subprocess.run([sys.executable, '-c', _SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_torch_bfc_allocator_training_matches_default():
    base = _run({})
    bfc = _run({'HETU_ALLOCATOR': 'bfc', 'HETU_BFC_REGION_MB': '256'})
    np.testing.assert_allclose(base['losses'], bfc['losses'], rtol=1e-5, atol=1e-6)
    st = bfc['stats']
    assert st['num_allocs'] > 0 and st['bytes_reserved'] >= 256 << 20
    assert st['peak_bytes_in_use'] >= st['bytes_in_use'] > 0


def test_pinned_pool_tensor_is_pinned_and_copies():
    from hetu_61a7_amd.ndarray import pinned_empty
    t = pinned_empty((1024, 256), torch.float32)
    t.copy_(torch.arange(1024 * 256, dtype=torch.float32).reshape(1024, 256))
    assert t.is_pinned()
    d = t.to('cuda', non_blocking=True)
    back = pinned_empty((1024, 256), torch.float32)
    back.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(back, t)
