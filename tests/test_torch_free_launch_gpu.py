"""SURVEY §7.1 / VERDICT r5 next 3: the launch path asks torch nothing.  Kernel launches,
device allocations, stream switches and collectives read the framework's own state
(``_base.cur_stream`` / ``cur_device`` / ``gpu_available``, ``runtime.use_stream``); a
steady-state training step therefore makes zero calls to torch's stream / device
queries.  Counted by wrapping them after warm-up."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht

pytestmark = pytest.mark.gpu

_WATCH = ('current_stream', 'current_device', 'is_available', 'default_stream')


class _Count(object):
    def __init__(self):
        self.n = {}
        self.saved = []

    def __enter__(self):
        for name in _WATCH:
            f = getattr(torch.cuda, name)
            self.saved.append((torch.cuda, name, f))

            def w(*a, _f=f, _n=name, **k):
                self.n[_n] = self.n.get(_n, 0) + 1
                return _f(*a, **k)
            setattr(torch.cuda, name, w)
        raw = getattr(torch._C, '_cuda_getCurrentRawStream', None)
        if raw is not None:
            self.saved.append((torch._C, '_cuda_getCurrentRawStream', raw))

            def r(*a, _f=raw, **k):
                self.n['_cuda_getCurrentRawStream'] = self.n.get('_cuda_getCurrentRawStream', 0) + 1
                return _f(*a, **k)
            torch._C._cuda_getCurrentRawStream = r
        return self

    def __exit__(self, *exc):
        for mod, name, f in self.saved:
            setattr(mod, name, f)
        return False


def _steps(run, k=5):
    with _Count() as c:
        for _ in range(k):
            run()
    torch.cuda.synchronize()
    return c.n


@pytest.mark.parametrize('graph', [False, True])
def test_bert_step_asks_torch_nothing(graph):
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    cfg = BertConfig(vocab_size=1200, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, batch_size=4, seq_len=16, max_position_embeddings=16,
                     hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1)
    feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-3)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=5, mixed_precision='bf16', use_hipgraph=graph)
    fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
    for _ in range(6):           # past the warm-up and the hipGraph capture (steady state)
        ex.run('train', feed_dict=fd)
    torch.cuda.synchronize()
    n = _steps(lambda: ex.run('train', feed_dict=fd))
    assert n == {}, n


@pytest.mark.parametrize('graph', [False, True])
def test_cnn_step_asks_torch_nothing(graph):
    rng = np.random.RandomState(0)
    X = rng.randn(8, 3, 32, 32).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 8)]
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    w1 = ht.init.he_normal((16, 3, 3, 3), name='c1')
    h = ht.relu_op(ht.batch_normalization_op(ht.conv2d_op(x, w1, padding=1, stride=1),
                                             ht.init.ones((16,), name='s1'), ht.init.zeros((16,), name='b1')))
    h = ht.max_pool2d_op(h, 2, 2, 0, 2)
    h = ht.array_reshape_op(h, (8, -1))
    w2 = ht.init.xavier_normal((16 * 16 * 16, 10), name='fc')
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, w2), y_), [0])
    train = ht.optim.MomentumOptimizer(0.01, 0.9).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, mixed_precision='bf16', use_hipgraph=graph)
    for _ in range(6):
        ex.run('train', feed_dict={x: X, y_: Y})
    torch.cuda.synchronize()
    n = _steps(lambda: ex.run('train', feed_dict={x: X, y_: Y}))
    assert n == {}, n
