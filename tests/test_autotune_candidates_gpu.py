"""Every hand-written candidate the autotuner may pick must compute the same product.

``kernels.autotune.choose`` times all candidates of a shape and keeps the fastest, so a
candidate that is wrong for one shape only shows up when the timing happens to favour it
(a training run that diverges on some boxes and not on others).  Here ``choose`` is wrapped:
for every key it first runs each hand-written candidate that answers, snapshots its result,
and compares it with the first one; then the normal choice proceeds.  A MoE step with the
dense-to-sparse gate (N = 2 gate GEMMs, split-K weight gradients, the masked expert GEMMs),
a Transformer/BERT-like step and a small CNN step exercise the GEMM entry points.
"""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht

pytestmark = pytest.mark.gpu


@pytest.fixture
def checked_choose(monkeypatch):
    from hetu_61a7_amd.kernels import autotune
    orig = autotune.choose
    monkeypatch.setattr(autotune, '_decisions', {})   # every shape is chosen afresh in this test
    bad, seen = [], set()

    def wrapped(key, candidates, mode='auto'):
        if key not in autotune._decisions and key not in seen and torch.cuda.is_available():
            seen.add(key)
            ref_name, ref = None, None
            for n, f in candidates.items():
                if not n.startswith('hip'):
                    continue
                try:
                    r = f()
                except Exception as e:      # noqa: BLE001 -- a raising candidate is a finding too
                    bad.append((str(key)[:120], n, 'raised %r' % (e,)))
                    continue
                if r is None or not torch.is_tensor(r):
                    continue
                r = r.detach().float().clone()
                if ref is None:
                    ref_name, ref = n, r
                    continue
                if r.shape != ref.shape:
                    bad.append((str(key)[:120], n, 'shape %s vs %s' % (tuple(r.shape), tuple(ref.shape))))
                    continue
                rel = float((r - ref).norm() / ref.norm().clamp_min(1e-12))
                if not np.isfinite(rel) or rel > 2e-2:
                    bad.append((str(key)[:120], n, 'rel %.3g vs %s' % (rel, ref_name)))
        return orig(key, candidates, mode)

    monkeypatch.setattr(autotune, 'choose', wrapped)
    yield bad, seen


def _run(ex, feed, n=2):
    out = []
    for _ in range(n):
        r = ex.run('train', feed_dict=feed, convert_to_numpy_ret_vals=True)
        out.append(float(np.asarray(r[0]).reshape(-1)[0]))
    return out


@pytest.mark.parametrize('gate', ['dts', 'topk'])
def test_moe_step_candidates_agree(checked_choose, gate):
    from hetu_61a7_amd.models.moe import moe_top, moe_random_batch
    bad, seen = checked_choose
    B, T, d = 8, 512, 1024
    X, Y = moe_random_batch(B, T, d)
    x, y_ = ht.Variable(name='x', trainable=False), ht.Variable(name='y_', trainable=False)
    loss, _ = moe_top(x, y_, B, T, d, 1024, 2, top=2, gate=gate)
    train = ht.optim.SGDOptimizer(0.125).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=7)
    ls = _run(ex, {x: X, y_: Y})
    assert np.isfinite(ls).all(), ls
    assert seen, 'no GEMM went through the autotuner'
    assert not bad, bad


def test_bert_step_candidates_agree(checked_choose):
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    bad, seen = checked_choose
    cfg = BertConfig(num_hidden_layers=2, batch_size=16, seq_len=128)
    feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-4)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=7)
    batch = synthetic_bert_batch(cfg)
    ls = _run(ex, {feeds[k]: v for k, v in batch.items()})
    assert np.isfinite(ls).all(), ls
    assert seen
    assert not bad, bad
