"""End-to-end model steps on the GPU (native HIP kernels) vs the CPU backend."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht

pytestmark = pytest.mark.gpu


def _logreg(ctx, X, Y, steps=10):
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W = ht.init.zeros((784, 10), name='W')
    b = ht.init.zeros((10,), name='b')
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.linear_op(x, W, b), y_), [0])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ctx)
    return [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(steps)]


def test_logreg_gpu_matches_cpu():
    rng = np.random.RandomState(0)
    X = rng.randn(128, 784).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 128)]
    a = _logreg(ht.cpu(0), X, Y)
    b = _logreg(ht.gpu(0), X, Y)
    np.testing.assert_allclose(a, b, rtol=1e-4)


def test_resnet50_bf16_step():
    from hetu_61a7_amd.models import resnet50_imagenet
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    loss, logits = resnet50_imagenet(x, y_, 1000)
    train = ht.optim.MomentumOptimizer(0.01, 0.9).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16')
    rng = np.random.RandomState(0)
    X = rng.randn(8, 3, 224, 224).astype(np.float32)
    Y = np.eye(1000, dtype=np.float32)[rng.randint(0, 1000, 8)]
    ls = [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(5)]
    assert np.isfinite(ls).all()
    # random init over 1000 classes: the first loss sits near ln(1000) = 6.9
    assert 4.0 < ls[0] < 10.0, ls
    assert min(ls[1:]) < ls[0], ls     # memorising one fixed batch


def test_resnet50_bf16_forward_matches_fp32():
    """Same weights, same batch: the bf16 mixed-precision forward (fused BN
    tails, MFMA convs, wide-channel BN statistics) tracks the fp32 one."""
    from hetu_61a7_amd.models import resnet50_imagenet
    from hetu_61a7_amd.ops import node as _node
    rng = np.random.RandomState(4)
    X = rng.randn(4, 3, 224, 224).astype(np.float32)
    Y = np.eye(1000, dtype=np.float32)[rng.randint(0, 1000, 4)]
    out = []
    for mp in (None, 'bf16'):
        _node.G_NODE_ID = 0
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        loss, logits = resnet50_imagenet(x, y_, 1000)
        train = ht.optim.MomentumOptimizer(0.0, 0.0).minimize(loss)
        ex = ht.Executor({'train': [loss, logits, train]}, ctx=ht.gpu(0), seed=11, mixed_precision=mp)
        l, lg, _ = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)
        out.append((float(np.asarray(l).reshape(-1)[0]), np.asarray(lg, dtype=np.float32)))
    (l32, g32), (l16, g16) = out
    assert abs(l16 - l32) < 0.05 * abs(l32), (l32, l16)
    assert np.abs(g16 - g32).max() < 0.25 * np.abs(g32).max() + 0.1


def test_resnet_cifar_gpu_vs_cpu_fp32():
    from hetu_61a7_amd.models.resnet import resnet_cifar
    rng = np.random.RandomState(1)
    X = rng.randn(8, 3, 32, 32).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 8)]
    res = []
    from hetu_61a7_amd.ops import node as _node
    for ctx in (ht.cpu(0), ht.gpu(0)):
        _node.G_NODE_ID = 0  # identical node ids -> identical seed+id initialisation
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        loss, _ = resnet_cifar(x, y_, 18, 10)
        train = ht.optim.SGDOptimizer(0.01).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ctx, seed=7)
        res.append([float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(3)])
    np.testing.assert_allclose(res[0], res[1], rtol=2e-3, atol=2e-3)


def test_hipgraph_mlp_matches_eager():
    rng = np.random.RandomState(2)
    X = rng.randn(64, 3072).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 64)]
    out = []
    from hetu_61a7_amd.ops import node as _node
    for g in (False, True):
        _node.G_NODE_ID = 0
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        from hetu_61a7_amd.models import mlp
        loss, _ = mlp(x, y_)
        train = ht.optim.AdamOptimizer(1e-3).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, use_hipgraph=g)
        out.append([float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(8)])
    np.testing.assert_allclose(out[0], out[1], rtol=1e-4, atol=1e-5)


def test_hipgraph_recaptures_when_feed_shape_changes():
    """a captured step fed a batch of another shape must not replay the stale graph: it runs
    eagerly, warms up and captures again -- losses equal the eager executor's throughout"""
    rng = np.random.RandomState(4)
    batches = [rng.randn(b, 784).astype(np.float32) for b in (32,) * 6 + (16,) * 6 + (32,) * 2]
    labels = [np.eye(10, dtype=np.float32)[rng.randint(0, 10, len(x))] for x in batches]
    out = []
    from hetu_61a7_amd.ops import node as _node
    for g in (False, True):
        _node.G_NODE_ID = 0
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        W = ht.init.xavier_normal((784, 10), name='W')
        loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(x, W), y_), [0])
        train = ht.optim.SGDOptimizer(0.1).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, use_hipgraph=g)
        out.append([float(np.asarray(ex.run('train', feed_dict={x: xb, y_: yb}, convert_to_numpy_ret_vals=True)[0])
                          .reshape(-1)[0]) for xb, yb in zip(batches, labels)])
    np.testing.assert_allclose(out[0], out[1], rtol=1e-4, atol=1e-5)


def test_hipgraph_replays_dropout_steps_like_eager():
    """dropout seeds are replay-safe (kernels/rng.py: fixed host seed per op
    and call, a device step counter advanced by a captured kernel), so a step with dropout
    is captured and replayed -- and draws exactly the eager executor's masks every step"""
    rng = np.random.RandomState(5)
    X = rng.randn(64, 784).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 64)]
    out, runners = [], []
    from hetu_61a7_amd.ops import node as _node
    for g in (False, True):
        _node.G_NODE_ID = 0
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        W = ht.init.xavier_normal((784, 10), name='Wd')
        h = ht.dropout_op(x, 0.8)
        loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, W), y_), [0])
        train = ht.optim.SGDOptimizer(0.1).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, use_hipgraph=g)
        out.append([float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0])
                          .reshape(-1)[0]) for _ in range(8)])
        runners.append(ex.subexecutor['train'].graph)
    runner = runners[1]
    assert runner.graph is not None and not getattr(runner, 'eager_only', False) and runner.random_ops
    assert np.isfinite(out[1]).all()
    assert len(set(round(v, 6) for v in out[1][4:])) > 1      # fresh masks (and updates) every replay
    np.testing.assert_allclose(out[0], out[1], rtol=1e-5, atol=1e-6)


def test_hipgraph_bert_with_dropout_matches_eager():
    """a BERT pretraining step (hidden / attention dropout in the fused LayerNorm,
    attention and GEMM-epilogue kernels) replays under hipGraph with the eager losses"""
    out = []
    for g in (False, True):
        out.append(_tiny_bert_losses(ht.gpu(0), mp='bf16', steps=6, hipgraph=g, dropout=0.1))
    assert np.isfinite(out[1]).all()
    np.testing.assert_allclose(out[0], out[1], rtol=2e-3, atol=2e-3)


def _tiny_bert_losses(ctx, mp=None, steps=4, hipgraph=False, dropout=0.0):
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    _node.G_NODE_ID = 0
    cfg = BertConfig(vocab_size=1200, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, batch_size=4, seq_len=16, max_position_embeddings=16,
                     hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-3)
    ex = ht.Executor({'train': [loss, train]}, ctx=ctx, seed=5, mixed_precision=mp, use_hipgraph=hipgraph)
    fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
    return [float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
            for _ in range(steps)]


def test_tiny_bert_gpu_matches_cpu():
    a = _tiny_bert_losses(ht.cpu(0))
    b = _tiny_bert_losses(ht.gpu(0))
    np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-3)
    c = _tiny_bert_losses(ht.gpu(0), mp='bf16', steps=6)
    assert np.isfinite(c).all() and c[-1] < c[0]


def test_moe_top_bf16_step():
    """Reference test_moe_top network in bf16 (4 experts, top-2): finite, and the
    MoE layer itself learns a regression target."""
    from hetu_61a7_amd.models.moe import moe_top, moe_random_batch
    from hetu_61a7_amd.layers.moe import TopKGate, Expert, MoELayer
    B, T, d = 2, 64, 128
    x, y_ = ht.Variable(name='x', trainable=False), ht.Variable(name='y_', trainable=False)
    loss, y = moe_top(x, y_, B, T, d, 256, 4, top=2)
    train = ht.optim.SGDOptimizer(0.5).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=3)
    X, Y = moe_random_batch(B, T, d)
    ls = [float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
          for _ in range(3)]
    assert np.isfinite(ls).all(), ls
    x2 = ht.Variable(name='x2', trainable=False)
    experts = [Expert(d, 256, activation='relu', name='expert_r%d' % i) for i in range(4)]
    yy, l_aux = MoELayer(TopKGate(d, B * T, 4, k=2, capacity_factor=2.0), experts, B * T, d)(x2)
    loss2 = ht.add_op(ht.reduce_mean_op(ht.mul_op(yy, yy), [0, 1]), ht.mul_byconst_op(l_aux, 0.01))
    train2 = ht.optim.SGDOptimizer(0.1).minimize(loss2)
    ex2 = ht.Executor({'train': [loss2, train2]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=3)
    X2 = X.reshape(B * T, d)
    l2 = [float(np.asarray(ex2.run('train', feed_dict={x2: X2}, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
          for _ in range(8)]
    assert np.isfinite(l2).all() and l2[-1] < l2[0], l2


@pytest.mark.parametrize('gate', ['topk', 'dts'])
def test_moe_expert_gradient_mask_epilogue_matches_two_pass(gate, monkeypatch):
    """The expert's ReLU + dropout backward masked inside the data-gradient GEMM
    (MatMulReluMaskOp) trains like the plain GEMM + relu_grad_c pair: same losses over
    a few SGD steps (bf16 rounding of the intermediate only)."""
    from hetu_61a7_amd.models.moe import moe_top, moe_random_batch
    from hetu_61a7_amd.ops import linalg, node as _node
    B, T, d = 2, 128, 256
    X, Y = moe_random_batch(B, T, d)
    res = {}
    # identical weights (initializer seeds follow node ids) and dropout seeds in both builds
    start = _node.G_NODE_ID
    for fused in (True, False):
        monkeypatch.setattr(linalg, '_GMASK_EPI', fused)
        _node.G_NODE_ID = start      # dropout seeds follow node ids and the executor seed
        x, y_ = ht.Variable(name='x', trainable=False), ht.Variable(name='y_', trainable=False)
        loss, _ = moe_top(x, y_, B, T, d, 512, 2, top=2, gate=gate)
        train = ht.optim.SGDOptimizer(0.05).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=5)
        kinds = {type(n).__name__ for n in ex.subexecutor['train'].topo_order}
        assert ('MatMulReluMaskOp' in kinds) == fused, kinds
        res[fused] = [float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0])
                            .reshape(-1)[0]) for _ in range(4)]
    assert np.isfinite(res[True]).all(), res
    np.testing.assert_allclose(res[True], res[False], rtol=2e-2, atol=1e-3)


def test_bert_base_width_bf16_forward_matches_fp32():
    """BERT-base widths (hidden 768, 12 heads, FFN 3072, seq 128) with two layers:
    the bf16 forward (fused attention, fused LayerNorm tails, MFMA GEMMs) stays
    close to the fp32 forward on identical weights."""
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    cfg = BertConfig(num_hidden_layers=2, batch_size=4, seq_len=128, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    out = []
    for mp in (None, 'bf16'):
        _node.G_NODE_ID = 0
        feeds, loss, train = bert_pretrain_graph(cfg, lr=0.0)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=5, mixed_precision=mp)
        fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
        out.append(float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0]))
    assert np.isfinite(out).all(), out
    assert abs(out[1] - out[0]) < 0.02 * abs(out[0]), out


def test_moe_d2048_bf16_forward_matches_fp32():
    """The bench MoE shape class (d_model 2048, top-2, 4 experts): bf16 loss
    tracks fp32 on identical weights and batch."""
    from hetu_61a7_amd.models.moe import moe_top, moe_random_batch
    from hetu_61a7_amd.ops import node as _node
    B, T, d = 2, 256, 2048
    X, Y = moe_random_batch(B, T, d)
    out = []
    for mp in (None, 'bf16'):
        _node.G_NODE_ID = 0
        x, y_ = ht.Variable(name='x', trainable=False), ht.Variable(name='y_', trainable=False)
        loss, _ = moe_top(x, y_, B, T, d, 2048, 4, top=2)
        train = ht.optim.SGDOptimizer(0.0).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision=mp, seed=3)
        out.append(float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y},
                                           convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0]))
    assert np.isfinite(out).all(), out
    assert abs(out[1] - out[0]) < 0.03 * abs(out[0]) + 1e-3, out
