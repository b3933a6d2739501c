"""CPU-backend graph/autodiff/executor tests (reference test strategy: CPU-vs-numpy)."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht


def _data(n=64, d=784, c=10, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, d).astype(np.float32)
    Y = np.eye(c, dtype=np.float32)[rng.randint(0, c, n)]
    return X, Y


def test_logreg_matches_numpy_sgd():
    X, Y = _data()
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W = ht.init.zeros((784, 10), name='W')
    b = ht.init.zeros((10,), name='b')
    logits = ht.linear_op(x, W, b)
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(logits, y_), [0])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    Wn = np.zeros((784, 10), np.float32)
    bn = np.zeros((10,), np.float32)
    for _ in range(20):
        l, _ = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)
        z = X @ Wn + bn
        p = np.exp(z - z.max(1, keepdims=True))
        p /= p.sum(1, keepdims=True)
        ref = -(Y * np.log(p)).sum(1).mean()
        np.testing.assert_allclose(l, ref, rtol=1e-4)
        g = (p - Y) / X.shape[0]
        Wn -= 0.1 * X.T @ g
        bn -= 0.1 * g.sum(0)


def test_mlp_autodiff_matches_torch():
    X, Y = _data(32, 20, 5, 1)
    rng = np.random.RandomState(3)
    w1 = rng.randn(20, 16).astype(np.float32) * 0.3
    w2 = rng.randn(16, 5).astype(np.float32) * 0.3
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W1 = ht.Variable(name='w1', value=w1)
    W2 = ht.Variable(name='w2', value=w2)
    h = ht.relu_op(ht.matmul_op(x, W1))
    h2 = ht.tanh_op(h) * 2.0 + ht.sigmoid_op(h)
    logits = ht.matmul_op(h2, W2)
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(logits, y_), [0])
    gW1, gW2 = ht.gradients(loss, [W1, W2])
    ex = ht.Executor([loss, gW1, gW2], ctx=ht.cpu(0))
    l, g1, g2 = ex.run(feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)
    tw1 = torch.tensor(w1, requires_grad=True)
    tw2 = torch.tensor(w2, requires_grad=True)
    th = torch.relu(torch.tensor(X) @ tw1)
    th2 = torch.tanh(th) * 2 + torch.sigmoid(th)
    tl = torch.nn.functional.cross_entropy(th2 @ tw2, torch.tensor(Y.argmax(1)))
    tl.backward()
    np.testing.assert_allclose(l, tl.item(), rtol=1e-5)
    np.testing.assert_allclose(g1, tw1.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(g2, tw2.grad.numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('opt', ['sgd', 'momentum', 'nesterov', 'adagrad', 'adam', 'adamw', 'lamb'])
def test_optimizers_match_reference_rules(opt):
    rng = np.random.RandomState(5)
    w0 = rng.randn(8, 4).astype(np.float32)
    X = rng.randn(16, 8).astype(np.float32)
    x = ht.Variable(name='x')
    W = ht.Variable(name='w_%s' % opt, value=w0)
    loss = ht.reduce_mean_op(ht.reduce_sum_op(ht.matmul_op(x, W) * ht.matmul_op(x, W), [1]), [0])
    O = ht.optim
    o = {'sgd': O.SGDOptimizer(0.05), 'momentum': O.MomentumOptimizer(0.05, 0.9),
         'nesterov': O.MomentumOptimizer(0.05, 0.9, nesterov=True), 'adagrad': O.AdaGradOptimizer(0.05),
         'adam': O.AdamOptimizer(0.05), 'adamw': O.AdamWOptimizer(0.05, weight_decay=0.01),
         'lamb': O.LambOptimizer(0.05, weight_decay=0.01)}[opt]
    train = o.minimize(loss)
    ex = ht.Executor([loss, train], ctx=ht.cpu(0))
    w = w0.copy()
    m = np.zeros_like(w)
    v = np.zeros_like(w)
    for t in range(1, 6):
        ex.run(feed_dict={x: X})
        g = 2 * X.T @ (X @ w) / X.shape[0]
        if opt == 'sgd':
            w -= 0.05 * g
        elif opt == 'momentum':
            m = 0.9 * m - 0.05 * g
            w += m
        elif opt == 'nesterov':
            tt = 0.05 * g
            m = 0.9 * (m - tt)
            w += m - tt
        elif opt == 'adagrad':
            m += g * g
            w -= 0.05 * g / (np.sqrt(m) + 1e-7)
        else:
            m = 0.9 * m + 0.1 * g
            v = 0.999 * v + 0.001 * g * g
            u = (m / (1 - 0.9 ** t)) / (np.sqrt(v / (1 - 0.999 ** t)) + 1e-7)
            if opt == 'adam':
                w -= 0.05 * u
            elif opt == 'adamw':
                w -= 0.05 * (u + 0.01 * w)
            else:
                ratio = np.linalg.norm(w) / np.linalg.norm(u)
                w -= 0.05 * ratio * (u + 0.01 * w)
    got = ex.config.placeholder_to_arr_map[W].numpy()
    np.testing.assert_allclose(got, w, rtol=2e-4, atol=1e-5)


def test_checkpoint_roundtrip(tmp_path):
    import pickle
    X, Y = _data(16, 10, 3)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W = ht.init.random_normal((10, 3), name='ckW')
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(x, W), y_), [0])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    ex.run('train', feed_dict={x: X, y_: Y})
    ex.save(str(tmp_path), 'ck.pkl')
    with open(tmp_path / 'ck.pkl', 'rb') as f:
        st = pickle.load(f)
    assert set(st) == {'ckW'} and st['ckW'].dtype == np.float32
    before = st['ckW'].copy()
    ex.run('train', feed_dict={x: X, y_: Y})
    ex.load(str(tmp_path), 'ck.pkl')
    np.testing.assert_allclose(ex.config.placeholder_to_arr_map[W].numpy(), before)


def test_conv_bn_pool_graph_cpu():
    rng = np.random.RandomState(0)
    X = rng.randn(4, 3, 32, 32).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 4)]
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    from hetu_61a7_amd.models.resnet import resnet_cifar
    loss, logits = resnet_cifar(x, y_, 18, 10)
    train = ht.optim.MomentumOptimizer(0.05).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    ls = [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(6)]
    assert np.isfinite(ls).all()
    assert ls[-1] < ls[0]


def test_timer_log_and_chrome_trace(tmp_path):
    import json
    import hetu_61a7_amd as ht
    x = ht.Variable(name='x')
    W = ht.init.random_normal((8, 4), name='W')
    loss = ht.reduce_mean_op(ht.relu_op(ht.matmul_op(x, W)), [0, 1])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'default': [loss, train]}, ctx=ht.cpu(0), timing='cpu')
    for _ in range(3):
        ex.run(feed_dict={x: np.ones((5, 8), np.float32)})
    n = ex.export_chrome_trace(str(tmp_path / 't.json'))
    tr = json.load(open(tmp_path / 't.json'))['traceEvents']
    assert n == len(tr) > 0 and {'name', 'ph', 'ts', 'dur'} <= set(tr[0])
    assert any(e['cat'] == 'MatMulOp' for e in tr)
    by_type = ex.logOut(log_level='type')
    assert 'MatMulOp' in by_type or any('MatMul' in k for k in by_type)


def test_deterministic_flag_toggles_fixed_kernel_choice():
    from hetu_61a7_amd import kernels as K
    from hetu_61a7_amd.kernels import autotune
    import torch
    K.set_deterministic(True)
    try:
        assert K.deterministic() and torch.are_deterministic_algorithms_enabled()
        assert autotune.choose(('det-test',), {'hip': lambda: 1, 'hip_b': lambda: 2}) == 'hip'
    finally:
        K.set_deterministic(False)
    assert not K.deterministic() and not torch.are_deterministic_algorithms_enabled()


def test_gradient_select_flags_aliased_outputs():
    """A fused backward that returns one tensor in two slots (LayerNorm dx == ds
    without dropout) marks it shared, so no fused join overwrites it in place."""
    import torch
    from hetu_61a7_amd.ops.nn import BNGradSelectOp, _may_overwrite
    t, u = torch.ones(4, 4), torch.zeros(4, 4)
    sel = BNGradSelectOp.__new__(BNGradSelectOp)
    sel.index = 1
    v = sel.compute([(t, t, torch.ones(4), torch.ones(4))])
    assert v is t and getattr(t, 'hetu_shared', False)
    w = sel.compute([(torch.ones(2), u, torch.ones(4), torch.ones(4))])
    assert w is u and not getattr(u, 'hetu_shared', False)

    class _J:
        acc_inplace = True
    assert _may_overwrite(_J(), u) and not _may_overwrite(_J(), t)


def test_dp_buckets_small_at_the_end():
    """All-reduce buckets tile the flat gradient contiguously and in order; the
    last (exposed) bucket is the smallest, caps grow toward the front."""
    import types
    from hetu_61a7_amd.optimizer import OptimizerOp
    sizes = [300, 5000, 70, 2600, 900, 4096, 128, 1500, 2048, 64]
    class P(object):
        def __init__(self, name):
            self.name = name
    params = [P('p%d' % i) for i in range(len(sizes))]
    offs, o = {}, 0
    for p, n in zip(params, sizes):
        offs[p] = (o, n, (n,))
        o += n
    op = OptimizerOp.__new__(OptimizerOp)
    op.flat = types.SimpleNamespace(offsets=offs)
    op.bucket_bytes = 4 * 4096           # full cap 4096 elements, last bucket cap 512
    op.bucket_of = {}
    op.excluded_from_dp = lambda p: False
    op._make_buckets(params)
    bs = op.buckets
    assert bs[0].start == 0 and bs[-1].end == o
    assert all(a.end == b.start for a, b in zip(bs, bs[1:]))
    assert sum(b.total for b in bs) == len(params)
    assert bs[-1].end - bs[-1].start <= 512 or bs[-1].total == 1
    assert all(op.bucket_of[p].start <= offs[p][0] < op.bucket_of[p].end for p in params)


def test_class_index_label_feeds_stay_fp32():
    """targets of index-label losses are marked so the mixed-precision feed cast skips
    them (bf16 holds integers exactly only up to 256: a cast would move token ids)"""
    import hetu_61a7_amd as ht
    x = ht.Variable(name='x')
    for make in (lambda t: ht.nll_loss_op(x, t, 4),
                 lambda t: ht.softmaxcrossentropy_sparse_op(x, t),
                 lambda t: ht.crossentropy_sparse_op(x, t)):
        t = ht.Variable(name='t', trainable=False)
        make(t)
        assert getattr(t, 'keep_fp32', False)
    dense = ht.Variable(name='d', trainable=False)
    assert not getattr(dense, 'keep_fp32', False)


def test_optimizer_moments_load_through_saved_layout():
    """the flat optimizer buffers align segments (SEG_ALIGN), so moments are
    saved with each parameter's (offset, numel) and loaded parameter by parameter; a
    record without a layout that does not match the buffer exactly is refused."""
    import pytest
    import torch
    from hetu_61a7_amd.utils.checkpoint import _load_flat_moments

    class P(object):
        def __init__(self, name):
            self.name = name

    class Flat(object):
        pass
    a, b = P('a'), P('b')
    fl = Flat()
    fl.params = [a, b]
    fl.offsets = {a: (0, 3, (3,)), b: (8, 5, (5,))}     # b starts at the 8-element boundary
    fl.s1 = torch.zeros(13)
    fl.s2 = None
    saved = np.arange(8, dtype=np.float32)                # old packed layout: a 0..2, b 3..7
    d = {'order': ['a', 'b'], 'layout': [('a', 0, 3), ('b', 3, 5)], 's1': saved}
    _load_flat_moments(fl, d, 0)
    assert fl.s1[:3].tolist() == [0, 1, 2] and fl.s1[8:13].tolist() == [3, 4, 5, 6, 7]
    assert fl.s1[3:8].abs().sum() == 0
    with pytest.raises(ValueError):
        _load_flat_moments(fl, {'order': ['a', 'b'], 's1': saved}, 0)
    ok = {'order': ['a', 'b'], 's1': np.ones(13, np.float32)}
    _load_flat_moments(fl, ok, 0)
    assert float(fl.s1.sum()) == 13
