"""Native CPU convolution / pooling / batch norm (csrc/cpu/cpu_ops.cc; the reference's
DNNL ops src/dnnl_ops/Conv2d.cpp, MaxPool.cpp, AvgPool.cpp, BatchNorm.cpp) against
PyTorch fp32 references, and a small CNN trained through the native CPU backend."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from hetu_61a7_amd.kernels import cpu_native as CN
from hetu_61a7_amd.kernels import conv as KC, pool as KP, norm as KN


@pytest.fixture
def native():
    CN.use(True)
    yield
    CN.use(False)


@pytest.mark.parametrize('n,c,h,k,ks,s,p', [(2, 3, 11, 5, 3, 1, 1), (3, 4, 9, 6, 3, 2, 1), (1, 2, 8, 3, 1, 1, 0),
                                           (2, 3, 12, 4, 5, 2, 2)])
def test_conv2d_fwd_bwd(native, n, c, h, k, ks, s, p):
    torch.manual_seed(0)
    x = torch.randn(n, c, h, h + 1, requires_grad=True)
    w = torch.randn(k, c, ks, ks, requires_grad=True)
    b = torch.randn(k)
    y = KC.conv2d(x.detach(), w.detach(), b, (s, s), (p, p))
    ref = F.conv2d(x, w, b, s, p)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    ref.backward(g)
    dx = KC.conv2d_backward_data(g, w.detach(), x.shape, (s, s), (p, p))
    torch.testing.assert_close(dx, x.grad, rtol=1e-4, atol=1e-4)
    dw = KC.conv2d_backward_filter(g, x.detach(), w.shape, (s, s), (p, p))
    torch.testing.assert_close(dw, w.grad, rtol=1e-4, atol=1e-3)


def test_pools(native):
    torch.manual_seed(1)
    x = torch.randn(2, 3, 9, 10, requires_grad=True)
    y, idx = KP.maxpool2d(x.detach(), 3, 3, 2, 2, 1, 1)
    ref = F.max_pool2d(x, 3, 2, 1)
    torch.testing.assert_close(y, ref.detach())
    g = torch.randn_like(ref)
    ref.backward(g)
    torch.testing.assert_close(KP.maxpool2d_backward(g, idx, x.shape, 3, 3, 2, 2, 1, 1), x.grad)
    x2 = x.detach().clone().requires_grad_(True)
    ya = KP.avgpool2d(x2.detach(), 2, 3, 2, 1, 0, 1)
    ra = F.avg_pool2d(x2, (2, 3), (2, 1), (0, 1))
    torch.testing.assert_close(ya, ra.detach(), rtol=1e-5, atol=1e-6)
    ga = torch.randn_like(ra)
    ra.backward(ga)
    torch.testing.assert_close(KP.avgpool2d_backward(ga, x.shape, 2, 3, 2, 1, 0, 1), x2.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('relu', [False, True])
def test_batchnorm(native, relu):
    torch.manual_seed(2)
    x = torch.randn(4, 5, 6, 7, requires_grad=True)
    gamma = torch.rand(5, requires_grad=True)
    beta = torch.randn(5, requires_grad=True)
    rm, rv = torch.zeros(5), torch.ones(5)
    rm2, rv2 = rm.clone(), rv.clone()
    y, mean, invstd = KN.bn_forward(x.detach(), gamma.detach(), beta.detach(), rm, rv, 0.1, 1e-5, True, relu=relu)
    ref = F.batch_norm(x, rm2, rv2, gamma, beta, True, 0.1, 1e-5)
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm, rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, rv2, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(ref)
    ref.backward(g)
    dx, ds, db, _ = KN.bn_backward(g, y, x.detach(), gamma.detach(), mean, invstd, relu=relu)
    torch.testing.assert_close(dx, x.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ds, gamma.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, beta.grad, rtol=1e-4, atol=1e-4)
    yi, _, _ = KN.bn_forward(x.detach(), gamma.detach(), beta.detach(), rm, rv, 0.1, 1e-5, False)
    torch.testing.assert_close(yi, F.batch_norm(x.detach(), rm, rv, gamma.detach(), beta.detach(), False, 0.1, 1e-5),
                               rtol=1e-4, atol=1e-5)


def test_cnn_trains_on_native_cpu_backend(native, monkeypatch):
    import hetu_61a7_amd as ht
    calls = {}
    for name in ('conv2d', 'conv2d_backward_filter', 'batchnorm', 'batchnorm_backward', 'maxpool2d',
                 'maxpool2d_backward'):
        fn = getattr(CN, name)
        monkeypatch.setattr(CN, name, (lambda fn, name: lambda *a, **k: (calls.__setitem__(name, calls.get(name, 0) + 1),
                                                                         fn(*a, **k))[1])(fn, name))
    rng = np.random.RandomState(0)
    xs = rng.randn(16, 3, 8, 8).astype(np.float32)
    ys = np.eye(4, dtype=np.float32)[rng.randint(0, 4, 16)]
    x = ht.Variable(name='x', trainable=False)
    y_ = ht.Variable(name='y', trainable=False)
    w1 = ht.init.random_normal((8, 3, 3, 3), stddev=0.1, name='w1')
    h = ht.conv2d_op(x, w1, padding=1, stride=1)
    h = ht.batch_normalization_op(h, ht.init.ones((8,), name='g'), ht.init.zeros((8,), name='b'))
    h = ht.relu_op(h)
    h = ht.max_pool2d_op(h, 2, 2, 0, 2)
    h = ht.array_reshape_op(h, (-1, 8 * 4 * 4))
    w2 = ht.init.random_normal((8 * 4 * 4, 4), stddev=0.1, name='w2')
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, w2), y_), [0])
    train = ht.optim.SGDOptimizer(learning_rate=0.1).minimize(loss)
    ex = ht.Executor([loss, train], ctx=ht.cpu(0))
    losses = [float(ex.run(feed_dict={x: xs, y_: ys}, convert_to_numpy_ret_vals=True)[0]) for _ in range(30)]
    assert losses[-1] < 0.5 * losses[0], losses
    assert all(calls.get(n, 0) >= 30 for n in ('conv2d', 'conv2d_backward_filter', 'batchnorm',
                                                'batchnorm_backward', 'maxpool2d', 'maxpool2d_backward')), calls
