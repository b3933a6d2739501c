"""Native C++/OpenMP CPU backend (libhetu_cpu.so) vs torch, and the logreg
MNIST CPU configuration (BASELINE config 1) through it."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht
from hetu_61a7_amd.kernels import cpu_native as CN


@pytest.mark.parametrize('ta,tb', [(False, False), (True, False), (False, True), (True, True)])
def test_gemm(ta, tb):
    rng = np.random.RandomState(0)
    M, K, N = 70, 300, 260
    a = torch.tensor(rng.randn(K, M) if ta else rng.randn(M, K), dtype=torch.float32)
    b = torch.tensor(rng.randn(N, K) if tb else rng.randn(K, N), dtype=torch.float32)
    bias = torch.tensor(rng.randn(N), dtype=torch.float32)
    A, B = (a.t() if ta else a), (b.t() if tb else b)
    np.testing.assert_allclose(CN.gemm(A, B, bias).numpy(), (A @ B + bias).numpy(), rtol=1e-4, atol=1e-4)


def test_elementwise_reduce_gather_ce():
    rng = np.random.RandomState(1)
    x = torch.tensor(rng.randn(33, 17), dtype=torch.float32)
    for op, ref in (('relu', torch.relu), ('sigmoid', torch.sigmoid), ('tanh', torch.tanh),
                    ('gelu', torch.nn.functional.gelu), ('exp', torch.exp)):
        np.testing.assert_allclose(CN.unary(op, x).numpy(), ref(x).numpy(), rtol=1e-5, atol=1e-6)
    g = torch.tensor(rng.randn(33, 17), dtype=torch.float32)
    np.testing.assert_allclose(CN.relu_grad(x, g).numpy(), (g * (x > 0)).numpy())
    np.testing.assert_allclose(CN.reduce_rows(x, 0.5).numpy(), (x.sum(0) * 0.5).numpy(), rtol=1e-5, atol=1e-6)
    ids = torch.tensor([[0, 5], [40, 2]])
    out = CN.gather_rows(x, ids)
    assert out.shape == (2, 2, 17) and float(out[1, 0].abs().sum()) == 0.0
    np.testing.assert_allclose(out[0, 1].numpy(), x[5].numpy())
    y = torch.softmax(torch.tensor(rng.randn(33, 17), dtype=torch.float32), -1)
    loss, lse = CN.softmax_ce(x, y)
    ref = -(y * torch.log_softmax(x, -1)).sum(-1)
    np.testing.assert_allclose(loss.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    xr = x.clone().requires_grad_(True)
    (-(y * torch.log_softmax(xr, -1)).sum(-1)).sum().backward()
    np.testing.assert_allclose(CN.softmax_ce_backward(x, y, torch.ones(1), lse).numpy(), xr.grad.numpy(),
                               rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('mode', ['sgd', 'momentum', 'nesterov', 'adagrad', 'adam', 'adamw'])
def test_optimizer_matches_reference(mode):
    from hetu_61a7_amd.kernels import optim as KO
    rng = np.random.RandomState(2)
    vals = [torch.tensor(rng.randn(1000), dtype=torch.float32) for _ in range(2)]
    outs = []
    for native in (False, True):
        CN.use(native)
        try:
            p, g = vals[0].clone(), vals[1].clone()
            s1, s2 = torch.zeros(1000), torch.zeros(1000)
            for t in range(1, 4):
                KO.optimizer_flat(mode, p, g, s1, s2, lr=0.01, l2=0.001, beta1t=0.9 ** t, beta2t=0.999 ** t,
                                  eps=1e-7, wd=0.01)
            outs.append(p.numpy().copy())
        finally:
            CN.use(False)
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-5, atol=1e-6)


def test_logreg_mnist_cpu_native_matches_aten():
    rng = np.random.RandomState(0)
    X = rng.randn(128, 784).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 128)]
    res = []
    for native in (False, True):
        CN.use(native)
        try:
            x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
            W = ht.init.zeros((784, 10), name='W')
            b = ht.init.zeros((10,), name='b')
            loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.linear_op(x, W, b), y_), [0])
            train = ht.optim.SGDOptimizer(0.1).minimize(loss)
            ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
            res.append([float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]))
                        for _ in range(10)])
        finally:
            CN.use(False)
    np.testing.assert_allclose(res[0], res[1], rtol=1e-5)
    assert res[1][-1] < res[1][0]
