"""Native C++/OpenMP CPU backend (csrc/cpu/*.cc) as the default CPU path: every op
family of the reference's DNNL/OpenMP backend (src/dnnl_ops: Softmax, Pad, Concat,
Transpose, Dropout, AddElewise, ReduceSumAxisZero, Initializers, ...) runs natively on
fp32 CPU tensors, matches torch's ATen (the oracle, HETU_CPU_BACKEND=aten semantics)
and records no ATen fallback."""
import numpy as np
import pytest
import torch

from hetu_61a7_amd.kernels import cpu_native as CN
from hetu_61a7_amd.kernels import elementwise as KE, softmax as KS, reduce as KR, tensor as KT, dropout as KD


@pytest.fixture(autouse=True)
def _native_on():
    old = CN.enabled()
    CN.use(True)
    CN.reset_fallbacks()
    yield
    assert CN.FALLBACKS == {}, CN.FALLBACKS
    CN.use(old)


def _aten(fn, *a, **k):
    CN.use(False)
    try:
        return fn(*a, **k)
    finally:
        CN.use(True)


@pytest.mark.parametrize('op', sorted(KE.U))
def test_unary_table(op):
    torch.manual_seed(0)
    x = torch.rand(3, 257) * 2 + 0.1       # positive: log / sqrt / rsqrt / pow defined
    if op in ('relu', 'abs', 'neg', 'sign', 'floor', 'leaky_relu', 'clamp', 'gelu', 'gelu_tanh', 'tanh', 'sigmoid',
              'sin', 'cos'):
        x = x - 1.2
    c, c2 = {'clamp': (-0.3, 0.4), 'leaky_relu': (0.1, 0.0), 'pow_c': (1.5, 0.0), 'cpow': (1.7, 0.0)}.get(op, (0.7, 0.0))
    got = KE.unary(op, x, c, c2)
    ref = _aten(KE.unary, op, x, c, c2)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize('op', ['add', 'sub', 'mul', 'div', 'max', 'min', 'relu_grad', 'gelu_grad', 'tanh_grad',
                                'sigmoid_grad', 'pow', 'add_relu'])
@pytest.mark.parametrize('shapes', [((4, 5, 6), (4, 5, 6)), ((4, 5, 6), (6,)), ((4, 5, 6), (5, 1)),
                                    ((4, 1, 6), (1, 5, 1)), ((2, 3, 4, 5), (3, 1, 1))])
def test_binary_broadcast(op, shapes):
    torch.manual_seed(1)
    a = torch.rand(*shapes[0]) + 0.5
    b = torch.rand(*shapes[1]) + 0.5
    if op in ('relu_grad', 'add_relu', 'max', 'min'):
        a = a - 1.0
    got = KE.binary(op, a, b)
    ref = _aten(KE.binary, op, a, b)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-6)


def test_binary_into_strided_out_and_scalar_operand():
    a = torch.randn(8, 16)
    out = torch.empty(8, 16)
    KE.binary('mul', a, torch.tensor(3.0), out=out)
    torch.testing.assert_close(out, a * 3.0)


@pytest.mark.parametrize('log', [False, True])
def test_softmax_and_backward(log):
    x = torch.randn(5, 7, 33)
    torch.testing.assert_close(KS.softmax(x, log), _aten(KS.softmax, x, log), rtol=1e-5, atol=1e-6)
    y = KS.softmax(x)
    dy = torch.randn_like(y)
    torch.testing.assert_close(KS.softmax_backward(y, dy), _aten(KS.softmax_backward, y, dy), rtol=1e-5, atol=1e-6)


def test_softmax_cross_entropy_dense_and_sparse():
    x = torch.randn(6, 4, 11)
    lab = torch.nn.functional.one_hot(torch.randint(0, 11, (6, 4)), 11).float()
    l1, s1 = KS.softmax_ce(x, lab)
    l0, s0 = _aten(KS.softmax_ce, x, lab)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-5)
    g = torch.rand(6, 4)
    torch.testing.assert_close(KS.softmax_ce_backward(x, lab, g), _aten(KS.softmax_ce_backward, x, lab, g),
                               rtol=1e-5, atol=1e-6)
    idx = torch.randint(0, 11, (24,))
    idx[3] = -1
    ls, lses = KS.softmax_ce_sparse(x.reshape(24, 11), idx, -1)
    l0, _ = _aten(KS.softmax_ce_sparse, x.reshape(24, 11), idx, -1)
    torch.testing.assert_close(ls, l0, rtol=1e-5, atol=1e-5)
    d1 = KS.softmax_ce_sparse_backward(x.reshape(24, 11), idx, torch.tensor(0.5), lses, -1)
    d0 = _aten(KS.softmax_ce_sparse_backward, x.reshape(24, 11), idx, torch.tensor(0.5), None, -1)
    torch.testing.assert_close(d1, d0, rtol=1e-5, atol=1e-6)


def test_layout_ops_concat_pad_transpose_repeat():
    a, b = torch.randn(3, 4, 5), torch.randn(3, 2, 5)
    torch.testing.assert_close(KT.concat([a, b], 1), torch.cat([a, b], 1), rtol=0, atol=0)
    p = KT.pad_constant(a, [(1, 0), (2, 3), (0, 1)], 0.5)
    torch.testing.assert_close(p, torch.nn.functional.pad(a, (0, 1, 2, 3, 1, 0), value=0.5), rtol=0, atol=0)
    torch.testing.assert_close(KT.unpad(p, [(1, 0), (2, 3), (0, 1)]), a, rtol=0, atol=0)
    t = torch.empty(5, 3, 4)
    KT.copy_into(t, a.permute(2, 0, 1))
    torch.testing.assert_close(t, a.permute(2, 0, 1).contiguous(), rtol=0, atol=0)
    torch.testing.assert_close(KT.repeat(a, (2, 1, 3, 2)), a.repeat(2, 1, 3, 2), rtol=0, atol=0)


def test_reductions():
    x = torch.randn(64, 37)
    torch.testing.assert_close(KR.reduce_sum(x, [0]), x.sum(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(KR.reduce_sum(x, [1]), x.sum(1), rtol=1e-5, atol=1e-5)
    y = torch.randn(3, 9, 4)
    torch.testing.assert_close(KR.reduce_mid(y), y.sum(1), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(KR.sum_to_shape(torch.randn(4, 5, 6), (5, 1)).shape, torch.Size([5, 1]))


def test_dropout_matches_the_gpu_philox_stream():
    """the CPU mask is Philox4x32-10 at counter = index / 4 (dropout.hip): recompute it
    here in numpy and check the kept elements and the 1/keep scale"""
    x = torch.ones(4099)
    keep, seed = 0.7, 12345
    y = KD.dropout(x, keep, seed)

    def philox(seed, ctr):
        M = 0xFFFFFFFF
        c = [ctr & M, (ctr >> 32) & M, 0, 0]
        k0, k1 = seed & M, (seed >> 32) & M
        for _ in range(10):
            p0, p1 = 0xD2511F53 * c[0], 0xCD9E8D57 * c[2]
            c = [(p1 >> 32) ^ c[1] ^ k0, p1 & M, (p0 >> 32) ^ c[3] ^ k1, p0 & M]
            k0, k1 = (k0 + 0x9E3779B9) & M, (k1 + 0xBB67AE85) & M
        return c
    for i in (0, 1, 2, 3, 4, 1000, 4098):
        u = (philox(seed, i // 4)[i % 4] >> 8) / 16777216.0 + 0.5 / 16777216.0
        assert float(y[i]) == pytest.approx(1 / keep if u < keep else 0.0)
    assert abs(float((y > 0).float().mean()) - keep) < 0.03


def test_initializers_native_generator():
    from hetu_61a7_amd import initializers as I
    u = I.UniformInit(-2.0, 3.0, (200, 500)).generate(7)
    assert float(u.min()) >= -2.0 and float(u.max()) < 3.0 and abs(float(u.mean()) - 0.5) < 0.02
    n = I.NormalInit(1.0, 2.0, (200, 500)).generate(7)
    assert abs(float(n.mean()) - 1.0) < 0.02 and abs(float(n.std()) - 2.0) < 0.02
    t = I.TruncatedNormalInit(0.0, 1.0, (200, 500)).generate(7)
    assert float(t.abs().max()) <= 2.0 and abs(float(t.std()) - 0.88) < 0.02
    assert torch.equal(I.NormalInit(1.0, 2.0, (200, 500)).generate(7), n)     # counter-based: reproducible
    assert not torch.equal(I.NormalInit(1.0, 2.0, (200, 500)).generate(8), n)
    assert torch.equal(I.ConstantInit(0.25, (3, 3)).generate(1), torch.full((3, 3), 0.25))


def test_logreg_step_issues_no_aten_compute():
    """BASELINE config 1 (bench.py --model logreg): a steady-state step on the CPU
    executor issues no ATen compute op (torch CPU profiler) and no native fallback"""
    import argparse
    from hetu_61a7_amd.models.cnn import logreg_bench
    step, B, cfg, metric, _ = logreg_bench(argparse.Namespace(batch=128), 1, 0, 0)
    for _ in range(3):
        step()
    ex = step.extra()
    assert ex['aten_compute_ops_per_step'] == [] and ex['native_cpu_fallbacks'] == {}, ex
