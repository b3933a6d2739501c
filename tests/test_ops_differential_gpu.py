"""CPU-vs-GPU differential tests over the operator library (reference
tests/tester.py:5-25 ``HetuTester`` + tests/test_ops.py): every op is built on a
CPU executor and on a GPU executor (fp32, HIP kernels) with identical inputs,
and the outputs and the gradients wrt every float input are compared.

The GEMM and convolution cases run with the hand-written kernels forced
(``HETU_GEMM=hip`` / ``HETU_CONV=hip`` semantics: the exact-fp32 MFMA GEMM and
implicit-GEMM convolution of gemm_f32.hip) and assert that those kernels ran and
nothing fell back to hipBLASLt / MIOpen."""
import numpy as np
import pytest

import hetu_61a7_amd as ht

pytestmark = pytest.mark.gpu


class HetuTester(object):
    def __init__(self, builder, shapes, int_inputs=(), rtol=1e-4, atol=1e-5, grad=True, seed=0):
        self.builder, self.shapes, self.int_inputs = builder, shapes, set(int_inputs)
        self.rtol, self.atol, self.grad = rtol, atol, grad
        rng = np.random.RandomState(seed)
        self.vals = []
        for i, s in enumerate(shapes):
            if i in self.int_inputs:
                self.vals.append(rng.randint(0, s[1], size=s[0]).astype(np.float32))
            else:
                self.vals.append(rng.uniform(-1.0, 1.0, size=s).astype(np.float32))

    def _run(self, ctx):
        xs = [ht.Variable(name='in%d' % i, trainable=False) for i in range(len(self.shapes))]
        y = self.builder(*xs)
        nodes = [y]
        wrt = [x for i, x in enumerate(xs) if i not in self.int_inputs]
        if self.grad:
            loss = ht.reduce_sum_op(ht.mul_op(y, y), None)
            nodes += ht.gradients(loss, wrt)
        ex = ht.Executor(nodes, ctx=ctx)
        out = ex.run(feed_dict=dict(zip(xs, self.vals)), convert_to_numpy_ret_vals=True)
        return [np.asarray(o) for o in out if o is not None]

    def check(self):
        a = self._run(ht.cpu(0))
        b = self._run(ht.gpu(0))
        assert len(a) == len(b)
        for x, y in zip(a, b):
            np.testing.assert_allclose(y, x, rtol=self.rtol, atol=self.atol)


CASES = {
    'add': (lambda a, b: ht.add_op(a, b), [(7, 9), (7, 9)]),
    'add_bcast': (lambda a, b: ht.add_op(a, b), [(7, 9), (9,)]),
    'minus': (lambda a, b: ht.minus_op(a, b), [(5, 6), (5, 6)]),
    'mul': (lambda a, b: ht.mul_op(a, b), [(5, 6), (5, 6)]),
    'div': (lambda a, b: ht.div_op(a, ht.addbyconst_op(ht.abs_op(b), 0.5)), [(5, 6), (5, 6)]),
    'byconst': (lambda a: ht.minus_byconst_op(ht.mul_byconst_op(ht.addbyconst_op(a, 2.0), 3.0), 1.0), [(4, 8)]),
    'div_const': (lambda a: ht.div_const_op(2.0, ht.addbyconst_op(ht.abs_op(a), 0.5)), [(4, 8)]),
    'relu': (lambda a: ht.relu_op(a), [(33, 65)]),
    'leaky_relu': (lambda a: ht.leaky_relu_op(a, 0.1), [(33, 65)]),
    'sigmoid': (lambda a: ht.sigmoid_op(a), [(16, 40)]),
    'tanh': (lambda a: ht.tanh_op(a), [(16, 40)]),
    'gelu': (lambda a: ht.gelu_op(a), [(16, 40)]),
    'exp_log': (lambda a: ht.log_op(ht.addbyconst_op(ht.exp_op(a), 1.0)), [(16, 40)]),
    'sqrt': (lambda a: ht.sqrt_op(ht.addbyconst_op(ht.abs_op(a), 0.1)), [(16, 40)]),
    'opposite': (lambda a: ht.opposite_op(a), [(8, 8)]),
    'matmul': (lambda a, b: ht.matmul_op(a, b), [(24, 40), (40, 16)]),
    'matmul_tt': (lambda a, b: ht.matmul_op(a, b, True, True), [(40, 24), (16, 40)]),
    'linear_relu': (lambda a, b, c: ht.linear_op(a, b, c, activation='relu'), [(24, 40), (40, 16), (16,)]),
    'batch_matmul': (lambda a, b: ht.batch_matmul_op(a, b), [(3, 8, 16), (3, 16, 12)]),
    'softmax': (lambda a: ht.softmax_op(a), [(12, 30)]),
    'softmax_ce': (lambda a, b: ht.softmaxcrossentropy_op(a, ht.softmax_op(b)), [(12, 30), (12, 30)]),
    'reduce_sum': (lambda a: ht.reduce_sum_op(a, [1]), [(6, 7, 8)]),
    'reduce_mean': (lambda a: ht.reduce_mean_op(a, [0, 2]), [(6, 7, 8)]),
    'reduce_axis0': (lambda a: ht.reducesumaxiszero_op(a), [(40, 24)]),
    'transpose': (lambda a: ht.transpose_op(a, (2, 0, 1)), [(3, 4, 5)]),
    'reshape': (lambda a: ht.array_reshape_op(a, (6, 20)), [(3, 4, 10)]),
    'slice': (lambda a: ht.slice_op(a, (1, 2), (3, 4)), [(6, 8)]),
    'concat': (lambda a, b: ht.concat_op(a, b, axis=1), [(4, 3), (4, 5)]),
    'pad': (lambda a: ht.pad_op(a, [[0, 0], [0, 0], [1, 2], [2, 1]]), [(2, 3, 4, 5)]),
    'broadcast': (lambda a, b: ht.broadcastto_op(a, b), [(5,), (3, 5)]),
    'layernorm': (lambda a, g, b: ht.layer_normalization_op(a, g, b, eps=1e-5), [(16, 32), (32,), (32,)]),
    'conv2d': (lambda x, w: ht.conv2d_op(x, w, padding=1, stride=1), [(2, 3, 8, 8), (4, 3, 3, 3)]),
    'conv2d_s2': (lambda x, w: ht.conv2d_op(x, w, padding=0, stride=2), [(2, 8, 9, 9), (8, 8, 1, 1)]),
    'conv_bias': (lambda x, w, b: ht.conv2d_add_bias_op(x, w, b, padding=1, stride=1),
                  [(2, 3, 6, 6), (4, 3, 3, 3), (4,)]),
    'maxpool': (lambda x: ht.max_pool2d_op(x, 2, 2, padding=0, stride=2), [(2, 3, 8, 8)]),
    'avgpool': (lambda x: ht.avg_pool2d_op(x, 3, 3, padding=1, stride=1), [(2, 3, 6, 6)]),
    'batchnorm': (lambda x, s, b: ht.batch_normalization_op(x, s, b, momentum=0.1, eps=1e-5),
                  [(4, 3, 5, 5), (3,), (3,)]),
    'embedding': (lambda t, i: ht.embedding_lookup_op(t, i), [(20, 8), (6, 20)]),
    'one_hot': (lambda i: ht.one_hot_op(i, 7), [(5, 7)]),
    'where': (lambda c, a, b: ht.where_op(ht.bool_op(c), a, b), [(4, 6), (4, 6), (4, 6)]),
}
INT_INPUTS = {'embedding': (1,), 'one_hot': (0,)}
NO_GRAD = {'one_hot', 'where'}


# cases whose GPU run must use the hand-written fp32 MFMA kernels: native-call names expected
HIP_GEMM_CONV = {
    'matmul': ('gemm_f32',), 'matmul_tt': ('gemm_f32',), 'linear_relu': ('gemm_f32',),
    'batch_matmul': ('gemm_f32',),
    'conv2d': ('conv_fwd_f32', 'conv_dgrad_f32', 'conv_wgrad_f32'),
    'conv2d_s2': ('conv_fwd_f32', 'conv_dgrad_f32', 'conv_wgrad_f32'),
    'conv_bias': ('conv_fwd_f32', 'conv_dgrad_f32', 'conv_wgrad_f32'),
}


@pytest.fixture
def force_hip(monkeypatch):
    from hetu_61a7_amd import kernels as K
    from hetu_61a7_amd.kernels import autotune
    # (every device GEMM / convolution is a hand-written kernel -- there is no library mode
    # to switch off; fresh autotune decisions so this test's shapes are chosen here)
    monkeypatch.setattr(autotune, '_decisions', {})
    K.reset_dispatch_stats()
    return K


@pytest.mark.parametrize('name', sorted(CASES))
def test_cpu_gpu_differential(name, force_hip):
    builder, shapes = CASES[name]
    if not all(hasattr(ht, n) for n in ('bool_op',)) and name == 'where':
        pytest.skip('bool_op missing')
    HetuTester(builder, shapes, int_inputs=INT_INPUTS.get(name, ()), grad=name not in NO_GRAD,
               rtol=2e-4, atol=2e-5).check()
    K = force_hip
    for k in HIP_GEMM_CONV.get(name, ()):
        assert K.NATIVE_CALLS.get(k, 0) >= 1, (name, k, K.NATIVE_CALLS, K.VENDOR_CALLS)
    if name in HIP_GEMM_CONV:
        assert not K.FALLBACKS, (name, K.FALLBACKS)
        assert not {k: v for k, v in K.VENDOR_CALLS.items() if k in ('gemm', 'bmm', 'conv')}, K.VENDOR_CALLS
