"""ONNX export / import (reference tests/onnx/test_mlp.py, test_cnn.py,
test_nodes.py).  onnxruntime is not installed: exported models are evaluated
with the NumPy ONNX interpreter (hetu_61a7_amd.onnx.runtime) and compared
with the executor's outputs; imported models are run by the executor and
compared with the interpreter.  Parity with onnxruntime itself: unpinned."""
import os

import numpy as np
import pytest

import hetu_61a7_amd as ht
from hetu_61a7_amd import init
from hetu_61a7_amd import onnx as ax


def _mlp():
    W1 = init.random_normal((784, 256), stddev=0.1, name='W1')
    W2 = init.random_normal((256, 256), stddev=0.1, name='W2')
    W3 = init.random_normal((256, 10), stddev=0.1, name='W3')
    b1 = init.random_normal((256,), stddev=0.1, name='b1')
    b2 = init.random_normal((256,), stddev=0.1, name='b2')
    b3 = init.random_normal((10,), stddev=0.1, name='b3')
    X = ht.Variable(name='X')
    z2 = ht.relu_op(ht.matmul_op(X, W1) + b1)
    z4 = ht.relu_op(ht.matmul_op(z2, W2) + b2)
    y = ht.softmax_op(ht.matmul_op(z4, W3) + b3)
    return X, y


def test_mlp_export_matches_executor(tmp_path):
    X, y = _mlp()
    ex = ht.Executor([y], ctx=ht.cpu(0))
    xv = np.random.RandomState(123).normal(scale=0.1, size=(128, 784)).astype(np.float32)
    ath = ex.run(feed_dict={X: xv}, convert_to_numpy_ret_vals=True)[0]
    path = str(tmp_path / 'ath.onnx')
    ax.hetu2onnx.export(ex, [X], [y], path)
    with open(path, 'rb') as f:
        model = ax.proto.parse_model(f.read())
    assert model.opset_import[0].version == 17
    pre = ax.runtime.run(model, {'X': xv})[0]
    np.testing.assert_allclose(pre, ath, rtol=1e-4, atol=1e-6)
    # round trip: import the file back and run it through the executor
    x2, y2 = ax.load_onnx(path)
    ex2 = ht.Executor([y2], ctx=ht.cpu(0))
    back = ex2.run(feed_dict={x2: xv}, convert_to_numpy_ret_vals=True)[0]
    np.testing.assert_allclose(back, ath, rtol=1e-4, atol=1e-6)


def test_cnn_export_and_import(tmp_path):
    rng = np.random.RandomState(0)
    X = ht.Variable(name='X')
    W1 = init.random_normal((8, 3, 3, 3), stddev=0.2, name='cw1')
    b1 = init.random_normal((8,), stddev=0.1, name='cb1')
    W2 = init.random_normal((8 * 4 * 4, 10), stddev=0.1, name='fw')
    h = ht.relu_op(ht.conv2d_add_bias_op(X, W1, b1, padding=1, stride=1))
    h = ht.max_pool2d_op(h, 2, 2, padding=0, stride=2)
    h = ht.avg_pool2d_op(h, 2, 2, padding=0, stride=2)
    h = ht.array_reshape_op(h, (-1, 8 * 4 * 4))
    y = ht.tanh_op(ht.matmul_op(h, W2))
    ex = ht.Executor([y], ctx=ht.cpu(0))
    xv = rng.randn(2, 3, 16, 16).astype(np.float32)
    ref = ex.run(feed_dict={X: xv}, convert_to_numpy_ret_vals=True)[0]
    path = str(tmp_path / 'cnn.onnx')
    m = ax.export(ex, [X], [y], path)
    got = ax.runtime.run(m, {'X': xv})[0]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    x2, y2 = ax.load_onnx(path)
    back = ht.Executor([y2], ctx=ht.cpu(0)).run(feed_dict={x2: xv}, convert_to_numpy_ret_vals=True)[0]
    np.testing.assert_allclose(back, ref, rtol=1e-4, atol=1e-5)


def test_node_coverage_export():
    """Every exported op type against the NumPy ONNX interpreter."""
    rng = np.random.RandomState(1)
    X = ht.Variable(name='X')
    W = init.random_normal((6, 6), stddev=0.3, name='W')
    b = init.random_normal((6,), stddev=0.1, name='b')
    g, be = init.ones((6,), name='lg'), init.zeros((6,), name='lb')
    h = ht.linear_op(X, W, b, activation='gelu')
    h = ht.layer_normalization_op(h, g, be, eps=1e-5)
    h = ht.addbyconst_op(ht.mul_byconst_op(h, 2.0), 0.5)
    h = ht.minus_byconst_op(h, 1.0)
    h = ht.transpose_op(h, (1, 0))
    h = ht.slice_op(h, (1, 0), (4, -1))
    h = ht.pad_op(h, [[1, 1], [0, 2]])
    h = ht.concatenate_op([h, ht.sigmoid_op(h)], axis=1)
    h = ht.reduce_sum_op(h, [1], keepdims=True) + ht.reduce_mean_op(h, [1], keepdims=True)
    h = ht.sqrt_op(ht.exp_op(ht.opposite_op(h)))
    y = ht.leaky_relu_op(ht.div_const_op(1.0, ht.addbyconst_op(h, 3.0)), 0.1)
    ex = ht.Executor([y], ctx=ht.cpu(0))
    xv = rng.randn(5, 6).astype(np.float32)
    ref = ex.run(feed_dict={X: xv}, convert_to_numpy_ret_vals=True)[0]
    m = ax.hetu2onnx.to_model(ex, [X], [y])
    ops = {n.op_type for n in m.graph.node}
    assert {'Gemm', 'Erf', 'LayerNormalization', 'Transpose', 'Slice', 'Pad', 'Concat', 'ReduceSum',
            'ReduceMean', 'LeakyRelu'} <= ops
    got = ax.runtime.run(m, {'X': xv})[0]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def test_batchnorm_inference_export():
    rng = np.random.RandomState(2)
    X = ht.Variable(name='X')
    s, bb = init.ones((4,), name='bs'), init.zeros((4,), name='bb')
    W = init.random_normal((4, 4, 1, 1), stddev=0.5, name='cw')
    h = ht.batch_normalization_op(ht.conv2d_op(X, W), s, bb, momentum=0.5, eps=1e-5)
    y = ht.relu_op(h)
    loss = ht.reduce_mean_op(y, [0, 1, 2, 3])
    train = ht.optim.SGDOptimizer(0.0).minimize(loss)    # lr 0: only the running stats move
    ex = ht.Executor({'train': [loss, train], 'infer': [y]}, ctx=ht.cpu(0))
    xv = rng.randn(3, 4, 5, 5).astype(np.float32)
    for _ in range(3):
        ex.run('train', feed_dict={X: xv})
    ref = ex.run('infer', feed_dict={X: xv}, convert_to_numpy_ret_vals=True)[0]
    m = ax.hetu2onnx.to_model(ex, [X], [y], name='infer')
    got = ax.runtime.run(m, {'X': xv})[0]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def test_unsupported_op_raises():
    X = ht.Variable(name='X')
    y = ht.argsort_op(X) if hasattr(ht, 'argsort_op') else ht.cumsum_with_bias_op(X)
    ex = ht.Executor([y], ctx=ht.cpu(0))
    ex.run(feed_dict={X: np.zeros((2, 3), np.float32)})
    with pytest.raises(NotImplementedError):
        ax.hetu2onnx.to_model(ex, [X], [y])
