"""ONNX model -> Hetu graph (reference python/hetu/onnx/onnx2hetu.py:32-215 and the
X2hetu handlers array.py / math.py / nn.py).

    x, y = ht.onnx.onnx2hetu.load_onnx('model.onnx')     # reference API: 1 in, 1 out
    ex = ht.Executor([y], ctx=ht.gpu(0)); ex.run(feed_dict={x: data})

Initializers become Variables carrying their values (trainable for float
tensors of rank >= 1, so an imported model can be fine-tuned); graph inputs
become placeholders.  ``from_onnx_graph`` returns every input/output.
"""
from __future__ import annotations

import numpy as np

from . import proto as P
from .runtime import to_array, attrs


def load_onnx(onnx_path):
    with open(onnx_path, 'rb') as f:
        model = P.parse_model(f.read())
    return from_onnx(model)


def from_onnx(model):
    ins, outs = from_onnx_graph(model)
    assert len(ins) == 1 and len(outs) == 1, 'only support length of input and output is 1 now.'
    return list(ins.values())[0], list(outs.values())[0]


def _const_of(env_np, name):
    return env_np.get(name)


def from_onnx_graph(model):
    """-> ({input name: placeholder}, {output name: node})"""
    from .. import ops as ht
    g = model.graph
    consts = {t.name: to_array(t) for t in g.initializer}
    env = {}
    for name, arr in consts.items():
        trainable = arr.dtype == np.float32 and arr.ndim >= 1
        env[name] = ht.Variable(name=name, value=arr, trainable=trainable)
    inputs = {}
    for vi in g.input:
        if vi.name in consts:
            continue
        v = ht.Variable(name=vi.name, trainable=False)
        env[vi.name] = inputs[vi.name] = v

    def scalar(name):
        a = consts.get(name)
        return None if a is None or a.size != 1 else float(a.reshape(-1)[0])

    for n in g.node:
        a = attrs(n)
        op = n.op_type
        x = [env.get(i) for i in n.input]
        o = None
        if op in ('Add', 'Mul', 'Sub', 'Div'):
            c0, c1 = scalar(n.input[0]), scalar(n.input[1])
            if op == 'Add':
                o = ht.addbyconst_op(x[0], c1) if c1 is not None else \
                    ht.addbyconst_op(x[1], c0) if c0 is not None else ht.add_op(x[0], x[1])
            elif op == 'Mul':
                o = ht.mul_byconst_op(x[0], c1) if c1 is not None else \
                    ht.mul_byconst_op(x[1], c0) if c0 is not None else ht.mul_op(x[0], x[1])
            elif op == 'Sub':
                o = ht.addbyconst_op(x[0], -c1) if c1 is not None else \
                    ht.minus_byconst_op(x[1], c0) if c0 is not None else ht.minus_op(x[0], x[1])
            else:
                o = ht.mul_byconst_op(x[0], 1.0 / c1) if c1 is not None else \
                    ht.div_const_op(c0, x[1]) if c0 is not None else ht.div_op(x[0], x[1])
        elif op == 'Sum':
            o = ht.sum_op(x)
        elif op in ('Relu', 'Sigmoid', 'Tanh', 'Sqrt', 'Neg', 'Exp', 'Log', 'Abs', 'Floor', 'Sin', 'Cos'):
            f = {'Relu': ht.relu_op, 'Sigmoid': ht.sigmoid_op, 'Tanh': ht.tanh_op, 'Sqrt': ht.sqrt_op,
                 'Neg': ht.opposite_op, 'Exp': ht.exp_op, 'Log': ht.log_op, 'Abs': ht.abs_op, 'Floor': ht.floor_op,
                 'Sin': ht.sin_op, 'Cos': ht.cos_op}[op]
            o = f(x[0])
        elif op == 'Reciprocal':
            o = ht.div_const_op(1.0, x[0])
        elif op == 'LeakyRelu':
            o = ht.leaky_relu_op(x[0], a.get('alpha', 0.01))
        elif op in ('Identity', 'Dropout'):
            o = x[0]
        elif op == 'MatMul':
            o = ht.matmul_op(x[0], x[1])
        elif op == 'Gemm':
            if a.get('alpha', 1.0) != 1.0 or a.get('beta', 1.0) != 1.0:
                raise NotImplementedError('Gemm with alpha/beta != 1')
            ta, tb = bool(a.get('transA', 0)), bool(a.get('transB', 0))
            o = ht.linear_op(x[0], x[1], x[2], ta, tb) if len(x) > 2 and x[2] is not None else \
                ht.matmul_op(x[0], x[1], ta, tb)
        elif op == 'Softmax':
            o = ht.softmax_op(x[0])
        elif op == 'Reshape':
            o = ht.array_reshape_op(x[0], [int(v) for v in consts[n.input[1]]])
        elif op == 'Transpose':
            o = ht.transpose_op(x[0], a.get('perm'))
        elif op == 'Concat':
            o = ht.concatenate_op(x, axis=a['axis'])
        elif op == 'Slice':
            starts = [int(v) for v in consts[n.input[1]]]
            ends = [int(v) for v in consts[n.input[2]]]
            axes = [int(v) for v in consts[n.input[3]]] if len(n.input) > 3 else list(range(len(starts)))
            if axes != list(range(len(axes))):
                raise NotImplementedError('Slice over non-leading axes list')
            o = ht.slice_op(x[0], starts, [e - s for s, e in zip(starts, ends)])
        elif op == 'Pad':
            p = [int(v) for v in consts[n.input[1]]]
            nd = len(p) // 2
            cv = scalar(n.input[2]) if len(n.input) > 2 and n.input[2] else 0.0
            o = ht.pad_op(x[0], [[p[i], p[i + nd]] for i in range(nd)], a.get('mode', 'constant').upper(), cv or 0.0)
        elif op == 'Conv':
            pads, st = a.get('pads', [0, 0, 0, 0]), a.get('strides', [1, 1])
            if pads[0] != pads[2] or pads[1] != pads[3]:
                raise NotImplementedError('asymmetric Conv padding')
            if len(x) > 2 and x[2] is not None:
                o = ht.conv2d_add_bias_op(x[0], x[1], x[2], padding=(pads[0], pads[1]), stride=tuple(st))
            else:
                o = ht.conv2d_op(x[0], x[1], padding=(pads[0], pads[1]), stride=tuple(st))
        elif op in ('MaxPool', 'AveragePool'):
            k, pads, st = a['kernel_shape'], a.get('pads', [0, 0, 0, 0]), a.get('strides', [1, 1])
            f = ht.max_pool2d_op if op == 'MaxPool' else ht.avg_pool2d_op
            o = f(x[0], k[0], k[1], padding=(pads[0], pads[1]), stride=tuple(st))
        elif op == 'BatchNormalization':
            o = ht.batch_normalization_op(x[0], x[1], x[2], momentum=1.0 - a.get('momentum', 0.9),
                                          eps=a.get('epsilon', 1e-5))
            o.running_mean_init = consts.get(n.input[3])
            o.running_var_init = consts.get(n.input[4])
        elif op == 'LayerNormalization':
            o = ht.layer_normalization_op(x[0], x[1], x[2], eps=a.get('epsilon', 1e-5))
        elif op == 'ReduceSum':
            axes = [int(v) for v in consts[n.input[1]]] if len(n.input) > 1 else None
            o = ht.reduce_sum_op(x[0], axes, keepdims=bool(a.get('keepdims', 1)))
        elif op == 'ReduceMean':
            o = ht.reduce_mean_op(x[0], a.get('axes'), keepdims=bool(a.get('keepdims', 1)))
        elif op == 'Cast':
            o = x[0]
        elif op == 'OneHot':
            depth = int(consts[n.input[1]].reshape(-1)[0])
            o = ht.one_hot_op(x[0], depth)
        elif op == 'Where':
            o = ht.where_op(x[0], x[1], x[2])
        else:
            raise NotImplementedError('ONNX import: %s' % op)
        env[n.output[0]] = o
    outputs = {vi.name: env[vi.name] for vi in g.output}
    return inputs, outputs
