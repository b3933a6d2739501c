"""A small NumPy ONNX interpreter for the operator set the exporter emits.

onnxruntime is not available in this image (the reference's tests use it:
tests/onnx/test_mlp.py:53-57), so exported models are checked by evaluating
them here: the interpreter implements each ONNX operator's specification
directly in NumPy, independently of the Hetu kernels that produced the
reference outputs.
"""
from __future__ import annotations

import math

import numpy as np

from . import proto as P

_ONNX2NP = {P.FLOAT: np.float32, P.DOUBLE: np.float64, P.INT64: np.int64, P.INT32: np.int32, P.BOOL: np.bool_,
            P.FLOAT16: np.float16, P.UINT8: np.uint8, P.INT8: np.int8}


def to_array(t):
    dt = _ONNX2NP[t.data_type]
    shape = tuple(t.dims)
    if t.raw_data:
        return np.frombuffer(t.raw_data, dtype=dt).reshape(shape).copy()
    if t.float_data:
        return np.array(t.float_data, dtype=dt).reshape(shape)
    if t.int64_data:
        return np.array(t.int64_data, dtype=dt).reshape(shape)
    if t.int32_data:
        return np.array(t.int32_data, dtype=dt).reshape(shape)
    if t.double_data:
        return np.array(t.double_data, dtype=dt).reshape(shape)
    return np.zeros(shape, dt)


def attrs(node):
    out = {}
    for a in node.attribute:
        if a.type == P.A_INT:
            out[a.name] = int(a.i)
        elif a.type == P.A_FLOAT:
            out[a.name] = float(a.f)
        elif a.type == P.A_STRING:
            out[a.name] = a.s.decode()
        elif a.type == P.A_INTS:
            out[a.name] = [int(x) for x in a.ints]
        elif a.type == P.A_FLOATS:
            out[a.name] = [float(x) for x in a.floats]
        elif a.type == P.A_TENSOR:
            out[a.name] = to_array(a.t)
    return out


def _erf(x):
    v = np.vectorize(math.erf, otypes=[np.float64])
    return v(x.astype(np.float64)).astype(x.dtype)


def _pool(x, k, pads, strides, mode, count_include_pad=0):
    N, C, H, W = x.shape
    ph0, pw0, ph1, pw1 = pads
    fill = -np.inf if mode == 'max' else 0.0
    xp = np.pad(x, ((0, 0), (0, 0), (ph0, ph1), (pw0, pw1)), constant_values=fill)
    ones = np.pad(np.ones((H, W), x.dtype), ((ph0, ph1), (pw0, pw1)))
    Ho = (H + ph0 + ph1 - k[0]) // strides[0] + 1
    Wo = (W + pw0 + pw1 - k[1]) // strides[1] + 1
    out = np.empty((N, C, Ho, Wo), x.dtype)
    for i in range(Ho):
        for j in range(Wo):
            win = xp[:, :, i * strides[0]:i * strides[0] + k[0], j * strides[1]:j * strides[1] + k[1]]
            if mode == 'max':
                out[:, :, i, j] = win.max((2, 3))
            else:
                cnt = k[0] * k[1] if count_include_pad else \
                    ones[i * strides[0]:i * strides[0] + k[0], j * strides[1]:j * strides[1] + k[1]].sum()
                out[:, :, i, j] = win.sum((2, 3)) / cnt
    return out


def _conv(x, w, b, pads, strides):
    N, C, H, W = x.shape
    F, _, kh, kw = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])))
    Ho = (H + pads[0] + pads[2] - kh) // strides[0] + 1
    Wo = (W + pads[1] + pads[3] - kw) // strides[1] + 1
    cols = np.empty((N, C, kh, kw, Ho, Wo), x.dtype)
    for i in range(kh):
        for j in range(kw):
            cols[:, :, i, j] = xp[:, :, i:i + strides[0] * Ho:strides[0], j:j + strides[1] * Wo:strides[1]]
    y = np.einsum('nckhij,fckh->nfij', cols, w, optimize=True)
    if b is not None:
        y = y + b.reshape(1, -1, 1, 1)
    return y.astype(x.dtype)


def run(model, feeds):
    """Evaluate ``model`` (ModelProto) on ``feeds`` {input name: array}; returns
    the list of graph outputs."""
    g = model.graph
    env = {t.name: to_array(t) for t in g.initializer}
    env.update({k: np.asarray(v) for k, v in feeds.items()})
    for n in g.node:
        a = attrs(n)
        x = [env[i] if i else None for i in n.input]
        op = n.op_type
        if op in ('Add', 'Sub', 'Mul', 'Div'):
            f = {'Add': np.add, 'Sub': np.subtract, 'Mul': np.multiply, 'Div': np.divide}[op]
            r = f(x[0], x[1])
            if x[0].dtype == np.float32 or x[1].dtype == np.float32:
                r = r.astype(np.float32)
        elif op == 'Sum':
            r = x[0]
            for y in x[1:]:
                r = r + y
        elif op in ('Relu', 'Sigmoid', 'Tanh', 'Sqrt', 'Neg', 'Exp', 'Log', 'Abs', 'Floor', 'Sin', 'Cos',
                    'Reciprocal', 'Erf', 'Identity'):
            f = {'Relu': lambda v: np.maximum(v, 0), 'Sigmoid': lambda v: 1 / (1 + np.exp(-v)), 'Tanh': np.tanh,
                 'Sqrt': np.sqrt, 'Neg': np.negative, 'Exp': np.exp, 'Log': np.log, 'Abs': np.abs,
                 'Floor': np.floor, 'Sin': np.sin, 'Cos': np.cos, 'Reciprocal': lambda v: 1 / v, 'Erf': _erf,
                 'Identity': lambda v: v}[op]
            r = f(x[0]).astype(x[0].dtype)
        elif op == 'LeakyRelu':
            al = a.get('alpha', 0.01)
            r = np.where(x[0] > 0, x[0], al * x[0]).astype(x[0].dtype)
        elif op == 'MatMul':
            r = np.matmul(x[0], x[1])
        elif op == 'Gemm':
            A = x[0].T if a.get('transA', 0) else x[0]
            B = x[1].T if a.get('transB', 0) else x[1]
            r = a.get('alpha', 1.0) * (A @ B)
            if len(x) > 2 and x[2] is not None:
                r = r + a.get('beta', 1.0) * x[2]
            r = r.astype(np.float32)
        elif op == 'Softmax':
            ax = a.get('axis', -1)
            e = np.exp(x[0] - x[0].max(ax, keepdims=True))
            r = e / e.sum(ax, keepdims=True)
        elif op == 'Reshape':
            shp = [int(s) for s in x[1]]
            shp = [x[0].shape[i] if s == 0 else s for i, s in enumerate(shp)]
            r = x[0].reshape(shp)
        elif op == 'Transpose':
            r = np.transpose(x[0], a.get('perm'))
        elif op == 'Concat':
            r = np.concatenate(x, axis=a['axis'])
        elif op == 'Slice':
            sl = [slice(None)] * x[0].ndim
            axes = x[3] if len(x) > 3 else range(len(x[1]))
            for s, e, ax in zip(x[1], x[2], axes):
                sl[int(ax)] = slice(int(s), int(e))
            r = x[0][tuple(sl)]
        elif op == 'Pad':
            p = [int(v) for v in x[1]]
            nd = x[0].ndim
            cv = float(np.asarray(x[2]).reshape(-1)[0]) if len(x) > 2 and x[2] is not None else 0.0
            mode = a.get('mode', 'constant')
            pw = [(p[i], p[i + nd]) for i in range(nd)]
            r = np.pad(x[0], pw, mode='constant', constant_values=cv) if mode == 'constant' else \
                np.pad(x[0], pw, mode={'reflect': 'reflect', 'edge': 'edge'}[mode])
        elif op == 'Conv':
            r = _conv(x[0], x[1], x[2] if len(x) > 2 else None, a.get('pads', [0, 0, 0, 0]), a.get('strides', [1, 1]))
        elif op in ('MaxPool', 'AveragePool'):
            r = _pool(x[0], a['kernel_shape'], a.get('pads', [0, 0, 0, 0]), a.get('strides', [1, 1]),
                      'max' if op == 'MaxPool' else 'avg', a.get('count_include_pad', 0))
        elif op == 'BatchNormalization':
            X, s, bb, m, v = x
            sh = (1, -1) + (1,) * (X.ndim - 2)
            r = ((X - m.reshape(sh)) / np.sqrt(v.reshape(sh) + a.get('epsilon', 1e-5)) * s.reshape(sh)
                 + bb.reshape(sh)).astype(X.dtype)
        elif op == 'LayerNormalization':
            X = x[0]
            ax = a.get('axis', -1)
            axes = tuple(range(ax % X.ndim, X.ndim))
            mu = X.mean(axes, keepdims=True)
            var = ((X - mu) ** 2).mean(axes, keepdims=True)
            r = ((X - mu) / np.sqrt(var + a.get('epsilon', 1e-5)) * x[1] + (x[2] if len(x) > 2 else 0)).astype(X.dtype)
        elif op in ('ReduceSum', 'ReduceMean'):
            if op == 'ReduceSum':
                axes = tuple(int(v) for v in x[1]) if len(x) > 1 and x[1] is not None else None
            else:
                axes = tuple(a['axes']) if 'axes' in a else None
            f = np.sum if op == 'ReduceSum' else np.mean
            r = f(x[0], axis=axes, keepdims=bool(a.get('keepdims', 1))).astype(x[0].dtype)
        elif op == 'Cast':
            r = x[0].astype(_ONNX2NP[a['to']])
        elif op == 'OneHot':
            depth = int(np.asarray(x[1]).reshape(-1)[0])
            off, on = x[2]
            idx = x[0].astype(np.int64)
            r = np.where(np.arange(depth) == idx[..., None], on, off).astype(x[2].dtype)
        elif op == 'Where':
            r = np.where(x[0], x[1], x[2])
        elif op == 'Shape':
            r = np.array(x[0].shape, np.int64)
        elif op == 'Expand':
            r = x[0] * np.ones([int(v) for v in x[1]], x[0].dtype)
        elif op == 'Dropout':
            r = x[0]
        else:
            raise NotImplementedError('ONNX runtime: %s' % op)
        env[n.output[0]] = np.asarray(r)
    return [env[o.name] for o in g.output]
