"""Hetu graph -> ONNX model (reference python/hetu/onnx/hetu2onnx.py:27-204 and the
opset handlers in onnx_opset/*.py: AddConst, AddElewise, BatchNorm, Concat,
Conv2d, Division, Dropout, Identity, MatrixMult, MultiplyConst, OneHot,
Opposite, Pad, Pool, Reduces, Relu, Reshape, Slice, Softmax, Sqrt, Tanh,
Transpose, Variable, Where) -- plus the ops this framework adds on top
(Linear/Gemm with fused activation, LayerNorm, GELU, Sigmoid, Exp/Log, Sum,
BroadcastTo, fused BN+ReLU(+residual), dropout+add+LayerNorm).

    ex = ht.Executor([y], ctx=ht.cpu(0)); ex.run(feed_dict={X: x})
    ht.onnx.hetu2onnx.export(ex, [X], [y], 'model.onnx')

Trained parameter values (fp32 masters) become initializers; fed placeholders
become graph inputs with the shapes of the executor's last run (or
``input_shapes``).  Default opset 17.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

from . import proto as P

_NP2ONNX = {np.dtype(np.float32): P.FLOAT, np.dtype(np.float64): P.DOUBLE, np.dtype(np.int64): P.INT64,
            np.dtype(np.int32): P.INT32, np.dtype(np.bool_): P.BOOL, np.dtype(np.float16): P.FLOAT16,
            np.dtype(np.uint8): P.UINT8, np.dtype(np.int8): P.INT8}


def make_tensor(name: str, arr) -> object:
    arr = np.ascontiguousarray(np.asarray(arr))
    if arr.dtype == np.float64:
        arr = arr.astype(np.float32)
    t = P.classes()['TensorProto']()
    t.name = name
    t.dims.extend(arr.shape)
    t.data_type = _NP2ONNX[arr.dtype]
    t.raw_data = arr.tobytes()
    return t


def _value_info(name, shape, elem=P.FLOAT):
    vi = P.classes()['ValueInfoProto']()
    vi.name = name
    tt = vi.type.tensor_type
    tt.elem_type = elem
    if shape is not None:
        for d in shape:
            dim = tt.shape.dim.add()
            if d is None or (isinstance(d, int) and d < 0):
                dim.dim_param = 'N'
            else:
                dim.dim_value = int(d)
    return vi


def _attr(name, v):
    a = P.classes()['AttributeProto']()
    a.name = name
    if isinstance(v, bool) or isinstance(v, (int, np.integer)):
        a.type, a.i = P.A_INT, int(v)
    elif isinstance(v, float):
        a.type, a.f = P.A_FLOAT, float(v)
    elif isinstance(v, str):
        a.type, a.s = P.A_STRING, v.encode()
    elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, np.integer)) for x in v):
        a.type = P.A_INTS
        a.ints.extend(int(x) for x in v)
    elif isinstance(v, (list, tuple)):
        a.type = P.A_FLOATS
        a.floats.extend(float(x) for x in v)
    else:
        raise TypeError('attribute %s: %r' % (name, v))
    return a


class _Builder(object):
    def __init__(self, opset):
        self.opset = opset
        self.nodes = []
        self.inits = []
        self.init_names = set()
        self.uid = 0

    def fresh(self, base):
        self.uid += 1
        return '%s__%d' % (base, self.uid)

    def const(self, arr, base='const'):
        name = self.fresh(base)
        self.inits.append(make_tensor(name, arr))
        self.init_names.add(name)
        return name

    def node(self, op_type, inputs, outputs=None, name=None, **attrs):
        n = P.classes()['NodeProto']()
        n.op_type = op_type
        n.name = name or self.fresh(op_type)
        n.input.extend(inputs)
        outputs = outputs or [self.fresh(op_type + '_out')]
        n.output.extend(outputs)
        for k, v in attrs.items():
            if v is not None:
                n.attribute.append(_attr(k, v))
        self.nodes.append(n)
        return outputs[0] if len(outputs) == 1 else outputs

    def gelu(self, x, out=None):
        # 0.5 * x * (1 + erf(x / sqrt(2)))  (erf form, reference Gelu.cu:6-11)
        d = self.node('Div', [x, self.const(np.float32(math.sqrt(2.0)))])
        e = self.node('Erf', [d])
        a = self.node('Add', [e, self.const(np.float32(1.0))])
        m = self.node('Mul', [x, a])
        return self.node('Mul', [m, self.const(np.float32(0.5))], [out] if out else None)


def _np(t):
    import torch
    if isinstance(t, torch.Tensor):
        return t.detach().float().cpu().numpy() if t.is_floating_point() else t.detach().cpu().numpy()
    return np.asarray(t)


def _emit(b: _Builder, n, ins: List[str], out: str, shapes: Dict):
    """Emit ONNX nodes computing hetu node ``n`` into tensor ``out``."""
    t = type(n).__name__
    simple = {'ReluOp': 'Relu', 'SigmoidOp': 'Sigmoid', 'TanhOp': 'Tanh', 'SqrtOp': 'Sqrt', 'OppositeOp': 'Neg',
              'ExpOp': 'Exp', 'LogOp': 'Log', 'AbsOp': 'Abs', 'FloorOp': 'Floor', 'SinOp': 'Sin', 'CosOp': 'Cos',
              'AddOp': 'Add', 'MinusOp': 'Sub', 'MulOp': 'Mul', 'DivOp': 'Div', 'SumOp': 'Sum'}
    if t in simple:
        return b.node(simple[t], ins, [out])
    if t in ('DropoutOp', 'Dropout2dOp'):
        return b.node('Identity', ins[:1], [out])
    if t == 'ReciprocalSqrtOp':
        return b.node('Reciprocal', [b.node('Sqrt', ins)], [out])
    if t == 'LeakyReluOp':
        return b.node('LeakyRelu', ins, [out], alpha=float(n.c))
    if t == 'GeluOp':
        return b.gelu(ins[0], out)
    if t == 'AddByConstOp':
        return b.node('Add', [ins[0], b.const(np.float32(n.const_attr))], [out])
    if t == 'MulByConstOp':
        return b.node('Mul', [ins[0], b.const(np.float32(n.const_attr))], [out])
    if t == 'MinusByConstOp':   # c - x
        return b.node('Sub', [b.const(np.float32(n.const_attr)), ins[0]], [out])
    if t == 'DivConstOp':       # c / x
        return b.node('Div', [b.const(np.float32(n.const_attr)), ins[0]], [out])
    if t in ('MatMulOp', 'LinearOp'):
        ta, tb = n.matmul_attr_trans_A, n.matmul_attr_trans_B
        if t == 'LinearOp':
            act = n.activation
            y = out if act is None else b.fresh('gemm_out')
            b.node('Gemm', ins[:3], [y], transA=int(ta), transB=int(tb))
            if act == 'relu':
                return b.node('Relu', [y], [out])
            if act == 'gelu':
                return b.gelu(y, out)
            return out
        A = b.node('Transpose', [ins[0]], perm=[1, 0]) if ta else ins[0]
        B = b.node('Transpose', [ins[1]], perm=[1, 0]) if tb else ins[1]
        return b.node('MatMul', [A, B], [out])
    if t == 'SoftmaxOp':
        return b.node('Softmax', ins, [out], axis=-1)
    if t == 'Array_ReshapeOp':
        return b.node('Reshape', [ins[0], b.const(np.array(n.output_shape, np.int64), 'shape')], [out])
    if t == 'TransposeOp':
        perm = list(n.perm) if n.perm is not None else list(range(len(shapes[n.inputs[0]])))[::-1]
        return b.node('Transpose', ins, [out], perm=perm)
    if t == 'ConcatenateOp':
        return b.node('Concat', ins, [out], axis=int(n.axis))
    if t == 'SliceOp':
        shp = shapes[n.inputs[0]]
        starts = list(n.begin)
        ends = [(shp[i] if s == -1 else starts[i] + s) for i, s in enumerate(n.size)]
        return b.node('Slice', [ins[0], b.const(np.array(starts, np.int64)), b.const(np.array(ends, np.int64)),
                                b.const(np.arange(len(starts), dtype=np.int64))], [out])
    if t == 'PadOp':
        pads = [p[0] for p in n.paddings] + [p[1] for p in n.paddings]
        return b.node('Pad', [ins[0], b.const(np.array(pads, np.int64)), b.const(np.float32(n.constant_values))],
                      [out], mode=n.mode)
    if t in ('Conv2dOp', 'Conv2dAddBiasOp'):
        w = shapes[n.inputs[1]]
        ph, pw = n.padding
        return b.node('Conv', ins, [out], kernel_shape=[w[2], w[3]], pads=[ph, pw, ph, pw],
                      strides=list(n.stride))
    if t in ('Max_Pool2dOp', 'Avg_Pool2dOp'):
        ph, pw = n.padding
        kw = dict(kernel_shape=[n.kh, n.kw], pads=[ph, pw, ph, pw], strides=list(n.stride))
        if t == 'Avg_Pool2dOp':
            kw['count_include_pad'] = 1
        return b.node('MaxPool' if t == 'Max_Pool2dOp' else 'AveragePool', ins[:1], [out], **kw)
    if t == 'Batch_NormalizationOp':
        C = shapes[n.inputs[1]][0]
        rm = _np(n.running_mean) if n.running_mean is not None else np.zeros(C, np.float32)
        rv = _np(n.running_var) if n.running_var is not None else np.ones(C, np.float32)
        y = b.node('BatchNormalization', [ins[0], ins[1], ins[2], b.const(rm, 'bn_mean'), b.const(rv, 'bn_var')],
                   [b.fresh('bn') if (n.relu or n.has_residual) else out], epsilon=float(n.eps),
                   momentum=float(1.0 - n.momentum))
        if n.has_residual:
            y = b.node('Add', [y, ins[3]], [b.fresh('bn_res') if n.relu else out])
        if n.relu:
            y = b.node('Relu', [y], [out])
        return y
    if t == 'Layer_NormalizationOp':
        return b.node('LayerNormalization', ins, [out], axis=-1, epsilon=float(n.eps))
    if t == 'DropoutAddLayerNormOp':
        s = b.node('Add', [ins[0], ins[1]]) if n.has_res else ins[0]
        return b.node('LayerNormalization', [s, ins[-2], ins[-1]], [out], axis=-1, epsilon=float(n.eps))
    if t in ('ReduceSumOp', 'ReduceMeanOp'):
        nd = len(shapes[n.inputs[0]])
        axes = n.axes if n.axes is not None else list(range(nd))
        axes = [axes] if isinstance(axes, int) else list(axes)
        if t == 'ReduceSumOp':
            return b.node('ReduceSum', [ins[0], b.const(np.array(axes, np.int64))], [out], keepdims=int(n.keepdims))
        return b.node('ReduceMean', ins, [out], axes=axes, keepdims=int(n.keepdims))
    if t == 'ReduceSumAxisZeroOp':
        return b.node('ReduceSum', [ins[0], b.const(np.array([0], np.int64))], [out], keepdims=0)
    if t == 'OneHotOp':
        idx = b.node('Cast', ins, to=P.INT64)
        return b.node('OneHot', [idx, b.const(np.array([n.num_classes], np.int64)),
                                 b.const(np.array([0.0, 1.0], np.float32))], [out], axis=-1)
    if t == 'WhereOp':
        c = b.node('Cast', [ins[0]], to=P.BOOL)
        return b.node('Where', [c, ins[1], ins[2]], [out])
    if t == 'BroadcastToOp':
        return b.node('Expand', [ins[0], b.node('Shape', [ins[1]])], [out])
    raise NotImplementedError('ONNX export: no handler for %s' % t)


def to_model(executor, inputs, outputs, job_name='HetutoOnnx', opset=17, input_shapes=None, name=None):
    from ..ops.executor import find_topo_sort
    from ..ops.variable import PlaceholderOp
    cfg = executor.config
    sub = executor.subexecutor[name] if name else next(iter(executor.subexecutor.values()))
    fed = dict(getattr(sub, 'last_feed_shapes', {}))
    if input_shapes:
        fed.update(input_shapes)
    topo = find_topo_sort(outputs)
    # shapes of every node: run the graph's own shape inference from the fed shapes
    shapes = {}
    for n in topo:
        if isinstance(n, PlaceholderOp):
            if n in fed:
                shapes[n] = tuple(fed[n])
            else:
                v = cfg.placeholder_to_arr_map.get(n)
                shapes[n] = tuple(v.shape) if v is not None else None
        else:
            try:
                shapes[n] = n.infer_shape([shapes[i] for i in n.inputs])
            except Exception:
                shapes[n] = None
    b = _Builder(opset)
    tname = {}
    graph_inputs = []
    for n in topo:
        if isinstance(n, PlaceholderOp):
            tname[n] = n.name
            if n in inputs or n in fed:
                graph_inputs.append(_value_info(n.name, shapes[n]))
            else:
                v = cfg.placeholder_to_arr_map.get(n)
                if v is None and getattr(n, 'tensor_value', None) is not None:
                    v = n.tensor_value
                if v is None:
                    raise ValueError('placeholder %s has neither a value nor a feed' % n.name)
                b.inits.append(make_tensor(n.name, _np(v)))
                b.init_names.add(n.name)
            continue
        out = 'output_%d' % outputs.index(n) if n in outputs else '%s_%d' % (type(n).__name__, n.id)
        tname[n] = out
        _emit(b, n, [tname[i] for i in n.inputs], out, shapes)
    m = P.ModelProto()
    m.ir_version = 8
    m.producer_name = 'hetu_61a7_amd'
    m.producer_version = '0.1.0'
    op = m.opset_import.add()
    op.domain, op.version = '', int(opset)
    g = m.graph
    g.name = job_name or 'HetutoOnnx'
    g.node.extend(b.nodes)
    g.initializer.extend(b.inits)
    g.input.extend(graph_inputs)
    for i, n in enumerate(outputs):
        g.output.append(_value_info('output_%d' % i, shapes.get(n)))
    return m


def export(executor, inputs, outputs, onnx_save_dir, job_name=None, opset=17, input_shapes=None):
    """Write the ONNX model of ``outputs`` (reference hetu2onnx.export signature)."""
    assert len(inputs) > 0 and len(outputs) > 0
    m = to_model(executor, inputs, outputs, job_name or 'HetutoOnnx', opset, input_shapes)
    with open(onnx_save_dir, 'wb') as f:
        f.write(m.SerializeToString())
    return m
