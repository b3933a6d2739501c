"""ONNX protobuf messages without the ``onnx`` package.

The reference needs ``onnx`` (+ onnxruntime in its tests, python/hetu/onnx/
hetu2onnx.py:19-24); neither is installed here, so the subset of onnx.proto the
exporter/importer use is declared at run time through protobuf descriptors
with the official field numbers -- files written here are regular ONNX model
files, and real ``.onnx`` files parse with these classes.  If the ``onnx``
package is importable its classes are used instead.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool

try:  # pragma: no cover - not installed in this image
    from google.protobuf import message_factory as _mf
except ImportError:  # pragma: no cover
    _mf = None

# TensorProto.DataType
FLOAT, UINT8, INT8, UINT16, INT16, INT32, INT64, STRING, BOOL, FLOAT16, DOUBLE = 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11
BFLOAT16 = 16
# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_GRAPH, A_FLOATS, A_INTS, A_STRINGS = 1, 2, 3, 4, 5, 6, 7, 8

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
_T = {'int64': _F.TYPE_INT64, 'int32': _F.TYPE_INT32, 'float': _F.TYPE_FLOAT, 'double': _F.TYPE_DOUBLE,
      'string': _F.TYPE_STRING, 'bytes': _F.TYPE_BYTES, 'uint64': _F.TYPE_UINT64, 'msg': _F.TYPE_MESSAGE,
      'enum': _F.TYPE_ENUM}

# (message, [(field, number, label, type, type_name)])  -- numbers from onnx/onnx.proto
_SCHEMA = [
    ('AttributeProto', [('name', 1, _OPT, 'string', None), ('ref_attr_name', 21, _OPT, 'string', None),
                        ('doc_string', 13, _OPT, 'string', None), ('type', 20, _OPT, 'int32', None),
                        ('f', 2, _OPT, 'float', None), ('i', 3, _OPT, 'int64', None), ('s', 4, _OPT, 'bytes', None),
                        ('t', 5, _OPT, 'msg', 'TensorProto'), ('g', 6, _OPT, 'msg', 'GraphProto'),
                        ('floats', 7, _REP, 'float', None), ('ints', 8, _REP, 'int64', None),
                        ('strings', 9, _REP, 'bytes', None), ('tensors', 10, _REP, 'msg', 'TensorProto'),
                        ('graphs', 11, _REP, 'msg', 'GraphProto')]),
    ('ValueInfoProto', [('name', 1, _OPT, 'string', None), ('type', 2, _OPT, 'msg', 'TypeProto'),
                        ('doc_string', 3, _OPT, 'string', None)]),
    ('NodeProto', [('input', 1, _REP, 'string', None), ('output', 2, _REP, 'string', None),
                   ('name', 3, _OPT, 'string', None), ('op_type', 4, _OPT, 'string', None),
                   ('domain', 7, _OPT, 'string', None), ('attribute', 5, _REP, 'msg', 'AttributeProto'),
                   ('doc_string', 6, _OPT, 'string', None)]),
    ('StringStringEntryProto', [('key', 1, _OPT, 'string', None), ('value', 2, _OPT, 'string', None)]),
    ('OperatorSetIdProto', [('domain', 1, _OPT, 'string', None), ('version', 2, _OPT, 'int64', None)]),
    ('ModelProto', [('ir_version', 1, _OPT, 'int64', None), ('opset_import', 8, _REP, 'msg', 'OperatorSetIdProto'),
                    ('producer_name', 2, _OPT, 'string', None), ('producer_version', 3, _OPT, 'string', None),
                    ('domain', 4, _OPT, 'string', None), ('model_version', 5, _OPT, 'int64', None),
                    ('doc_string', 6, _OPT, 'string', None), ('graph', 7, _OPT, 'msg', 'GraphProto'),
                    ('metadata_props', 14, _REP, 'msg', 'StringStringEntryProto')]),
    ('GraphProto', [('node', 1, _REP, 'msg', 'NodeProto'), ('name', 2, _OPT, 'string', None),
                    ('initializer', 5, _REP, 'msg', 'TensorProto'), ('doc_string', 10, _OPT, 'string', None),
                    ('input', 11, _REP, 'msg', 'ValueInfoProto'), ('output', 12, _REP, 'msg', 'ValueInfoProto'),
                    ('value_info', 13, _REP, 'msg', 'ValueInfoProto')]),
    ('TensorProto', [('dims', 1, _REP, 'int64', None), ('data_type', 2, _OPT, 'int32', None),
                     ('float_data', 4, _REP, 'float', None), ('int32_data', 5, _REP, 'int32', None),
                     ('string_data', 6, _REP, 'bytes', None), ('int64_data', 7, _REP, 'int64', None),
                     ('name', 8, _OPT, 'string', None), ('doc_string', 12, _OPT, 'string', None),
                     ('raw_data', 9, _OPT, 'bytes', None), ('double_data', 10, _REP, 'double', None),
                     ('uint64_data', 11, _REP, 'uint64', None)]),
    ('TensorShapeProto', [('dim', 1, _REP, 'msg', 'TensorShapeProto.Dimension')]),
    ('TensorShapeProto.Dimension', [('dim_value', 1, _OPT, 'int64', None), ('dim_param', 2, _OPT, 'string', None),
                                    ('denotation', 3, _OPT, 'string', None)]),
    ('TypeProto', [('tensor_type', 1, _OPT, 'msg', 'TypeProto.Tensor'), ('denotation', 6, _OPT, 'string', None)]),
    ('TypeProto.Tensor', [('elem_type', 1, _OPT, 'int32', None), ('shape', 2, _OPT, 'msg', 'TensorShapeProto')]),
]

_PKG = 'onnx'
_classes = None


def _build():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = 'hetu_onnx_subset.proto'
    fdp.package = _PKG
    fdp.syntax = 'proto2'
    top = {}
    for name, fields in _SCHEMA:
        parts = name.split('.')
        if len(parts) == 1:
            m = fdp.message_type.add()
            m.name = name
            top[name] = m
        else:
            m = top[parts[0]].nested_type.add()
            m.name = parts[1]
        for fname, num, label, typ, tname in fields:
            f = m.field.add()
            f.name, f.number, f.label, f.type = fname, num, label, _T[typ]
            if tname:
                f.type_name = '.%s.%s' % (_PKG, tname)
            if label == _REP and fname.endswith('_data') and typ != 'bytes':   # [packed = true] in onnx.proto
                f.options.packed = True
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    out = {}
    for name, _ in _SCHEMA:
        d = pool.FindMessageTypeByName('%s.%s' % (_PKG, name))
        if hasattr(_mf, 'GetMessageClass'):
            out[name] = _mf.GetMessageClass(d)
        else:  # pragma: no cover - older protobuf
            out[name] = _mf.MessageFactory(pool).GetPrototype(d)
    return out


def classes():
    """{'ModelProto': cls, ...} -- from the ``onnx`` package when present."""
    global _classes
    if _classes is None:
        try:  # pragma: no cover
            import onnx
            _classes = {n.split('.')[0]: getattr(onnx, n.split('.')[0]) for n, _ in _SCHEMA if '.' not in n}
        except ImportError:
            _classes = _build()
    return _classes


def ModelProto():
    return classes()['ModelProto']()


def parse_model(data: bytes):
    m = ModelProto()
    m.ParseFromString(data)
    return m
