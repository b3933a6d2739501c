"""ONNX interchange (reference python/hetu/onnx): ``hetu2onnx.export`` and
``onnx2hetu.load_onnx`` over a self-contained protobuf schema (``proto``), plus
a NumPy reference interpreter (``runtime``) used to check exported models."""
from . import proto, hetu2onnx, onnx2hetu, runtime  # noqa: F401
from .hetu2onnx import export  # noqa: F401
from .onnx2hetu import load_onnx, from_onnx  # noqa: F401
