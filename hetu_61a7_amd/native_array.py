"""Framework-owned strided arrays over the native array runtime (``csrc/runtime/array.cc``,
in ``libhetu_alloc.so``): the reference's DLArray C ABI (``src/common/dlarray.h:18-66``,
``c_runtime_api.cc:93-142`` DLArrayAlloc / Free / CopyFromTo).

An ``Array`` is a refcounted native header -- data, byte offset, device, dtype, shape,
strides -- over memory from the framework's own pools: the BFC HBM pool of the device
(the same pool torch's pluggable-allocator hook draws from), the pinned-host BFC pool,
or host memory.  Views (reshape / transpose / slice / broadcast) share the allocation.
``Array.torch()`` exports a DLPack capsule that torch wraps without copying or owning:
the tensor's deleter drops one native reference, and the last reference returns the
memory to its pool.  ``empty`` / ``zeros`` / ``empty_like`` are the framework's
allocation entry points for executor buffers and kernel outputs.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _base

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.float64: 6, torch.int8: 7, torch.bool: 8}
_DT_INV = {v: k for k, v in _DT.items()}
MAX_DIM = 8
_lib = None
_AVAILABLE = [None]
STATS = {'arrays': 0, 'torch_views': 0}

# torch's raw capsule importer (torch.utils.dlpack.from_dlpack adds ~2 us of protocol checks)
_from_dlpack = getattr(torch._C, '_from_dlpack', None) or torch.utils.dlpack.from_dlpack

_capsule_new = ctypes.pythonapi.PyCapsule_New
_capsule_new.restype = ctypes.py_object
_capsule_new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def lib():
    global _lib
    if _lib is None:
        from .memory_pool import lib as alloc_lib
        L = alloc_lib()
        P, I32, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        for name, args, res in (
                ('hetu_array_empty', [I32, P, I32, I32, I32, I32, P, P], I32),
                ('hetu_array_view', [P, I32, P, P, I64, P], I32),
                ('hetu_array_retain', [P], None),
                ('hetu_array_release', [P], None),
                ('hetu_array_info', [P, P, P, P, P, P, P, P], I32),
                ('hetu_array_copy', [P, P, P], I32),
                ('hetu_array_to_dlpack', [P], P),
                ('hetu_array_from_dlpack', [P, I32, P], I32),
                ('hetu_array_stats', [P], None)):
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _lib = L
    return _lib


_fast = [None]


def _fastmod():
    """the CPython extension _hetu_array (csrc/runtime/pyarray.cc) or False"""
    if _fast[0] is None:
        _fast[0] = False
        try:
            import importlib.util
            import sysconfig
            path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib',
                                '_hetu_array' + sysconfig.get_config_var('EXT_SUFFIX'))
            if os.path.exists(path):
                lib()      # libhetu_alloc.so loaded first (RTLD_GLOBAL)
                spec = importlib.util.spec_from_file_location('_hetu_array', path)
                m = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(m)
                _fast[0] = m
        except (ImportError, OSError):
            _fast[0] = False
    return _fast[0]


def available():
    if _AVAILABLE[0] is None:
        try:
            lib()
            _AVAILABLE[0] = os.environ.get('HETU_NATIVE_ARRAYS', '1') != '0'
        except (RuntimeError, OSError, AttributeError):
            _AVAILABLE[0] = False
    return _AVAILABLE[0]


def _i64(xs):
    return (ctypes.c_int64 * max(len(xs), 1))(*[int(x) for x in xs])


class Array(object):
    """A native strided array (owns one reference to its header)."""

    __slots__ = ('h', '__weakref__')

    def __init__(self, handle):
        self.h = handle

    # -- creation ---------------------------------------------------------------------
    @classmethod
    def empty(cls, shape, dtype=torch.float32, device='cpu', stream=None, pinned=False):
        device = torch.device(device)
        shape = tuple(int(s) for s in shape)
        h = ctypes.c_void_p()
        dev_type = 2 if device.type == 'cuda' else 1
        dev_id = (device.index if device.index is not None else _base.cur_device()) if dev_type == 2 else 0
        if dev_type == 2 and stream is None:
            stream = _base.cur_stream()
        rc = lib().hetu_array_empty(len(shape), _i64(shape), _DT[dtype], dev_type, dev_id, int(bool(pinned)),
                                    stream, ctypes.byref(h))
        if rc == 2:
            raise MemoryError('hetu_array_empty: out of memory (%s %s on %s)' % (shape, dtype, device))
        if rc != 0:
            raise ValueError('hetu_array_empty(%s, %s) failed (%d)' % (shape, dtype, rc))
        STATS['arrays'] += 1
        return cls(h.value)

    @classmethod
    def from_torch(cls, t):
        """borrow a torch tensor's memory (DLPack; the array keeps the tensor alive)"""
        cap = torch.utils.dlpack.to_dlpack(t)
        ptr = ctypes.pythonapi.PyCapsule_GetPointer
        ptr.restype, ptr.argtypes = ctypes.c_void_p, [ctypes.py_object, ctypes.c_char_p]
        m = ptr(cap, b'dltensor')
        ctypes.pythonapi.PyCapsule_SetName.argtypes = [ctypes.py_object, ctypes.c_char_p]
        ctypes.pythonapi.PyCapsule_SetName(cap, b'used_dltensor')     # ownership moves to the array
        h = ctypes.c_void_p()
        if lib().hetu_array_from_dlpack(m, _DT[t.dtype], ctypes.byref(h)) != 0:
            raise ValueError('hetu_array_from_dlpack failed')
        return cls(h.value)

    # -- header -----------------------------------------------------------------------
    def info(self):
        data, nd, dt, dtp, did = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        shp, st = (ctypes.c_int64 * MAX_DIM)(), (ctypes.c_int64 * MAX_DIM)()
        lib().hetu_array_info(self.h, ctypes.byref(data), ctypes.byref(nd), shp, st, ctypes.byref(dt),
                              ctypes.byref(dtp), ctypes.byref(did))
        n = nd.value
        return {'data': data.value or 0, 'shape': tuple(shp[:n]), 'strides': tuple(st[:n]),
                'dtype': _DT_INV[dt.value], 'device': ('cuda:%d' % did.value) if dtp.value == 2 else 'cpu'}

    @property
    def shape(self):
        return self.info()['shape']

    @property
    def data_ptr(self):
        return self.info()['data']

    # -- views / copies -----------------------------------------------------------------
    def view(self, shape, strides, byte_offset=0):
        h = ctypes.c_void_p()
        rc = lib().hetu_array_view(self.h, len(shape), _i64(shape), _i64(strides), int(byte_offset), ctypes.byref(h))
        if rc != 0:
            raise ValueError('hetu_array_view out of bounds (%s, %s, +%d)' % (shape, strides, byte_offset))
        return Array(h.value)

    def reshape(self, shape):
        inf = self.info()
        n = 1
        for s in inf['shape']:
            n *= s
        shape = list(shape)
        if -1 in shape:
            k = shape.index(-1)
            rest = 1
            for i, s in enumerate(shape):
                if i != k:
                    rest *= s
            shape[k] = n // rest
        st, acc = [0] * len(shape), 1
        for d in range(len(shape) - 1, -1, -1):
            st[d] = acc
            acc *= shape[d]
        return self.view(shape, st)

    def broadcast_to(self, shape):
        """stride-0 view (reference NDArray.broadcast_to, ndarray.py:298-381)"""
        inf = self.info()
        s0, st0 = inf['shape'], inf['strides']
        lead = len(shape) - len(s0)
        st = [0] * lead + [st0[i] if s0[i] == shape[lead + i] else 0 for i in range(len(s0))]
        return self.view(shape, st)

    def copy_from(self, src, stream=None):
        if stream is None and _base.gpu_available():
            stream = _base.cur_stream()
        rc = lib().hetu_array_copy(self.h, src.h, stream)
        if rc == 4:     # general strides: the device copy kernel through torch views
            from .kernels.tensor import copy_into
            copy_into(self.torch(), src.torch())
            return self
        if rc != 0:
            raise RuntimeError('hetu_array_copy failed (%d)' % rc)
        return self

    # -- export -------------------------------------------------------------------------
    def torch(self):
        """a torch tensor over this array's memory (DLPack, zero copy, non-owning)"""
        m = lib().hetu_array_to_dlpack(self.h)
        STATS['torch_views'] += 1
        return _from_dlpack(_capsule_new(m, b'dltensor', None))

    def __del__(self):
        h = getattr(self, 'h', None)
        if h and _lib is not None:
            try:
                _lib.hetu_array_release(h)
            except Exception:
                pass
            self.h = None


def stats():
    out = (ctypes.c_int64 * 3)()
    lib().hetu_array_stats(out)
    return {'live_arrays': out[0], 'live_allocations': out[1], 'created': out[2]}


# ---- allocation entry points (executor buffers, kernel outputs) -------------------------
def _cl_strides(shape):
    n, c, h, w = shape
    return (h * w * c, 1, w * c, c)


_CL = torch.channels_last
_CUDA = torch.device('cuda')


def _shape(size):
    if len(size) == 1:
        s0 = size[0]
        ty = type(s0)
        if ty is tuple:
            return s0
        if ty is torch.Size or ty is list:
            return tuple(s0)
        return (int(s0),)
    return size


_BFC = [None]
_CPU = torch.device('cpu')


def _device_ok(device):
    """device arrays share the BFC pool of the pluggable-allocator hook: with torch's own
    caching allocator in charge (HETU_ALLOCATOR=torch) device memory stays torch's"""
    if device.type != 'cuda':
        return True
    if _BFC[0] is None:
        from . import memory_pool
        if not memory_pool.torch_bfc_enabled():
            return False      # (not cached: the pool may still be installed later)
        _BFC[0] = True
    return _BFC[0]


def empty(*size, dtype=torch.float32, device=None, memory_format=None, pinned=False, pin_memory=False,
          requires_grad=False):
    """``torch.empty`` signature, framework-owned memory: a torch view (DLPack, zero copy) of
    a new native array (channels_last: an NHWC allocation seen as NCHW).  The hot path is
    one call into the CPython extension plus torch's capsule import (~2 us, below
    torch.empty's own cost)."""
    shape = _shape(size)
    pinned = pinned or pin_memory
    if device is None:
        device = _CPU
    elif type(device) is not torch.device:
        device = torch.device(device)
    fm = _fast[0]
    if fm is None:
        fm = _fastmod() if available() else False
    if fm is False or not _AVAILABLE[0] or not _device_ok(device):
        kw = {'memory_format': memory_format} if memory_format is not None else {}
        t = torch.empty(shape, dtype=dtype, device=device, **kw)
        return t.pin_memory() if pinned and not t.is_cuda and _base.gpu_available() else t
    cl = memory_format is _CL and len(shape) == 4
    if cl:
        shape = (shape[0], shape[2], shape[3], shape[1])
    if device.type == 'cuda':
        idx = device.index if device.index is not None else _base.cur_device()
        cap = fm.empty(shape, _DT[dtype], 2, idx, 0, _base.cur_stream())
    else:
        cap = fm.empty(shape, _DT[dtype], 1, 0, 1 if (pinned and _base.gpu_available()) else 0, 0)
    STATS['arrays'] += 1
    t = _from_dlpack(cap)
    return t.permute(0, 3, 1, 2) if cl else t


def zeros(*size, dtype=torch.float32, device=None, memory_format=None):
    t = empty(*size, dtype=dtype, device=device, memory_format=memory_format)
    if t.numel():
        if t.is_cuda:
            from .kernels.tensor import fill_
            base = t.permute(0, 2, 3, 1) if (t.dim() == 4 and not t.is_contiguous()) else t
            fill_(base, 0)
        else:
            t.zero_()
    return t


def empty_like(t, dtype=None, device=None, memory_format=None):
    """same shape, dtype (or ``dtype``), device and dense layout (contiguous or channels-last)"""
    dtype = dtype or t.dtype
    if memory_format is None or memory_format == torch.preserve_format:
        memory_format = torch.channels_last if (t.dim() == 4 and not t.is_contiguous() and
                                                t.is_contiguous(memory_format=torch.channels_last)) else None
    return empty(t.shape, dtype=dtype, device=device or t.device, memory_format=memory_format)


def zeros_like(t, dtype=None):
    z = empty_like(t, dtype=dtype)
    if z.numel():
        if z.is_cuda:
            from .kernels.tensor import fill_
            fill_(z.permute(0, 2, 3, 1) if (z.dim() == 4 and not z.is_contiguous()) else z, 0)
        else:
            z.zero_()
    return z
