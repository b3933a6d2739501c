"""Framework-owned HIP streams and events (``csrc/runtime/device_api.cc`` in
``libhetu_alloc.so``; reference ``src/cuda_common/gpu_runtime.cc:61-118`` and
``python/hetu/stream.py``).

The executor's compute / H2D / D2H streams, the RCCL communicator's comm stream, the
PS staging streams and the dataloader's prefetch stream are created by
``hipStreamCreateWithPriority`` here, and their events by ``hipEventCreateWithFlags``.
torch only ever sees such a stream as a non-owning ``torch.cuda.ExternalStream`` over
the handle (``DeviceStream.torch``), for the rare library op that must be ordered on
it and for ``record_stream`` bookkeeping of the caching allocator.
"""
from __future__ import annotations

import atexit
import ctypes
import os

import torch

from . import _base
from ._base import _LIB_DIR

_PATH = os.path.join(_LIB_DIR, 'libhetu_alloc.so')
_lib = None
CREATED = {'streams': 0, 'events': 0}
# set at interpreter exit: streams / events still alive then are left to the driver (the
# HIP runtime may already be torn down when module globals are collected)
_SHUTDOWN = [False]


def _at_exit():
    _SHUTDOWN[0] = True


atexit.register(_at_exit)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(_PATH, mode=ctypes.RTLD_GLOBAL)
        P, I, I64, PP = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)
        for name, args in (('hetu_stream_create', [I, I, PP]), ('hetu_stream_destroy', [P]), ('hetu_stream_sync', [P]),
                           ('hetu_stream_query', [P]), ('hetu_event_create', [I, I, PP]), ('hetu_event_destroy', [P]),
                           ('hetu_event_record', [P, P]), ('hetu_event_sync', [P]), ('hetu_event_query', [P]),
                           ('hetu_event_elapsed', [P, P, ctypes.POINTER(ctypes.c_float)]),
                           ('hetu_stream_wait_event', [P, P]), ('hetu_memcpy_async', [P, P, I64, I, P]),
                           ('hetu_memcpy_peer_async', [P, I, P, I, I64, P]), ('hetu_memset_async', [P, I, I64, P]),
                           ('hetu_device_sync', [I]), ('hetu_stream_begin_capture', [P, I]),
                           ('hetu_stream_end_capture', [P, PP]), ('hetu_graph_instantiate', [P, PP]),
                           ('hetu_graph_launch', [P, P]), ('hetu_graph_destroy', [P]), ('hetu_graph_exec_destroy', [P]),
                           ('hetu_graph_nodes', [P, ctypes.POINTER(ctypes.c_int64)])):
            f = getattr(L, name)
            f.argtypes, f.restype = args, I
        L.hetu_error_string.argtypes, L.hetu_error_string.restype = [I], ctypes.c_char_p
        _lib = L
    return _lib


def _check(r, what):
    if r != 0:
        raise RuntimeError('HIP %s failed: %s' % (what, lib().hetu_error_string(r).decode()))


def _handle(stream):
    """raw hipStream_t of a DeviceStream, a torch stream, an int handle, or None (the
    framework's current stream of this thread)"""
    if stream is None:
        return _base.cur_stream()
    if isinstance(stream, DeviceStream):
        return stream.handle
    if isinstance(stream, int):
        return stream
    h = getattr(stream, 'handle', None)        # stream.Stream
    if h is not None and not hasattr(stream, 'cuda_stream'):
        return h
    return stream.cuda_stream


_DEFAULT_TS = {}


def _default_torch_stream(dev):
    t = _DEFAULT_TS.get(dev)
    if t is None:
        t = _DEFAULT_TS[dev] = torch.cuda.default_stream(dev)
    return t


def _set_torch(ts):
    torch._C._cuda_setStream(stream_id=ts.stream_id, device_index=ts.device_index, device_type=ts.device_type)


def _torch_view(stream):
    """(raw handle, torch stream object) of a stream argument"""
    if isinstance(stream, DeviceStream):
        return stream.handle, stream.torch
    if isinstance(stream, int):
        if stream == 0:
            return 0, _default_torch_stream(_base.cur_device())
        return stream, torch.cuda.ExternalStream(stream, device=torch.device('cuda', _base.cur_device()))
    ts = getattr(stream, 'torch_stream', None)   # stream.Stream
    if ts is not None or hasattr(stream, 'native'):
        if ts is None:
            return None, None
        return ts.cuda_stream, ts
    return stream.cuda_stream, stream


class use_stream(object):
    """``with use_stream(s):`` makes ``s`` this thread's current stream: framework kernel
    launches, device allocations and collectives read it (``_base.cur_stream``, no torch
    call), and torch's current stream follows it (``_cuda_setStream``) for the few torch
    ops that still run.  ``s``: a DeviceStream, a torch stream, a ``stream.Stream``, a raw
    handle, or None (no change).  The reference routes ops to streams per call
    (``gpu_ops/executor.py`` stream_handle arguments); here the stream is ambient."""
    __slots__ = ('h', 'ts', 'prev')

    def __init__(self, stream):
        self.h, self.ts = (None, None) if stream is None else _torch_view(stream)

    def __enter__(self):
        if self.h is None:
            self.prev = None
            return self
        tls = _base._TLS
        self.prev = (getattr(tls, 'h', 0), getattr(tls, 'ts', None))
        tls.h, tls.ts = self.h, self.ts
        _set_torch(self.ts)
        return self

    def __exit__(self, *exc):
        if self.prev is None:
            return False
        tls = _base._TLS
        h, ts = self.prev
        tls.h, tls.ts = h, ts
        _set_torch(ts if ts is not None else _default_torch_stream(self.ts.device_index))
        return False


_EDGE = {}


def stream_edge(src, dst=None):
    """``dst`` (default: the current stream) waits for the work queued so far on ``src``,
    through a cached event per source stream (no event creation per edge)"""
    h = _handle(src)
    ev = _EDGE.get(h)
    if ev is None:
        ev = _EDGE[h] = DeviceEvent()
    ev.record(src)
    ev.wait(dst)


def current_stream():
    """this thread's current stream as a raw handle (0: the null stream)"""
    return _base.cur_stream()


_PERSISTENT = []   # streams that live as long as the process (see DeviceStream(persistent=True))


class DeviceStream(object):
    """A HIP stream created by the framework (non-blocking, optional priority).
    ``persistent``: never destroyed -- for streams tensors are ``record_stream``-ed on
    (communicator, PS staging, prefetch): torch's caching allocator records events on such
    a stream when those tensors are freed, possibly after the stream's owner is gone."""

    def __init__(self, device=None, priority=0, persistent=False):
        self.persistent = persistent
        self.device = _base.cur_device() if device is None else int(device)
        h = ctypes.c_void_p()
        _check(lib().hetu_stream_create(self.device, int(priority), ctypes.byref(h)), 'stream create')
        self.handle = h.value
        self.priority = priority
        self.torch = torch.cuda.ExternalStream(self.handle, device=torch.device('cuda', self.device))
        CREATED['streams'] += 1
        if persistent:
            _PERSISTENT.append(self)

    @property
    def cuda_stream(self):
        return self.handle

    def synchronize(self):
        _check(lib().hetu_stream_sync(self.handle), 'stream sync')

    def query(self):
        return lib().hetu_stream_query(self.handle) == 0

    def wait_event(self, event):
        event.wait(self)

    def wait_stream(self, other):
        """device-side: this stream waits for the work queued so far on ``other`` (one
        cached event per stream: hipStreamWaitEvent takes the event's state at the call,
        so re-recording it for the next edge is safe)"""
        ev = getattr(self, '_edge_ev', None)
        if ev is None:
            ev = self._edge_ev = DeviceEvent(self.device)
        ev.record(other)
        ev.wait(self)

    def __del__(self):
        h = getattr(self, 'handle', None)
        if h and _lib is not None and not _SHUTDOWN[0] and not getattr(self, 'persistent', False):
            try:
                lib().hetu_stream_sync(h)
                from . import memory_pool
                memory_pool.forget_stream(self.device, h)
                lib().hetu_stream_destroy(h)
            except Exception:
                pass
            self.handle = None


class DeviceEvent(object):
    """A HIP event (timing disabled unless ``timing``: cheaper record and wait)."""

    def __init__(self, device=None, timing=False, enable_timing=None):
        if enable_timing is not None:
            timing = enable_timing
        self.device = _base.cur_device() if device is None else int(device)
        h = ctypes.c_void_p()
        _check(lib().hetu_event_create(self.device, int(bool(timing)), ctypes.byref(h)), 'event create')
        self.handle = h.value
        CREATED['events'] += 1

    def record(self, stream=None):
        _check(lib().hetu_event_record(self.handle, _handle(stream)), 'event record')
        return self

    def wait(self, stream=None):
        _check(lib().hetu_stream_wait_event(_handle(stream), self.handle), 'stream wait event')

    def synchronize(self):
        _check(lib().hetu_event_sync(self.handle), 'event sync')

    def query(self):
        return lib().hetu_event_query(self.handle) == 0

    def elapsed_time(self, end):
        """milliseconds from this event to ``end`` (both recorded, timing enabled)"""
        ms = ctypes.c_float()
        _check(lib().hetu_event_elapsed(self.handle, end.handle, ctypes.byref(ms)), 'event elapsed')
        return float(ms.value)

    def __del__(self):
        h = getattr(self, 'handle', None)
        if h and _lib is not None and not _SHUTDOWN[0]:
            try:
                lib().hetu_event_destroy(h)
            except Exception:
                pass
            self.handle = None


def memcpy_async(dst, src, nbytes, kind, stream=None):
    """kind: 'h2h' | 'h2d' | 'd2h' | 'd2d' on a framework or torch stream"""
    k = {'h2h': 0, 'h2d': 1, 'd2h': 2, 'd2d': 3}[kind]
    _check(lib().hetu_memcpy_async(dst, src, int(nbytes), k, _handle(stream)), 'memcpy')


class Graph(object):
    """A HIP graph captured from a framework stream (``hipStreamBeginCapture`` ..
    ``hipStreamEndCapture``, instantiated once, replayed with ``hipGraphLaunch``):
    the executor's replayed steady-state step when the BFC pool is the device
    allocator (its private capture pool keeps the step's buffers out of everyone
    else's reach, memory_pool.capture_pool)."""

    RELAXED = 2

    def __init__(self):
        self.graph = None
        self.exec = None

    def begin(self, stream):
        _check(lib().hetu_stream_begin_capture(_handle(stream), self.RELAXED), 'stream begin capture')

    def end(self, stream):
        g = ctypes.c_void_p()
        _check(lib().hetu_stream_end_capture(_handle(stream), ctypes.byref(g)), 'stream end capture')
        self.graph = g.value
        x = ctypes.c_void_p()
        _check(lib().hetu_graph_instantiate(self.graph, ctypes.byref(x)), 'graph instantiate')
        self.exec = x.value

    def nodes(self):
        n = ctypes.c_int64()
        _check(lib().hetu_graph_nodes(self.graph, ctypes.byref(n)), 'graph nodes')
        return int(n.value)

    def replay(self, stream=None):
        _check(lib().hetu_graph_launch(self.exec, _handle(stream)), 'graph launch')

    def __del__(self):
        try:
            if _lib is not None and not _SHUTDOWN[0]:
                if getattr(self, 'exec', None):
                    lib().hetu_graph_exec_destroy(self.exec)
                if getattr(self, 'graph', None):
                    lib().hetu_graph_destroy(self.graph)
        except Exception:
            pass
