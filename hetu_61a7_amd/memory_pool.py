"""Native memory pools (reference src/memory_pool/{allocator.h,BFC_allocator.h}
-- declared but never built there -- and gpu_ops/memory_pool.py's static plan;
SURVEY §2.2 N2/N3, §2.1 P17).

``BFCAllocator`` wraps ``libhetu_alloc.so`` (C++): best-fit-with-coalescing
over large hipMalloc / hipHostMalloc regions with stream-tagged free lists.

* ``enable_torch_bfc()`` -- called by ``import hetu_61a7_amd`` unless
  ``HETU_ALLOCATOR=torch`` -- installs the BFC allocator as the device allocator of
  the whole process through ``torch.cuda.memory.CUDAPluggableAllocator``, so every
  tensor the executor creates is carved from a few multi-GiB HBM regions and torch's
  caching allocator reserves nothing.
* ``pinned_pool()`` is the process-wide pinned-DRAM pool used for PS / HET
  cache staging buffers (``pinned_empty``).
* ``device_stats()`` mirrors the reference ``AllocatorStats``.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ._base import _LIB_DIR

_ALLOC_PATH = os.path.join(_LIB_DIR, 'libhetu_alloc.so')
_lib = None

DEVICE, PINNED_HOST, HOST, HOST_TAGGED = 0, 1, 2, 3
_STAT_KEYS = ('num_allocs', 'bytes_in_use', 'peak_bytes_in_use', 'largest_alloc_size', 'bytes_reserved',
              'bytes_limit', 'num_regions', 'num_free_chunks')


def available():
    return os.path.exists(_ALLOC_PATH)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_ALLOC_PATH):
            raise RuntimeError('libhetu_alloc.so not built (%s); run make -C csrc' % _ALLOC_PATH)
        L = ctypes.CDLL(_ALLOC_PATH, mode=ctypes.RTLD_GLOBAL)
        P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        for name, args, res in (('hetu_bfc_create', [I32, I32, I64, I64], P),
                                ('hetu_bfc_destroy', [P], None),
                                ('hetu_bfc_alloc', [P, I64, P], P),
                                ('hetu_bfc_free', [P, P, P], None),
                                ('hetu_bfc_record_stream', [P, P, P], None),
                                ('hetu_bfc_set_cache', [P, I32], None),
                                ('hetu_bfc_forget_stream', [P, P], None),
                                ('hetu_torch_forget_stream', [I32, P], None),
                                ('hetu_torch_record_stream', [I32, P, P], None),
                                ('hetu_bfc_size', [P, P], I64),
                                ('hetu_bfc_release', [P], I64),
                                ('hetu_bfc_check', [P], I32),
                                ('hetu_bfc_stats', [P, P], None),
                                ('hetu_torch_stats', [I32, P], None),
                                ('hetu_torch_pool_begin', [I32, P], I64),
                                ('hetu_torch_pool_end', [I32], None),
                                ('hetu_torch_pool_stats', [I64, P], None),
                                ('hetu_torch_pool_release', [I64], None)):
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _lib = L
    return _lib


class BFCAllocator(object):
    def __init__(self, kind=DEVICE, device=0, limit_bytes=0, first_region=1 << 30):
        self.kind = kind
        self.h = lib().hetu_bfc_create(kind, device, int(limit_bytes), int(first_region))

    def alloc(self, nbytes, stream=None):
        return lib().hetu_bfc_alloc(self.h, int(nbytes), stream)

    def free(self, ptr, stream=None):
        lib().hetu_bfc_free(self.h, ptr, stream)

    def record_stream(self, ptr, stream):
        """ptr is also used on ``stream``: held back from reuse after its free until
        that stream's work queued before the free has completed"""
        lib().hetu_bfc_record_stream(self.h, ptr, stream)

    def forget_stream(self, stream):
        """``stream`` is being destroyed (its work complete): its chunks become clean"""
        lib().hetu_bfc_forget_stream(self.h, stream)

    def set_cache(self, on):
        """exact-size reuse cache in front of the bins (on by default for device pools)"""
        lib().hetu_bfc_set_cache(self.h, int(bool(on)))

    def size_of(self, ptr):
        return lib().hetu_bfc_size(self.h, ptr)

    def release(self):
        return lib().hetu_bfc_release(self.h)

    def check(self):
        return bool(lib().hetu_bfc_check(self.h))

    def stats(self):
        out = (ctypes.c_int64 * 8)()
        lib().hetu_bfc_stats(self.h, out)
        return dict(zip(_STAT_KEYS, list(out)))

    def tensor(self, shape, dtype=torch.float32):
        """Host tensor backed by this pool (pinned for PINNED_HOST); the chunk
        returns to the pool when the tensor is garbage collected."""
        assert self.kind != DEVICE
        n = 1
        for s in shape:
            n *= int(s)
        nbytes = max(n * torch.empty((), dtype=dtype).element_size(), 1)
        ptr = self.alloc(nbytes)
        if not ptr:
            raise MemoryError('BFC pool exhausted (%d bytes)' % nbytes)
        buf = (ctypes.c_char * nbytes).from_address(ptr)
        t = torch.frombuffer(buf, dtype=torch.uint8, count=nbytes).view(dtype)[:n].view(tuple(shape))
        import weakref
        weakref.finalize(buf, self.free, ptr)
        t._hetu_pool_buf = buf     # keep the ctypes owner alive as long as the tensor
        return t

    def __del__(self):
        try:
            from .runtime import _SHUTDOWN
            # at interpreter exit the HIP runtime may already be gone: the regions go
            # back to the driver with the process
            if self.h and _lib is not None and not _SHUTDOWN[0]:
                _lib.hetu_bfc_destroy(self.h)
        except Exception:
            pass
        self.h = None


_pinned = None


def pinned_pool():
    global _pinned
    if _pinned is None:
        _pinned = BFCAllocator(PINNED_HOST if torch.cuda.is_available() else HOST, 0, 0, 256 << 20)
    return _pinned


_torch_bfc = False


def enable_torch_bfc():
    """Route every torch device allocation of this process through the native
    BFC allocator.  Must run before the first device allocation."""
    global _torch_bfc
    if _torch_bfc:
        return True
    lib()
    from torch.cuda.memory import CUDAPluggableAllocator, change_current_allocator
    change_current_allocator(CUDAPluggableAllocator(_ALLOC_PATH, 'hetu_torch_alloc', 'hetu_torch_free'))
    _torch_bfc = True
    return True


def torch_bfc_enabled():
    return _torch_bfc


def record_stream(t, stream):
    """``t.record_stream(stream)`` for whichever device allocator owns t: the BFC
    pool's own side-stream hold when it is the process allocator (torch's pluggable
    allocator interface has no record_stream hook), torch's caching allocator
    otherwise.  ``stream``: a torch stream, a runtime.DeviceStream, or a raw handle (the
    framework's current stream: ``runtime.current_stream()``)."""
    if isinstance(stream, int):
        if _torch_bfc:
            lib().hetu_torch_record_stream(t.device.index or 0, t.untyped_storage().data_ptr(), stream)
            return
        from .runtime import _torch_view
        stream = _torch_view(stream)[1]
    if _torch_bfc:
        h = stream.handle if hasattr(stream, 'handle') else stream.cuda_stream
        # the allocation's start: a view with an offset (t.data_ptr()) would miss the block
        lib().hetu_torch_record_stream(t.device.index or 0, t.untyped_storage().data_ptr(), h)
    else:
        t.record_stream(stream.torch if hasattr(stream, 'torch') and not isinstance(stream, torch.cuda.Stream)
                        else stream)


def forget_stream(device, handle):
    """a framework stream is about to be destroyed (runtime.DeviceStream.__del__, after
    synchronising it): the device allocator and the capture pools move the chunks filed
    under it to their clean bins instead of keeping a dead handle"""
    if _torch_bfc and _lib is not None:
        _lib.hetu_torch_forget_stream(int(device), handle)


def device_stats(device=0):
    out = (ctypes.c_int64 * 8)()
    lib().hetu_torch_stats(int(device), out)
    return dict(zip(_STAT_KEYS, list(out)))


class capture_pool(object):
    """``with capture_pool(device, stream) as pool:`` -- every device allocation in the
    block made on ``stream`` (or on a stream being captured) comes from a private BFC
    pool (the native graph-capture pool: a captured step's buffers are replayed by the
    graph and must never be handed to other code).
    ``pool.stats()`` mirrors device_stats; ``pool.release()`` returns its memory
    (only once the graph that uses it is gone)."""

    def __init__(self, device=0, stream=None):
        self.device = int(device)
        self.stream = stream
        self.id = None

    def __enter__(self):
        s = self.stream
        h = None if s is None else (s.handle if hasattr(s, 'handle') else s.cuda_stream)
        self.id = lib().hetu_torch_pool_begin(self.device, h)
        return self

    def __exit__(self, *exc):
        lib().hetu_torch_pool_end(self.device)
        return False

    def stats(self):
        out = (ctypes.c_int64 * 8)()
        lib().hetu_torch_pool_stats(self.id, out)
        return dict(zip(_STAT_KEYS, list(out)))

    def release(self):
        if self.id is not None:
            lib().hetu_torch_pool_release(self.id)
            self.id = None
