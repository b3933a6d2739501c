"""Native library loader (reference ``python/hetu/_base.py:15-95``).

The MI355X kernels live in ``hetu_61a7_amd/lib/libhetu_kernels.so`` (hand-written
HIP for gfx950, C ABI, built by ``__graft_entry__.build()`` / ``make -C csrc``).
The host runtime pieces (BFC pinned allocator, PS server/worker, HET cache)
live in ``libhetu_runtime.so``.

torch is imported first so that its bundled HIP runtime (soname
``libamdhip64.so.7``) is the one our libraries bind to: one HIP runtime per
process, shared streams, shared caching allocator.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the native loads, see module doc)

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib')


class NativeLibraryError(RuntimeError):
    pass


def _load(name):
    path = os.path.join(_LIB_DIR, name)
    if not os.path.exists(path):
        return None, path
    try:
        return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL), path
    except OSError as e:  # pragma: no cover - surfaced by require_*
        return e, path


if os.environ.get('HETU_KERNELS_LIB'):   # A/B runs: a kernel library built with other flags
    _KPATH = os.path.abspath(os.environ['HETU_KERNELS_LIB'])
    try:
        _KLIB = ctypes.CDLL(_KPATH, mode=ctypes.RTLD_GLOBAL) if os.path.exists(_KPATH) else None
    except OSError as _e:  # pragma: no cover
        _KLIB = _e
else:
    _KLIB, _KPATH = _load('libhetu_kernels.so')
_RLIB, _RPATH = _load('libhetu_runtime.so')


def kernels_lib():
    """Return the HIP kernel library or raise loudly (never fall back on GPU)."""
    if _KLIB is None or isinstance(_KLIB, OSError):
        raise NativeLibraryError(
            'HIP kernel library not available (%s): %s. Build it with '
            '`python -c "import __graft_entry__ as g; g.build()"` or `make -C csrc`.'
            % (_KPATH, _KLIB))
    return _KLIB


def runtime_lib():
    if _RLIB is None or isinstance(_RLIB, OSError):
        raise NativeLibraryError('native runtime library not available (%s): %s' % (_RPATH, _RLIB))
    return _RLIB


def has_kernels() -> bool:
    return _KLIB is not None and not isinstance(_KLIB, OSError)


def has_runtime() -> bool:
    return _RLIB is not None and not isinstance(_RLIB, OSError)


def check_call(ret):
    if ret != 0:
        msg = ''
        if has_kernels():
            try:
                f = _KLIB.HetuGetLastError
                f.restype = ctypes.c_char_p
                msg = f().decode()
            except AttributeError:
                pass
        raise RuntimeError('native call failed (%d): %s' % (ret, msg))


# ---- framework-owned execution state (the launch path asks torch nothing) ----
# The current HIP stream of this thread (a raw hipStream_t; 0 = the device's null stream),
# set only by ``runtime.use_stream`` (which keeps torch's current stream in step for the
# few torch ops that still run), the current device of the process and whether a GPU is
# present: read by every kernel launch and device allocation without a torch call.
import threading as _threading

_TLS = _threading.local()


def cur_stream() -> int:
    return getattr(_TLS, 'h', 0)


_GPU = [None]


def gpu_available() -> bool:
    g = _GPU[0]
    if g is None:
        g = _GPU[0] = bool(torch.cuda.is_available())
    return g


_DEV = [None]


def cur_device() -> int:
    d = _DEV[0]
    if d is None:
        d = _DEV[0] = int(torch.cuda.current_device()) if gpu_available() else 0
    return d


def set_device(d: int):
    """the process's device (torch's current device follows)"""
    d = int(d)
    torch.cuda.set_device(d)
    _DEV[0] = d
