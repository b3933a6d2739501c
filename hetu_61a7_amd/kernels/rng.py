"""Graph-safe random state (``csrc/kernels/random.hip``).

The reference draws a fresh host seed per forward call (``gpu_ops/Dropout.py:24-26``)
and passes it by value to the kernel.  A captured hipGraph would replay that one seed
forever.  Here the randomness has two parts:

* the host seed of a launch, ``next_seed(key)``: a fixed function of the executor's
  base seed, the op (``key``) and the call's index within the step -- identical on every
  step, so the captured launch arguments stay valid;
* a per-device step counter in HBM that every seeded kernel adds into its Philox key
  (``common.h rng_seed``).  The first seeded op of each step advances it with a
  one-thread kernel on the step's stream; under capture that kernel is part of the
  graph, so every replay advances it and draws fresh masks.

Eager and replayed steps therefore draw exactly the same masks (the GPU test compares
their losses), and the backward of a step regenerates the forward's mask from the saved
host seed and the unchanged counter.  On the CPU (no device counter) the step index is
folded into the host seed instead.
"""
from __future__ import annotations

import torch

from .. import _base
from . import fn, check, stream_ptr, P, I64, I32, F32

_BASE = [1234]
_EPOCH = [0]          # host step index (bumped by the executors at every step start)
_EPOCH0 = [0]         # _EPOCH at the last set_base_seed
_ADVANCED = {}        # device -> epoch its counter was last advanced for
_CALLS = {}           # key -> draws in the current step
_CTR = {}             # device -> int64 [1] device counter (kept alive for the process)
_M64 = (1 << 64) - 1
from ..utils.hipgraph import _HOST_RANDOM  # noqa: E402


def _mix(x):
    """splitmix64 finaliser"""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def effective_seed(seed, device=None):
    """the Philox key a kernel launched now with host seed ``seed`` uses (reads the device
    counter: a host sync -- tests and CPU references only)"""
    d = _base.cur_device() if device is None else int(device)
    c = _CTR.get(d)
    off = int(c.cpu()[0]) if c is not None else 0
    return (int(seed) + off * 0x9E3779B97F4A7C15) & _M64


def set_base_seed(seed):
    """a new executor's random stream: base seed ``seed``, the step counters restart at 0
    (so an executor's masks depend on its seed and step index alone)"""
    _BASE[0] = int(seed) & _M64
    _EPOCH0[0] = _EPOCH[0]               # CPU seeds mix in the step index since this point
    _ADVANCED.clear()
    for c in _CTR.values():
        c.zero_()


def new_step():
    """a training / evaluation step begins (SubExecutor / pipeline executor)"""
    _EPOCH[0] += 1
    _CALLS.clear()


def epoch():
    return _EPOCH[0]


def counter(device=None):
    """the device's step counter (registered with the kernel library on first use)"""
    d = _base.cur_device() if device is None else int(device)
    c = _CTR.get(d)
    if c is None:
        from .. import native_array as _NA
        c = _NA.zeros(1, dtype=torch.int64, device=torch.device('cuda', d))
        check(fn('hetu_rng_register', [I32, P])(d, c.data_ptr()), 'rng_register')
        _CTR[d] = c
    return c


def advance(by=1, device=None):
    """counter += by on the current stream (captured with the step)"""
    c = counter(device)
    check(fn('hetu_rng_advance', [P, I64, P])(c.data_ptr(), int(by), stream_ptr()), 'rng_advance')


def next_seed(key, on_gpu=True):
    """host seed of the next draw of op ``key`` in this step (never 0: 0 means 'no
    dropout' to the gradient ops).  On the GPU the first draw of a step advances the
    device counter first."""
    e = _EPOCH[0]
    if on_gpu:
        d = _base.cur_device()
        if _ADVANCED.get(d) != e:
            advance(1, d)
            _ADVANCED[d] = e
    c = _CALLS.get(key, 0)
    _CALLS[key] = c + 1
    _HOST_RANDOM[0] += 1
    s = _mix(_BASE[0] ^ _mix((int(key) << 20) ^ c))
    if not on_gpu:
        s = _mix(s ^ (e - _EPOCH0[0]))   # no device counter: the step varies the seed
    s &= (1 << 63) - 1                   # int64 launch argument
    return s or 1


# ---- random fills / channel dropout ---------------------------------------------------------
def uniform_(t, lo=0.0, hi=1.0, seed=None, key=0):
    """t ~ U[lo, hi) in place (fp32 / bf16 device tensor, contiguous)"""
    seed = next_seed(key) if seed is None else seed
    check(fn('hetu_uniform', [P, I64, F32, F32, I64, I32, P])(
        t.data_ptr(), t.numel(), float(lo), float(hi), int(seed), 1 if t.dtype == torch.bfloat16 else 0,
        stream_ptr()), 'uniform')
    return t


def normal_(t, mean=0.0, std=1.0, trunc=0.0, seed=None, key=0):
    """t ~ N(mean, std) in place; trunc > 0 redraws values beyond trunc * std"""
    seed = next_seed(key) if seed is None else seed
    check(fn('hetu_normal', [P, I64, F32, F32, F32, I64, I32, P])(
        t.data_ptr(), t.numel(), float(mean), float(std), float(trunc), int(seed),
        1 if t.dtype == torch.bfloat16 else 0, stream_ptr()), 'normal')
    return t


def dropout2d(x, keep, seed):
    """channel dropout of an [N, C, H, W] device tensor (NCHW or channels-last memory):
    plane (n, c) kept with probability ``keep``, scaled by 1 / keep"""
    from .. import native_array as _NA
    n, c = int(x.shape[0]), int(x.shape[1])
    hw = int(x[0, 0].numel()) if x.dim() > 2 else 1
    cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
    if not cl:
        x = x.contiguous()
    y = _NA.empty(tuple(x.shape), dtype=x.dtype, device=x.device,
                  memory_format=torch.channels_last if cl else None)
    check(fn('hetu_dropout2d', [P, P, I64, I32, I64, I32, F32, I64, I32, P])(
        x.data_ptr(), y.data_ptr(), x.numel(), c, hw, 1 if cl else 0, float(keep), int(seed),
        1 if x.dtype == torch.bfloat16 else 0, stream_ptr()), 'dropout2d')
    return y


def arange(n, start, step, dtype=torch.float32, device='cuda'):
    from .. import native_array as _NA
    y = _NA.empty(int(n), dtype=dtype, device=device)
    check(fn('hetu_arange', [P, I64, ctypes_double(), ctypes_double(), I32, P])(
        y.data_ptr(), int(n), float(start), float(step), 1 if dtype == torch.bfloat16 else 0, stream_ptr()),
        'arange')
    return y


def ctypes_double():
    import ctypes
    return ctypes.c_double
