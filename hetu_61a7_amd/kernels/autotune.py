"""Per-shape kernel selection by measurement.

``choose(key, {name: fn})`` times every candidate once per key (events on the
current stream; after two warm calls, interleaved rounds of a few repetitions,
best round per candidate) and caches the fastest.
Used to pick, per convolution / GEMM shape, among the hand-written kernels (tile
shapes, split-K depths, K-loop forms).  Never measures inside a hipGraph capture
(returns the first candidate there; warm-up steps run eagerly before capture).

Decisions persist across processes: ``save(path)`` writes them as JSON (keys by ``repr``),
and ``HETU_AUTOTUNE_CACHE=path`` (or ``load(path)``) makes a later process take them
without measuring -- a production job skips its tuning steps, and a profiling run whose
serialised dispatches would time candidates differently (``rocprofv3 --pmc``) runs the
kernels the plain run chose.
"""
from __future__ import annotations

import os

import torch  # noqa: F401

from ..runtime import DeviceEvent

_decisions = {}
_times = {}
_loaded = {}     # repr(key) -> candidate name, from a saved cache
REPS = int(os.environ.get('HETU_AUTOTUNE_REPS', '5'))
ROUNDS = int(os.environ.get('HETU_AUTOTUNE_ROUNDS', '3'))


def _gpu():
    from .._base import gpu_available
    return gpu_available()


def _capturing():
    from ..utils.hipgraph import capturing
    return capturing()


def choose(key, candidates, mode=None):
    """the fastest candidate for ``key`` (cached); candidates return None for shapes they
    do not take.  (``mode`` is ignored: every candidate is a hand-written kernel.)"""
    d = _decisions.get(key)
    if d is not None and d in candidates:
        return d
    if _loaded:
        d = _loaded.get(repr(key))
        if d is not None and d in candidates:
            _decisions[key] = d
            return d
    names = list(candidates)
    from . import deterministic
    if deterministic():
        # fixed choice: the first hand-written kernel (in the order every call site lists
        # them) that takes the shape
        if _gpu() and not _capturing():
            for n in names:
                if candidates[n]() is not None:
                    _decisions[key] = n
                    return n
        return names[0]
    if len(names) == 1 or not _gpu() or _capturing():
        return names[0]
    live = []
    for n in names:
        f = candidates[n]
        if f() is None:  # unsupported shape
            continue
        f()  # second warm call: first-use code-object loads
        live.append(n)
    # ROUNDS interleaved rounds (a, b, c, a, b, c, ...) of REPS calls each; a
    # candidate's time is its best round, so a clock / co-tenant dip during one
    # candidate's window does not decide the choice
    times = {}
    for _ in range(ROUNDS):
        for n in live:
            f = candidates[n]
            s, e = DeviceEvent(timing=True), DeviceEvent(timing=True)
            s.record()
            for _ in range(REPS):
                f()
            e.record()
            e.synchronize()
            t = s.elapsed_time(e) / REPS
            times[n] = min(times.get(n, t), t)
    if times:
        best = min(times, key=times.get)
    else:
        best = names[0]      # no candidate takes the shape: the caller raises NoKernelError
    _decisions[key] = best
    _times[key] = times
    return best


def report():
    """{key: (chosen, {candidate: ms})} -- for profiles/ and logs."""
    return {k: (_decisions[k], _times.get(k, {})) for k in _decisions}


def dump(path):
    with open(path, 'w') as f:
        for k, (c, t) in report().items():
            f.write('%s -> %s  %s\n' % (k, c, ' '.join('%s=%.1fus' % (n, v * 1e3) for n, v in t.items())))


def save(path):
    """the decisions so far as JSON {repr(key): candidate}"""
    import json
    with open(path, 'w') as f:
        json.dump({repr(k): v for k, v in _decisions.items()}, f, indent=0, sort_keys=True)


def load(path):
    """take the decisions of a saved cache (measured choices of this process win)"""
    import json
    with open(path) as f:
        _loaded.update(json.load(f))
    return len(_loaded)


if os.environ.get('HETU_AUTOTUNE_CACHE') and os.path.exists(os.environ['HETU_AUTOTUNE_CACHE']):
    load(os.environ['HETU_AUTOTUNE_CACHE'])
