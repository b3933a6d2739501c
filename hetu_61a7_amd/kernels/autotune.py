"""Per-shape kernel selection by measurement.

``choose(key, {name: fn})`` times every candidate once per key (events on the
current stream; after two warm calls, interleaved rounds of a few repetitions,
best round per candidate) and caches the fastest.
Used to pick, per convolution / GEMM shape, between the hand-written MFMA
kernels and the vendor library, so a hand-written kernel runs wherever it is at
least as fast (within ``NATIVE_BIAS``, 3 %, of the fastest library candidate).  Never measures inside a hipGraph capture (returns the
first candidate there; warm-up steps run eagerly before capture).
"""
from __future__ import annotations

import os

import torch

_decisions = {}
_times = {}
REPS = int(os.environ.get('HETU_AUTOTUNE_REPS', '5'))
ROUNDS = int(os.environ.get('HETU_AUTOTUNE_ROUNDS', '3'))
# tie-break toward the hand-written kernels: taken when within this fraction of the fastest
# library candidate (HETU_AUTOTUNE_NATIVE_BIAS=0 restores the strict minimum)
NATIVE_BIAS = float(os.environ.get('HETU_AUTOTUNE_NATIVE_BIAS', '0.03'))


def _hand_written(name):
    return name.startswith('hip')


def choose(key, candidates, mode='auto'):
    """``mode``: 'auto' times every candidate; 'hip' only the hand-written ones (names
    starting with ``hip``); a library candidate is then the last resort for a shape no
    hand-written kernel takes, counted in ``kernels.FALLBACKS``; 'vendor' picks the
    first library candidate."""
    d = _decisions.get(key)
    if d is not None:
        return d
    names = list(candidates)
    library = [n for n in names if not _hand_written(n)]
    if mode == 'vendor':
        return library[0] if library else names[0]
    if mode == 'hip':
        hw = [n for n in names if _hand_written(n)]
        if hw:
            names = hw
    from . import deterministic
    if deterministic():
        # fixed choice: the first hand-written kernel (in the order every call site lists
        # them) that takes the shape
        if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
            for n in names:
                if candidates[n]() is not None:
                    _decisions[key] = n
                    return n
        return names[0]
    if len(names) == 1 or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        return names[0]
    live = []
    for n in names:
        f = candidates[n]
        if f() is None:  # unsupported shape
            continue
        f()  # second warm call: first-use library heuristics / code-object loads
        live.append(n)
    # ROUNDS interleaved rounds (a, b, c, a, b, c, ...) of REPS calls each; a
    # candidate's time is its best round, so a clock / co-tenant dip during one
    # candidate's window does not decide the choice
    times = {}
    for _ in range(ROUNDS):
        for n in live:
            f = candidates[n]
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(REPS):
                f()
            e.record()
            e.synchronize()
            t = s.elapsed_time(e) / REPS
            times[n] = min(times.get(n, t), t)
    if times:
        best = min(times, key=times.get)
        # a hand-written kernel within NATIVE_BIAS of the fastest library candidate is taken:
        # timing noise does not hand shapes the native path serves as well to the vendor library
        hw = [n for n in times if _hand_written(n)]
        if hw and not _hand_written(best):
            h = min(hw, key=times.get)
            if times[h] <= times[best] * (1.0 + NATIVE_BIAS):
                best = h
    elif mode == 'hip' and library:
        from . import record_fallback
        record_fallback('%s: no hand-written kernel' % (key[0],))
        best = library[0]
    else:
        best = names[-1]
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
