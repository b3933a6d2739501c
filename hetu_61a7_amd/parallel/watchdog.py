"""RCCL watchdog (SURVEY §5.3 "failure detection"): turns a dead peer or an RCCL
asynchronous error into a non-zero process exit, so ``heturun --max-restarts`` relaunches
the group and the workers resume from the last committed snapshot.

The reference blocks in ``ncclCommGetAsyncError``-less collectives and host-syncs every
comm event (``src/communication/mpi_nccl_communication.cu:137-143,313-324``,
``gpu_ops/executor.py:1034-1036``); a peer that dies leaves every other rank parked in
that sync forever.  Here every collective issued through the in-house communicator
(``parallel/rccl.py``) records a completion event that the watchdog tracks with a
deadline, and one daemon thread per process:

* polls ``ncclCommGetAsyncError`` (``hcomm_async_error``) of every live communicator;
* polls the error word of the one-shot IPC all-reduce (host-mapped, no GPU call);
* queries the completion event of every in-flight collective, and fails the process
  when one is older than ``HETU_COMM_TIMEOUT`` seconds (default 1800).

On failure it prints the stuck collective (op, element count, dtype, the caller's label --
the optimizer labels its gradient buckets), aborts every communicator (``ncclCommAbort``
unblocks kernels spinning on a dead peer) and ``os._exit``s with ``HETU_WATCHDOG_EXIT``
(default 75).  ``HETU_WATCHDOG=0`` disables it.  Communicators only need
``async_error()`` and ``abort()``, so the CPU tests drive it with fake ones.
"""
from __future__ import annotations

import collections
import os
import sys
import threading
import time
import weakref

EXIT_CODE = int(os.environ.get('HETU_WATCHDOG_EXIT', '75'))
_TLS = threading.local()


class labelled(object):
    """``with watchdog.labelled('grad bucket 3/12'):`` -- collectives issued inside carry
    the label into the watchdog's report."""
    __slots__ = ('text', 'prev')

    def __init__(self, text):
        self.text = text

    def __enter__(self):
        self.prev = getattr(_TLS, 'label', None)
        _TLS.label = self.text
        return self

    def __exit__(self, *exc):
        _TLS.label = self.prev
        return False


def current_label():
    return getattr(_TLS, 'label', None)


class _Pending(object):
    __slots__ = ('t0', 'event', 'what', 'label', 'comm')

    def __init__(self, t0, event, what, label, comm):
        self.t0, self.event, self.what, self.label, self.comm = t0, event, what, label, comm

    def describe(self, now):
        s = '%s on %s, in flight %.1f s' % (self.what, self.comm, now - self.t0)
        return s + (' [%s]' % self.label if self.label else '')


class Watchdog(object):
    """One monitor thread per process (``get()``); ``on_failure`` (tests) replaces the
    abort-and-exit action."""

    def __init__(self, timeout_s=None, poll_s=None, on_failure=None):
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get('HETU_COMM_TIMEOUT', '1800'))
        self.poll_s = float(poll_s if poll_s is not None else os.environ.get('HETU_WATCHDOG_POLL', '1.0'))
        self.on_failure = on_failure
        self._comms = []              # weakrefs to communicators
        self._flags = []              # (weakref owner, callable -> int error code)
        self._pending = collections.deque()
        self._mu = threading.Lock()
        self._stop = threading.Event()
        self._thread = None
        self.polls = 0
        self.tracked = 0
        self.completed = 0
        self.failed = None

    # ---- registration (main thread) ----------------------------------------------
    def register(self, comm):
        with self._mu:
            self._comms.append(weakref.ref(comm))
        self.start()

    def register_flag(self, owner, fn):
        """``fn()`` returns a non-zero error code once ``owner`` failed (IPC all-reduce)"""
        with self._mu:
            self._flags.append((weakref.ref(owner), fn))
        self.start()

    def track(self, event, what, comm):
        """an issued collective: ``event.query()`` turns True when it completed"""
        p = _Pending(time.monotonic(), event, what, current_label(), comm)
        with self._mu:
            self._pending.append(p)
            self.tracked += 1
            if len(self._pending) > 4096:          # the thread is slow: prune here too
                self._prune_locked()

    def wait(self, event, what, comm=None, spin_s=50e-6):
        """host wait for ``event`` under the same deadline (the host barrier)"""
        t0 = time.monotonic()
        while not event.query():
            now = time.monotonic()
            if now - t0 > self.timeout_s:
                self._fail('host wait for %s on %s exceeded HETU_COMM_TIMEOUT=%gs' % (what, comm, self.timeout_s))
                return False
            time.sleep(spin_s if now - t0 < 0.01 else 1e-3)
        return True

    # ---- the monitor thread -------------------------------------------------------
    def start(self):
        if self._thread is not None or os.environ.get('HETU_WATCHDOG', '1') == '0':
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name='hetu-comm-watchdog', daemon=True)
        self._thread.start()

    def stop(self):
        t = self._thread
        if t is None:
            return
        self._stop.set()
        t.join(timeout=max(5.0, 2 * self.poll_s))
        self._thread = None

    @property
    def running(self):
        return self._thread is not None and self._thread.is_alive()

    def _prune_locked(self):
        keep = collections.deque()
        for p in self._pending:
            if p.event.query():
                self.completed += 1
            else:
                keep.append(p)
        self._pending = keep

    def poll_once(self):
        """one pass of the checks; returns the failure text or None"""
        self.polls += 1
        with self._mu:
            comms = [r() for r in self._comms]
            self._comms = [r for r, c in zip(self._comms, comms) if c is not None]
            flags = [(o(), fn) for o, fn in self._flags]
            self._flags = [(o, fn) for (o, fn), (live, _) in zip(self._flags, flags) if live is not None]
            self._prune_locked()
            stuck = list(self._pending)
        for c in comms:
            if c is None:
                continue
            try:
                err = int(c.async_error())
            except Exception as e:      # noqa: BLE001 -- a broken handle is an error too
                return 'async error probe of %r raised %s' % (c, e)
            if err:
                return 'RCCL asynchronous error %d on %r' % (err, c)
        for live, fn in flags:
            if live is not None:
                e = int(fn())
                if e:
                    return '%r reported error %d' % (live, e)
        now = time.monotonic()
        late = [p for p in stuck if now - p.t0 > self.timeout_s]
        if late:
            return 'collective exceeded HETU_COMM_TIMEOUT=%gs: %s' % (
                self.timeout_s, '; '.join(p.describe(now) for p in late[:8]))
        return None

    def _loop(self):
        while not self._stop.wait(self.poll_s):
            try:
                why = self.poll_once()
            except Exception as e:          # noqa: BLE001 -- the monitor must not die silently
                why = 'watchdog poll raised %r' % (e,)
            if why:
                self._fail(why)
                return

    def _fail(self, why):
        self.failed = why
        now = time.monotonic()
        with self._mu:
            pend = list(self._pending)
            comms = [r() for r in self._comms]
        lines = ['hetu watchdog (rank %s): %s' % (os.environ.get('RANK', '0'), why)]
        for p in pend[:16]:
            lines.append('  in flight: ' + p.describe(now))
        sys.stderr.write('\n'.join(lines) + '\n')
        sys.stderr.flush()
        if self.on_failure is not None:
            self.on_failure(why)
            return
        for c in comms:
            if c is not None:
                try:
                    c.abort()
                except Exception:           # noqa: BLE001 -- exiting anyway
                    pass
        os._exit(EXIT_CODE)

    def stats(self):
        return {'running': self.running, 'polls': self.polls, 'tracked': self.tracked,
                'completed': self.completed, 'in_flight': len(self._pending),
                'communicators': len(self._comms), 'timeout_s': self.timeout_s}


_WD = None


def get() -> Watchdog:
    global _WD
    if _WD is None:
        _WD = Watchdog()
    return _WD


def enabled() -> bool:
    return os.environ.get('HETU_WATCHDOG', '1') != '0'


def shutdown():
    global _WD
    if _WD is not None:
        _WD.stop()
        _WD = None
