"""HIP streams and events (reference ``python/hetu/stream.py:16-105``).

On MI355X a ``Stream`` is a HIP stream created by the framework's device runtime
(``runtime.DeviceStream``: ``hipStreamCreateWithPriority`` in libhetu_alloc.so) and an
``Event`` a HIP event (``runtime.DeviceEvent``).  The executor routes compute, H2D, D2H
and comm work to separate streams and links them with ``hipStreamWaitEvent``
(``Stream.wait_event``) instead of the reference's host-side ``event.sync()``.  Kernels
launched inside ``with stream:`` run on it (``torch_stream`` is the non-owning
``torch.cuda.ExternalStream`` view torch's current stream follows; framework launches
read the thread's current stream from ``runtime.use_stream``, not from torch).
"""
from __future__ import annotations

import time

import torch

from .ndarray import is_gpu_ctx


class Stream(object):
    def __init__(self, ctx=None, priority: int = 0, torch_stream=None):
        self.ctx = ctx
        self.native = None
        if torch_stream is not None:
            self.torch_stream = torch_stream
        elif ctx is not None and is_gpu_ctx(ctx) and torch.cuda.is_available():
            from .runtime import DeviceStream
            self.native = DeviceStream(ctx.device_id, priority)
            self.torch_stream = self.native.torch
        else:
            self.torch_stream = None

    @property
    def handle(self):
        return self.torch_stream.cuda_stream if self.torch_stream is not None else None

    def sync(self):
        if self.native is not None:
            self.native.synchronize()
        elif self.torch_stream is not None:
            self.torch_stream.synchronize()

    def wait_event(self, event: 'Event'):
        if self.torch_stream is not None and event.native is not None:
            event.native.wait(self.torch_stream)

    def __enter__(self):
        if self.torch_stream is not None:
            from .runtime import use_stream
            self._ctx = use_stream(self.native if self.native is not None else self.torch_stream)
            self._ctx.__enter__()
        return self

    def __exit__(self, *a):
        if self.torch_stream is not None:
            self._ctx.__exit__(*a)
        return False


class Event(object):
    def __init__(self, ctx=None, timing: bool = False):
        self.ctx = ctx
        if ctx is not None and is_gpu_ctx(ctx) and torch.cuda.is_available():
            from .runtime import DeviceEvent
            self.native = DeviceEvent(ctx.device_id, timing)
        else:
            self.native = None
        self._t = None

    @property
    def torch_event(self):      # compatibility name: the HIP event object (or None on CPU)
        return self.native

    def record(self, stream_handle: Stream = None):
        if self.native is not None:
            s = stream_handle.torch_stream if stream_handle is not None else None
            self.native.record(s)
        else:
            self._t = time.perf_counter()

    def sync(self):
        if self.native is not None:
            self.native.synchronize()

    def time_since(self, other: 'Event') -> float:
        """Milliseconds between ``other`` and this event."""
        if self.native is not None:
            return other.native.elapsed_time(self.native)
        return (self._t - other._t) * 1000.0


class PSEvent(object):
    """Wait handle for an outstanding PS request on one key (ref ``stream.py:73-87``)."""

    def __init__(self, agent, node_id):
        self.agent = agent
        self.node_id = node_id
        self.futures = []

    def update_ts(self, fut):
        self.futures.append(fut)

    def sync(self):
        for f in self.futures:
            f.wait() if hasattr(f, 'wait') else None
        self.futures = []
        if self.agent is not None:
            self.agent.wait(self.node_id)


class CSEvent(PSEvent):
    """Also waits on outstanding HET-cache futures (ref ``stream.py:90-105``)."""


def create_stream_handle(ctx):
    return Stream(ctx)


def create_event_handle(ctx, timing=False):
    return Event(ctx, timing)
