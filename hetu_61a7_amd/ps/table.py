"""Worker-side handles of PS-managed parameters (reference
``gpu_ops/ParameterServerCommunicate.py:13-338`` and ``Variable.py:55-81``).

``PSTable``   an embedding table that lives on the PS server (host DRAM),
              optionally fronted by the HET cache.  Lookups return device rows;
              gradients are pre-multiplied by ``-lr`` on the GPU, staged through
              pinned host memory and pushed asynchronously (the server adds them,
              as in the reference where server-side optimizers are unused).
``PSDense``   the whole flat dense parameter buffer of an optimizer as ONE PS
              key: one DDPushPull per step instead of one request per tensor.

Synchronisation (reference ``bsp``): -1 ASP, 0 BSP (worker barrier between
push and pull), >0 SSP with that staleness bound.
"""
from __future__ import annotations

import os
import torch

from . import worker as psw
from .worker import PARAM_DENSE, PARAM_SPARSE, PARAM_CACHE
from ..memory_pool import record_stream
from ..runtime import DeviceEvent, use_stream, stream_edge
from .._base import cur_stream, gpu_available
from .. import native_array as _NA


def _scaled_f32(x, c):
    """fp32 c * x on the native kernels for device tensors (cast + scale, no ATen launch)"""
    if not x.is_cuda:
        return x.float() * c
    from ..kernels.elementwise import unary, cast
    from ..kernels.tensor import copy_into
    if not x.is_contiguous():
        x = copy_into(_NA.empty(tuple(x.shape), dtype=x.dtype, device=x.device), x)
    return unary('mul_c', cast(x, torch.float32), c)


def _dev_copy(dst, src):
    """dst = src between device tensors (dtype cast included) on the native kernels"""
    if dst.is_cuda and src.is_cuda:
        from ..kernels.tensor import copy_into
        return copy_into(dst, src)
    return dst.copy_(src)


def _pinned(n, dtype=torch.float32):
    from ..ndarray import pinned_empty
    return pinned_empty((n,), dtype)


_STREAMS = {}
# host seconds spent blocked on the PS / HET cache (ticket waits, staging-copy events):
# the "PS wait" term of bench.py's Wide&Deep step breakdown
WAIT_S = [0.0]


class _waiting(object):
    __slots__ = ('t0',)

    def __enter__(self):
        import time
        self.t0 = time.perf_counter()

    def __exit__(self, *a):
        import time
        WAIT_S[0] += time.perf_counter() - self.t0
        return False


def side_streams(device):
    """(h2d, d2h) copy streams of a device (reference HetuConfig h2d/d2h streams,
    executor.py:319-334): PS/cache transfers run there, ordered against the compute
    stream by events, so they overlap compute instead of queueing behind it."""
    s = _STREAMS.get(device)
    if s is None:
        from ..runtime import DeviceStream
        from .._base import cur_device
        idx = torch.device(device).index
        idx = cur_device() if idx is None else idx
        # framework-created HIP streams, used through runtime.use_stream
        s = _STREAMS[device] = (DeviceStream(idx, persistent=True), DeviceStream(idx, persistent=True))
    return s


def host_ids(t):
    """int64 host copy of an id tensor.  A device tensor made from a host feed carries
    its source (``hetu_host``, set by the executor's feed path): no device sync.  Other
    device ids are copied on the d2h stream after the producer and waited for alone."""
    h = getattr(t, 'hetu_host', None)
    if h is not None and h.numel() == t.numel():
        return h.reshape(-1).long().contiguous()
    t = t.reshape(-1)
    if not t.is_cuda:
        return t.long().contiguous()
    _, d2h = side_streams(t.device)
    d2h.wait_stream(None)                      # after the producer on the current stream
    out = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    with use_stream(d2h):
        out.copy_(t, non_blocking=True)
        ev = DeviceEvent().record(d2h)
    record_stream(t, d2h)
    ev.synchronize()
    return out.long()


class _Staging(object):
    """Grow-only pinned buffer + an event guarding its reuse."""

    def __init__(self, dtype=torch.float32):
        self.buf = None
        self.dtype = dtype
        self.event = None
        self.ticket = None       # the push that reads this buffer (gradient staging)

    def get(self, n):
        if self.event is not None:
            self.event.synchronize()
            self.event = None
        if self.buf is None or self.buf.numel() < n:
            self.buf = _pinned(max(n, 1), self.dtype)
        return self.buf[:n]

    def guard(self, stream=None):
        if gpu_available():
            # one event per buffer, re-recorded: its last use is what a reuse waits for
            ev = getattr(self, '_ev', None)
            if ev is None:
                ev = self._ev = DeviceEvent()
            self.event = ev.record(stream)


_LIVE = []
# HETU_PS_DEFER_PUSH=1: push a step's embedding gradient behind the next step's staging
# instead of at the step's end.  Off: with the double-buffered staging the end-of-step push
# no longer waits for the previous one, and deferring measured slower (the next lookup then
# waits for the prefetch queued behind the push): WDL 187-191 k vs 121-144 k samples/s
# (profiles/wdl_ps_push_ab_r6.txt)
_DEFER_PUSH = os.environ.get('HETU_PS_DEFER_PUSH', '0') == '1'


def close_all():
    """Drain outstanding pushes of every PS table (before the worker finalises)."""
    for t in _LIVE:
        t.close()
    _LIVE.clear()


def drain_dense():
    """finish every overlapped dense exchange in flight (an evaluation step must see the
    parameters the last training step pulled)"""
    for t in _LIVE:
        if isinstance(t, PSDense):
            t.drain()


class PSTable(object):
    def __init__(self, node, config):
        _LIVE.append(self)
        self.node = node
        self.key = node.id
        self.agent = psw.get_agent()
        self.rows = int(node.shape[0])
        self.width = int(torch.Size(node.shape[1:]).numel())
        self.shape = tuple(node.shape)
        self.device = config.device
        self.bsp = config.bsp
        policy = config.cstable_policy
        ptype = PARAM_CACHE if policy else PARAM_SPARSE
        init = node.initializer
        if init is None:
            raise ValueError('PS-managed table %s needs an initializer' % node.name)
        self.agent.init_tensor(self.key, ptype, self.shape, init, config.seed + self.key)
        self.cache = None
        if policy:
            from .cstable import CacheSparseTable
            limit = max(self.rows // 10, 1)
            self.cache = CacheSparseTable(limit, self.rows, self.width, self.key, policy,
                                          config.cache_bound)
        else:
            self.agent.BarrierWorker()
        self.out_stage = _Staging()
        # gradient staging, double-buffered: a deferred push still reads one buffer while
        # the next step's gradient lands in the other
        self.grad_stages = (_Staging(), _Staging())
        self.gs_flip = 0
        self.pending = None
        self.pending_push = None
        self._prefetch_due = False
        self.version = 0
        # prefetch (reference executor.py:531-536, HetuConfig(prefetch=True)): when the
        # ids of the NEXT batch are known (dataloader-fed lookups) and training is
        # asynchronous (bsp=-1), the cache lookup of batch i+1 is queued right after
        # the lookup of batch i, so it runs on the cache thread while the GPU computes
        # step i.  Rows batch i+1 shares with batch i then miss step i's own update
        # (staleness 1, inside the HET cache's pull bound); BSP/SSP never prefetch.
        self.next_ids_fn = None
        self.pf_stages = (_Staging(), _Staging())
        self.pf_flip = 0
        self.prefetched = None
        self.prefetch_hits = 0

    # tensor-like attributes the graph code may query
    @property
    def dtype(self):
        return torch.float32

    def numel(self):
        return self.rows * self.width

    def _wait_ticket(self, t):
        with _waiting():
            if self.cache is not None:
                self.cache.wait(t)
            else:
                self.agent.WaitTicket(t)

    def _wait_push(self):
        """every push issued so far (a deferred one is issued first) has completed"""
        if self.pending_push is not None:
            self.flush_grad(force=True)
        for st in self.grad_stages:
            if st.ticket is not None:
                self._wait_ticket(st.ticket)
                st.ticket = None
        self.pending = None

    def _deferrable(self):
        """ASP with prefetch: a step's gradient push waits for the next step's gradient
        staging (by then its D2H copy has long completed), and the prefetch of the batch
        after next is issued right behind it -- the host never blocks on this step's device
        work, and prefetched rows still carry every push up to the step before (staleness 1,
        as the un-deferred schedule)"""
        return (_DEFER_PUSH and self.cache is not None and self.next_ids_fn is not None
                and self.bsp is not None and self.bsp < 0)

    def _take_prefetched(self, ids):
        pf, self.prefetched = self.prefetched, None
        if pf is None:
            return None, None
        pids, dest, ticket, stage = pf
        with _waiting():
            self.cache.wait(ticket)
        if pids.numel() != ids.numel() or not torch.equal(pids, ids):
            return None, None
        self.prefetch_hits += 1
        return dest, stage

    def _prefetch_next(self):
        if self.next_ids_fn is None or self.cache is None or self.bsp is None or self.bsp >= 0:
            return
        nxt = self.next_ids_fn()
        if nxt is None:
            return
        nxt = nxt.reshape(-1).long().contiguous()
        stage = self.pf_stages[self.pf_flip]
        self.pf_flip ^= 1
        dest = stage.get(nxt.numel() * self.width).view(-1, self.width)
        t = self.cache.embedding_lookup(nxt, dest)
        self.prefetched = (nxt, dest, t, stage)

    def lookup(self, idx, out_dtype=None):
        ids = host_ids(idx)
        dest, stage = self._take_prefetched(ids)
        if dest is None:
            self._wait_push()      # on-demand pull sees every push issued so far
            stage = self.out_stage
            dest = stage.get(ids.numel() * self.width).view(-1, self.width)
            with _waiting():
                if self.cache is not None:
                    self.cache.embedding_lookup(ids, dest, sync=True)
                else:
                    t = self.agent.SparsePull(self.key, ids, dest)
                    self.agent.WaitTicket(t)
        if self.pending_push is not None and self._deferrable():
            self._prefetch_due = True        # issued behind the deferred push (stage_grad)
        else:
            self._prefetch_next()
        if self.device.type == 'cuda':
            # H2D on the copy stream; the compute stream waits for it by event only
            h2d, _ = side_streams(self.device)
            with use_stream(h2d):
                out = dest.to(self.device, non_blocking=True)
                stage.guard(h2d)
            stream_edge(h2d)                         # the current stream waits for the copy
            record_stream(out, cur_stream())
            if out_dtype is not None and out_dtype != out.dtype:
                from ..kernels.elementwise import cast
                out = cast(out, out_dtype)
        else:
            out = dest.clone()
        return out.view(*idx.shape, self.width)

    def stage_grad(self, slices, lr):
        """Scale by -lr on the device and start the D2H copy (called as soon as the
        gradient exists, so it overlaps the rest of backward)."""
        if self.pending_push is not None:
            self.flush_grad(force=True)      # the previous step's deferred push
        if self._prefetch_due:
            self._prefetch_due = False
            self._prefetch_next()
        stage = self.grad_stages[self.gs_flip]
        self.gs_flip ^= 1
        if stage.ticket is not None:         # the push that last read this buffer
            self._wait_ticket(stage.ticket)
            stage.ticket = None
        ids = host_ids(slices.indices)
        vals = slices.values.reshape(-1, self.width)
        scaled = _scaled_f32(vals, -lr)
        host = stage.get(scaled.numel()).view(-1, self.width)
        if scaled.is_cuda:
            # D2H on the copy stream after the scaling kernel; the compute stream goes on
            _, d2h = side_streams(scaled.device)
            d2h.wait_stream(None)
            with use_stream(d2h):
                host.copy_(scaled, non_blocking=True)
                stage.guard(d2h)
            record_stream(scaled, d2h)
        else:
            host.copy_(scaled)
        self.pending_push = (ids, host, stage)

    def flush_grad(self, force=True):
        """Push the staged gradient (after its D2H copy completed).  ``force=False`` (the
        optimizer's end of step) leaves it to the next step's staging when deferrable."""
        if self.pending_push is None:
            return
        if not force and self._deferrable():
            return
        ids, host, stage = self.pending_push
        self.pending_push = None
        if stage.event is not None:
            with _waiting():
                stage.event.synchronize()
            stage.event = None
        if self.cache is not None:
            self.pending = self.cache.embedding_update(ids, host)
        else:
            self.pending = self.agent.SparsePush(self.key, ids, host)
        stage.ticket = self.pending
        self.version += 1
        if self.bsp == 0:
            self._wait_push()
            if self.cache is not None:
                self.cache.flush()
            self.agent.BarrierWorker()
        elif self.bsp and self.bsp > 0:
            self._wait_push()
            self.agent.ssp_sync(self.key, self.version)

    def close(self):
        self.flush_grad()
        self._wait_push()
        if self.cache is not None:
            self.cache.flush()

    def invalidate(self):
        """Forget every worker-side copy of the table's rows (after the server
        loaded a checkpoint): pending pushes are drained first by ``close``."""
        self.close()
        if self.prefetched is not None:
            self.cache.wait(self.prefetched[2])
            self.prefetched = None
        if self.cache is not None:
            self.cache.clear()

    def to_dense(self):
        """Full table (host) -- checkpointing / tests."""
        self._wait_push()
        if self.cache is not None:
            self.cache.flush()
        out = torch.empty(self.rows, self.width)
        ids = torch.arange(self.rows, dtype=torch.int64)
        t = self.agent.SparsePull(self.key, ids, out)
        self.agent.WaitTicket(t)
        return out.view(self.shape)


class PSDense(object):
    """Flat dense parameters held by the PS (pure PS mode)."""

    def __init__(self, flat, key, config, publish=None, overlap=None):
        _LIVE.append(self)          # close_all() (worker_finish) drains the overlapped exchange
        self.flat = flat
        self.key = key
        self.agent = psw.get_agent()
        self.bsp = config.bsp
        # ASP with prefetch (the executor's default): the dense push-pull of step t runs on a
        # helper thread while step t+1 computes, and its pulled values replace the worker's
        # copy at the end of step t+1 -- staleness 1, the same bound the prefetched embedding
        # rows already have (reference executor prefetch=True).  BSP / SSP stay synchronous.
        if overlap is None:
            overlap = (self.bsp is None or self.bsp < 0) and bool(getattr(config, 'prefetch', False))
        self.overlap = overlap
        self._thread = None
        self._inflight = False
        n = flat.numel
        self.agent.InitTensor(key, PARAM_DENSE, n, 1, 0, 0.0, 0.0, 0)
        # one worker publishes its initial values (worker 0 by default; a
        # pipeline stage's first replica for a per-stage key); everyone starts from them
        if publish is None:
            publish = self.agent.rank() == 0
        if publish:
            host = flat.param.detach().float().cpu().contiguous()
            t = self.agent.Push(key, host)
            self.agent.WaitTicket(t)
        self.agent.BarrierWorker()
        self.push_buf = _pinned(n)
        self.pull_buf = _pinned(n)
        self._pull_into_device()
        if self.bsp and self.bsp > 0:
            self.agent.ssp_init(key, self.agent.nrank(), self.bsp)
        self.version = 0

    def repull(self):
        """Reload the worker's copy from the server (after a checkpoint load)."""
        self.drain()
        self._pull_into_device()

    # ---- overlapped exchange (ASP + prefetch) -----------------------------------------------
    def _worker(self):
        while True:
            ev = self._q.get()
            if ev is None:
                return
            try:
                ev.synchronize()                 # the scaled gradient is in push_buf
                t = self.agent.DDPushPull(self.key, self.push_buf, self.pull_buf)
                self.agent.WaitTicket(t)
            except BaseException as e:           # noqa: BLE001 -- re-raised by the step thread
                self._err = e
            finally:
                self._done.set()

    def _start(self):
        import queue
        import threading
        self._q = queue.Queue()
        self._done = threading.Event()
        self._err = None
        self._thread = threading.Thread(target=self._worker, name='hetu-ps-dense', daemon=True)
        self._thread.start()

    def _apply_inflight(self):
        """wait for the exchange in flight and load its pulled values into the device copy"""
        if not self._inflight:
            return
        with _waiting():
            self._done.wait()
        self._inflight = False
        if self._err is not None:
            e, self._err = self._err, None
            raise e
        n = self.flat.numel
        self.flat.param.copy_(self.pull_buf[:n], non_blocking=True)
        if self.flat.shadow is not None:
            _dev_copy(self.flat.shadow, self.flat.param)

    def drain(self):
        """finish the exchange in flight (before a checkpoint, an evaluation or shutdown)"""
        if self._thread is not None:
            self._apply_inflight()

    def close(self):
        """drain, then stop the helper thread (before the agent finalises)"""
        if self._thread is None:
            return
        try:
            self.drain()
        finally:
            self._q.put(None)
            self._thread.join(timeout=60)
            self._thread = None

    def _step_overlapped(self, g, lr):
        if self._thread is None:
            self._start()
        self._apply_inflight()                   # step t-1's exchange: usually long done
        n = self.flat.numel
        scaled = _scaled_f32(g, -lr)
        _, d2h = side_streams(g.device)
        d2h.wait_stream(None)
        with use_stream(d2h):
            self.push_buf[:n].copy_(scaled, non_blocking=True)
            ev = DeviceEvent().record(d2h)
        record_stream(scaled, d2h)
        self.version += 1
        self._done.clear()
        self._inflight = True
        self._q.put(ev)

    def _pull_into_device(self):
        t = self.agent.Pull(self.key, self.pull_buf)
        self.agent.WaitTicket(t)
        self.flat.param.copy_(self.pull_buf[:self.flat.numel], non_blocking=True)
        if self.flat.shadow is not None:
            _dev_copy(self.flat.shadow, self.flat.param)

    def step(self, lr):
        n = self.flat.numel
        g = self.flat.grad[:n]
        if self.overlap and g.is_cuda:
            return self._step_overlapped(g, lr)
        self.push_buf[:n].copy_(_scaled_f32(g, -lr), non_blocking=True)
        if g.is_cuda:
            DeviceEvent().record(None).synchronize()
        self.version += 1
        if self.bsp == 0:
            t = self.agent.Push(self.key, self.push_buf)
            self.agent.WaitTicket(t)
            self.agent.BarrierWorker()
            self._pull_into_device()
        elif self.bsp and self.bsp > 0:
            t = self.agent.Push(self.key, self.push_buf)
            self.agent.WaitTicket(t)
            self.agent.ssp_sync(self.key, self.version)
            self._pull_into_device()
        else:
            t = self.agent.DDPushPull(self.key, self.push_buf, self.pull_buf)
            with _waiting():
                self.agent.WaitTicket(t)
            self.flat.param.copy_(self.pull_buf[:n], non_blocking=True)
            if self.flat.shadow is not None:
                _dev_copy(self.flat.shadow, self.flat.param)
