"""Python side of the in-house RCCL communicator (``csrc/comm/hetu_comm.cc``,
``libhetu_comm.so``): the GPU collectives of :class:`parallel.comm.Communicator`.

Reference: ``communicator/mpi_nccl_comm.py:164-342`` (NCCL_Communicator) over
``src/communication/mpi_nccl_communication.cu``.  MI355X design:

* rendezvous through the job's TCP store (torchrun / heturun ``MASTER_ADDR``), no MPI;
* the collective runs on a per-communicator high-priority comm stream ordered after
  the producer with a stream edge (``wait_stream``), and an async op returns a handle
  whose ``wait()`` is another stream edge back onto the consumer's stream -- no host
  synchronisation anywhere (the reference host-syncs every comm op's event,
  ``executor.py:1034-1036``);
* tensors used on the comm stream are ``record_stream``-ed so the caching allocator
  does not recycle them while the collective is in flight;
* ``reduce_scatter_bf16`` / ``all_reduce_bf16``: the gradient crosses the wire in bf16
  (half the bytes) but is summed in fp32 -- a direct all-to-all reduce-scatter over
  the xGMI full mesh (every peer pair has its own link) followed by an fp32 local sum
  kernel and a bf16 all-gather ("bf16/fp32 gradient buckets").
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
from ..memory_pool import record_stream
from .._base import cur_stream

_LIB = None
_NCCL_DT = {torch.float32: 7, torch.float16: 6, torch.bfloat16: 9, torch.int32: 2, torch.int64: 4,
            torch.uint8: 1, torch.int8: 0, torch.float64: 8}
_NCCL_OP = {'sum': 0, 'prod': 1, 'max': 2, 'min': 3, 'mean': 4, 'avg': 4}
_TIMING = os.environ.get('HETU_COMM_TRACE', '0') == '1'   # timed completion events (bucket timeline)


class RCCLError(RuntimeError):
    pass


def _rccl_path():
    import glob
    d = os.path.join(os.path.dirname(torch.__file__), 'lib')
    cands = glob.glob(os.path.join(d, 'librccl.so*')) + ['/opt/rocm/lib/librccl.so.1']
    return os.environ.get('HETU_RCCL_LIB', cands[0] if cands else 'librccl.so.1')


def lib():
    """libhetu_comm.so with RCCL loaded, or None (no library / no RCCL)."""
    global _LIB
    if _LIB is not None:
        return _LIB or None
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'lib', 'libhetu_comm.so')
    try:
        L = ctypes.CDLL(path)
    except OSError:
        _LIB = False
        return None
    P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sig = {
        'hcomm_load': ([ctypes.c_char_p], I), 'hcomm_loaded': ([], I), 'hcomm_version': ([], I),
        'hcomm_error_string': ([I], ctypes.c_char_p), 'hcomm_set_channels': ([I, I], None),
        'hcomm_unique_id': ([ctypes.c_char_p], I), 'hcomm_unique_id_bytes': ([], I),
        'hcomm_init': ([ctypes.c_char_p, I, I, ctypes.POINTER(P)], I),
        'hcomm_split': ([P, I, I, ctypes.POINTER(P)], I), 'hcomm_destroy': ([P], I), 'hcomm_abort': ([P], I),
        'hcomm_async_error': ([P], I), 'hcomm_count': ([P], I), 'hcomm_user_rank': ([P], I),
        'hcomm_all_reduce': ([P, P, P, SZ, I, I, P], I), 'hcomm_reduce_scatter': ([P, P, P, SZ, I, I, P], I),
        'hcomm_all_gather': ([P, P, P, SZ, I, P], I), 'hcomm_broadcast': ([P, P, P, SZ, I, I, P], I),
        'hcomm_reduce': ([P, P, P, SZ, I, I, I, P], I), 'hcomm_send': ([P, P, SZ, I, I, P], I),
        'hcomm_recv': ([P, P, SZ, I, I, P], I), 'hcomm_group_start': ([], I), 'hcomm_group_end': ([], I),
        'hcomm_all_to_all': ([P, P, P, SZ, I, P], I),
        'hcomm_all_to_all_v': ([P, P, P, P, P, P, P, I, P], I),
        'hcomm_init_all': ([I, ctypes.POINTER(I), ctypes.POINTER(P)], I),
        'hcomm_multi_all_reduce': ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), SZ, I, I,
                                    ctypes.POINTER(P), I], I),
        'hcomm_multi_all_to_all': ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), SZ, I,
                                    ctypes.POINTER(P), I], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes, f.restype = args, res
    if L.hcomm_load(_rccl_path().encode()) != 0:
        _LIB = False
        return None
    _LIB = L
    return L


def available() -> bool:
    return torch.cuda.is_available() and lib() is not None


def _check(r, what):
    if r != 0:
        L = lib()
        msg = L.hcomm_error_string(r).decode() if L is not None and r > 0 else 'error %d' % r
        raise RCCLError('RCCL %s failed: %s' % (what, msg))


class Work(object):
    """Handle of an async collective: ``wait()`` orders the caller's current stream
    after it (no host sync); ``synchronize()`` blocks the host."""
    __slots__ = ('event', 'post')

    def __init__(self, event, post=None):
        self.event, self.post = event, post

    def wait(self):
        self.event.wait(None)          # the framework's current stream
        if self.post is not None:
            self.post()
            self.post = None
        return True

    def is_completed(self):
        return self.event.query()

    def synchronize(self):
        self.event.synchronize()


class NativeComm(object):
    """One RCCL communicator (a group of ``nrank`` ranks, this process = ``rank``)."""

    _store_seq = {}
    created = 0     # communicators this process created (init_rank + split), bench JSON

    def __init__(self, handle, rank, nrank):
        self.handle = ctypes.c_void_p(handle) if not isinstance(handle, ctypes.c_void_p) else handle
        self.rank, self.nrank = rank, nrank
        from ..runtime import DeviceStream
        # the comm stream: a framework-created high-priority HIP stream (torch sees its
        # ExternalStream view only for the allocator's record_stream bookkeeping)
        self._dstream = DeviceStream(priority=-1, persistent=True)
        self.stream = self._dstream.torch
        self._bf16_ws = {}
        from . import watchdog
        self._wd = watchdog.get() if watchdog.enabled() else None
        if self._wd is not None:
            self._wd.register(self)

    # ---- construction -----------------------------------------------------------
    @classmethod
    def from_store(cls, store, key, rank, nrank, channels=None):
        """Rendezvous: group rank 0 creates the unique id and publishes it in the TCP
        store under ``key``; everyone initialises its rank.  All members call."""
        L = lib()
        if L is None:
            raise RCCLError('libhetu_comm / RCCL unavailable')
        if channels:
            L.hcomm_set_channels(int(channels[0]), int(channels[1]))
        nb = L.hcomm_unique_id_bytes()
        if rank == 0:
            buf = ctypes.create_string_buffer(nb)
            _check(L.hcomm_unique_id(buf), 'get_unique_id')
            store.set(key, buf.raw)
            uid = buf.raw
        else:
            uid = bytes(store.get(key))
        h = ctypes.c_void_p()
        _check(L.hcomm_init(uid, int(nrank), int(rank), ctypes.byref(h)), 'comm_init_rank')
        NativeComm.created += 1
        return cls(h, rank, nrank)

    def split(self, color, key):
        """ncclCommSplit: every rank of this communicator calls; ``color < 0`` opts out."""
        h = ctypes.c_void_p()
        _check(lib().hcomm_split(self.handle, int(color), int(key), ctypes.byref(h)), 'comm_split')
        if color < 0 or not h.value:
            return None
        L = lib()
        NativeComm.created += 1
        return NativeComm(h, L.hcomm_user_rank(h), L.hcomm_count(h))

    def destroy(self):
        if self.handle and self.handle.value:
            lib().hcomm_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def abort(self):
        if self.handle and self.handle.value:
            lib().hcomm_abort(self.handle)
            self.handle = ctypes.c_void_p()

    def async_error(self):
        """ncclCommGetAsyncError (0 = healthy; a destroyed communicator reads healthy)"""
        h = self.handle
        if not (h and h.value):
            return 0
        return lib().hcomm_async_error(h)

    # ---- stream plumbing --------------------------------------------------------
    def _run(self, fn, tensors, async_op, post=None, what='collective'):
        """Run ``fn(stream_ptr)``: on the comm stream after the current stream's work
        (async), or on the current stream itself (sync).  Outside hipGraph capture the
        completion event goes to the watchdog (deadline ``HETU_COMM_TIMEOUT``)."""
        from ..runtime import DeviceEvent
        from ..utils.hipgraph import _CAPTURING
        cur = cur_stream()
        wd = self._wd if not _CAPTURING[0] else None
        if not async_op:
            fn(cur)
            if wd is not None:
                wd.track(DeviceEvent().record(cur), self._what(what, tensors), self)
            if post is not None:
                post()
            return None
        s = self.stream
        self._dstream.wait_stream(cur)
        fn(self._dstream.handle)
        for t in tensors:
            if t is not None and t.is_cuda:
                record_stream(t, s)
        ev = DeviceEvent(timing=_TIMING)
        ev.record(s)
        if wd is not None:
            wd.track(ev, self._what(what, tensors), self)
        return Work(ev, post)

    @staticmethod
    def _what(what, tensors):
        t = next((x for x in tensors if x is not None), None)
        return what if t is None else '%s(%d x %s)' % (what, t.numel(), str(t.dtype).replace('torch.', ''))

    # ---- collectives ------------------------------------------------------------
    def all_reduce(self, t, op='sum', async_op=False):
        assert t.is_contiguous()
        L = lib()
        nop = _NCCL_OP[op]
        return self._run(lambda st: _check(L.hcomm_all_reduce(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                              _NCCL_DT[t.dtype], nop, st), 'all_reduce'),
                         (t,), async_op, what='all_reduce')

    def reduce_scatter(self, out, inp, op='sum', async_op=False):
        inp = inp.contiguous()
        assert out.is_contiguous() and out.numel() * self.nrank == inp.numel()
        L = lib()
        return self._run(lambda st: _check(L.hcomm_reduce_scatter(self.handle, inp.data_ptr(), out.data_ptr(),
                                                                  out.numel(), _NCCL_DT[inp.dtype], _NCCL_OP[op],
                                                                  st), 'reduce_scatter'),
                         (out, inp), async_op, what='reduce_scatter')

    def all_gather(self, out, inp, async_op=False):
        inp = inp.contiguous()
        assert out.is_contiguous() and out.numel() == inp.numel() * self.nrank
        L = lib()
        return self._run(lambda st: _check(L.hcomm_all_gather(self.handle, inp.data_ptr(), out.data_ptr(),
                                                              inp.numel(), _NCCL_DT[inp.dtype], st), 'all_gather'),
                         (out, inp), async_op, what='all_gather')

    def broadcast(self, t, root=0, async_op=False):
        assert t.is_contiguous()
        L = lib()
        return self._run(lambda st: _check(L.hcomm_broadcast(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                             _NCCL_DT[t.dtype], int(root), st), 'broadcast'),
                         (t,), async_op, what='broadcast')

    def reduce(self, t, root=0, op='sum', async_op=False):
        assert t.is_contiguous()
        L = lib()
        return self._run(lambda st: _check(L.hcomm_reduce(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                          _NCCL_DT[t.dtype], _NCCL_OP[op], int(root), st),
                                           'reduce'), (t,), async_op, what='reduce')

    def all_to_all(self, out, inp, async_op=False):
        inp = inp.contiguous()
        assert out.is_contiguous() and out.numel() == inp.numel() and inp.numel() % self.nrank == 0
        L = lib()
        chunk = inp.numel() // self.nrank
        return self._run(lambda st: _check(L.hcomm_all_to_all(self.handle, inp.data_ptr(), out.data_ptr(), chunk,
                                                              _NCCL_DT[inp.dtype], st), 'all_to_all'),
                         (out, inp), async_op, what='all_to_all')

    def p2p(self, ops, async_op=True):
        """ops: [('send'|'recv', tensor, peer)] as one RCCL group."""
        L = lib()

        def run(st):
            _check(L.hcomm_group_start(), 'group_start')
            for kind, t, peer in ops:
                f = L.hcomm_send if kind == 'send' else L.hcomm_recv
                _check(f(self.handle, t.data_ptr(), t.numel(), _NCCL_DT[t.dtype], int(peer), st), kind)
            _check(L.hcomm_group_end(), 'group_end')
        return self._run(run, [t for _, t, _ in ops], async_op,
                         what='p2p[%s]' % ','.join('%s:%d' % (k, p) for k, _, p in ops))

    # ---- bf16 wire, fp32 accumulation --------------------------------------------
    def _ws(self, n, dtype, tag):
        k = (tag, dtype)
        b = self._bf16_ws.get(k)
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 1), dtype=dtype, device='cuda')
            self._bf16_ws[k] = b
        return b[:n]

    def all_reduce_bf16(self, t, async_op=False):
        """fp32 ``t`` summed across ranks with bf16 on the wire: bf16 all-to-all (=
        reduce-scatter traffic, padded to P chunks of a multiple of 8), fp32 sum of the
        P received chunks, bf16 all-gather of the reduced chunk, fp32 result in place."""
        from ..kernels import comm as KC
        P, n = self.nrank, t.numel()
        assert t.dtype == torch.float32 and t.is_contiguous()
        if not async_op:
            # the workspaces are shared with async calls on the comm stream: a sync call on
            # the caller's stream must not overtake a bucket still using them
            from ..runtime import DeviceEvent
            DeviceEvent().record(self._dstream).wait(None)
        c = -(-n // (8 * P)) * 8
        send = self._ws(c * P, torch.bfloat16, 'send')
        recv = self._ws(c * P, torch.bfloat16, 'recv')
        red = self._ws(c, torch.bfloat16, 'red')
        L = lib()

        def run(st):
            KC.cast_f32_bf16(t, send, st)
            _check(L.hcomm_all_to_all(self.handle, send.data_ptr(), recv.data_ptr(), c, 9, st), 'all_to_all')
            KC.sum_chunks_bf16(recv, P, c, red, st)           # fp32 accumulate, bf16 out
            _check(L.hcomm_all_gather(self.handle, red.data_ptr(), send.data_ptr(), c, 9, st), 'all_gather')
            KC.cast_bf16_f32(send, t, st)
        return self._run(run, (t, send, recv, red), async_op, what='all_reduce_bf16')

    def __repr__(self):
        return 'NativeComm(rank=%d, nrank=%d)' % (self.rank, self.nrank)


class MultiDeviceComm(object):
    """Single-process multi-GPU communicator (reference ``nccl_communication.cu``
    NCCL_AllReduce / NCCL_AllToAll over ``ncclCommInitAll``): one process
    holds one RCCL communicator per device and issues each collective as one group,
    every device's part on that device's current stream."""

    def __init__(self, devices):
        L = lib()
        if L is None:
            raise RCCLError('libhetu_comm / RCCL unavailable')
        self.devices = [int(d) for d in devices]
        n = len(self.devices)
        self.handles = (ctypes.c_void_p * n)()
        _check(L.hcomm_init_all(n, (ctypes.c_int * n)(*self.devices), self.handles), 'comm_init_all')

    def _ptrs(self, ts):
        assert len(ts) == len(self.devices)
        for t, d in zip(ts, self.devices):
            assert t.is_cuda and t.device.index == d and t.is_contiguous(), (t.device, d)
        return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])

    def _streams(self):
        return (ctypes.c_void_p * len(self.devices))(*[torch.cuda.current_stream(d).cuda_stream
                                                         for d in self.devices])

    def all_reduce(self, tensors, op='sum'):
        """in place: every device's tensor becomes the reduction over all devices"""
        p = self._ptrs(tensors)
        _check(lib().hcomm_multi_all_reduce(self.handles, p, p, tensors[0].numel(), _NCCL_DT[tensors[0].dtype],
                                            _NCCL_OP[op], self._streams(), len(tensors)), 'multi_all_reduce')
        return tensors

    def all_to_all(self, outs, ins):
        n = len(self.devices)
        assert ins[0].numel() % n == 0
        _check(lib().hcomm_multi_all_to_all(self.handles, self._ptrs(ins), self._ptrs(outs), ins[0].numel() // n,
                                            _NCCL_DT[ins[0].dtype], self._streams(), n), 'multi_all_to_all')
        return outs

    def destroy(self):
        L = lib()
        for h in self.handles:
            if h:
                L.hcomm_destroy(ctypes.c_void_p(h))
        self.handles = (ctypes.c_void_p * 0)()


def world_from_dist(group=None, key_prefix='hetu_rccl') -> Optional[NativeComm]:
    """Native communicator over the ranks of an initialised torch.distributed group
    (its store carries the unique id).  Every member calls."""
    import torch.distributed as dist
    if not available() or not dist.is_initialized():
        return None
    store = dist.distributed_c10d._get_default_store()
    ranks = None if group is None else dist.get_process_group_ranks(group)
    rank = dist.get_rank(group)
    nrank = dist.get_world_size(group)
    name = 'world' if ranks is None else '_'.join(map(str, ranks))
    seq = NativeComm._store_seq[name] = NativeComm._store_seq.get(name, 0) + 1   # same order on every member
    key = '%s/%s/%d' % (key_prefix, name, seq)
    ch = os.environ.get('HETU_RCCL_CHANNELS')
    channels = tuple(int(x) for x in ch.split(',')) if ch else None
    return NativeComm.from_store(store, key, rank, nrank, channels)
