"""One-shot small-message all-reduce over IPC-mapped peer buffers (last
bullet; kernel: ``csrc/kernels/ipc_allreduce.hip``).

Each rank exports one device slab (two data parities + a flag row) with
``hipIpcGetMemHandle``; the handles are exchanged once over the process group; every
call is then a single one-workgroup kernel per rank that publishes its input, raises
its flag in every peer's slab, waits for the peers' flags (bounded spin) and reduces the
peers' copies straight from their memory over xGMI.  No RCCL call, no host sync: for the
few-hundred-byte reductions of a step (loss scalars, the DTS gate's expert histogram,
the bench's max-reduce of its timer) the latency is one flag round trip instead of an
RCCL ring's protocol.

    ar = IPCAllReduce(rank, nranks, exchange=lambda b: gathered_list_of_bytes, device=dev)
    y = ar(x)                 # fp32, x.numel() <= cap; op 'sum' or 'max'
    ar.check()                # raises if a call timed out waiting for a peer (host read)

Opt-in (``HETU_IPC_ALLREDUCE=1`` routes ``Communicator.all_reduce`` of fp32 tensors up to
``cap`` elements through it, when every rank of the communicator is on this node).  A
timed-out call is reported by the next routed call, the next ``barrier()`` and the
watchdog thread (``parallel/watchdog.py``), which exits the process.  The 2-process
same-GPU tests are ``tests/test_ipc_allreduce_gpu.py``.
"""
from __future__ import annotations

import ctypes

import torch

from .. import native_array as _NA

_OPS = {'sum': 0, 'max': 1}
# spin iterations (each a short sleep) before a call gives up on a missing peer: about a
# few seconds -- a failed call is reported by check(), it never hangs the GPU
SPIN_CAP = 1 << 25


class IPCAllReduce(object):
    def __init__(self, rank, nranks, exchange, cap=4096, device=None):
        from ..kernels import kernels_lib, check
        self.lib = kernels_lib()
        self.rank, self.nranks, self.cap = int(rank), int(nranks), int(cap)
        if not 1 <= self.nranks <= 16:
            raise ValueError('IPCAllReduce supports 1..16 ranks, got %d' % nranks)
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        L = self.lib
        L.hetu_ipcar_alloc.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        L.hetu_ipcar_open.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        L.hetu_ipcar_close.argtypes = [ctypes.c_void_p]
        L.hetu_ipcar_free.argtypes = [ctypes.c_void_p]
        L.hetu_ipcar_allreduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        with torch.cuda.device(self.device):
            self.slab = ctypes.c_void_p()
            hbuf = (ctypes.c_ubyte * 64)()
            check(L.hetu_ipcar_alloc(self.cap, ctypes.byref(self.slab), hbuf), 'ipcar_alloc')
            hbytes = bytes(hbuf)[:int(L.hetu_ipcar_handle_bytes())]
            handles = list(exchange(hbytes))
            if len(handles) != self.nranks:
                raise RuntimeError('IPCAllReduce: exchange returned %d handles for %d ranks' % (len(handles), nranks))
            self.ptrs = (ctypes.c_void_p * self.nranks)()
            self.opened = []
            for j, h in enumerate(handles):
                if j == self.rank:
                    self.ptrs[j] = self.slab.value
                    continue
                hb = (ctypes.c_ubyte * 64).from_buffer_copy(bytes(h) + b'\0' * (64 - len(h)))
                p = ctypes.c_void_p()
                check(L.hetu_ipcar_open(hb, ctypes.byref(p)), 'ipcar_open(rank %d)' % j)
                self.ptrs[j] = p.value
                self.opened.append(p)
            # the error word lives in pinned host memory (device-mapped): check() and the
            # watchdog read it without a GPU call or a stream sync
            self.err = _NA.empty((1,), dtype=torch.int32, device='cpu', pinned=True)
            self.err.zero_()
        self.epoch = 0
        from . import watchdog
        if watchdog.enabled():
            err = self.err
            watchdog.get().register_flag(self, lambda: int(err[0]))

    def __call__(self, x, op='sum', out=None):
        from ..kernels import check, stream_ptr
        if x.dtype != torch.float32 or not x.is_cuda or x.numel() > self.cap:
            raise ValueError('IPCAllReduce takes fp32 device tensors of at most %d elements' % self.cap)
        if not x.is_contiguous():
            from ..kernels.tensor import copy_into
            x = copy_into(_NA.empty(tuple(x.shape), dtype=x.dtype, device=x.device), x)
        if out is None:
            out = _NA.empty(tuple(x.shape), dtype=torch.float32, device=x.device)
        self.epoch += 1
        check(self.lib.hetu_ipcar_allreduce(x.data_ptr(), out.data_ptr(), x.numel(), self.cap, self.epoch,
                                            self.rank, self.nranks, self.ptrs, _OPS[op], self.err.data_ptr(),
                                            SPIN_CAP, stream_ptr()), 'ipcar_allreduce')
        return out

    def check(self):
        """raise if any completed call so far timed out waiting for a peer (one host read
        of the mapped error word; calls still in flight are seen by a later check)"""
        e = int(self.err[0])
        if e:
            raise RuntimeError('IPCAllReduce: call %d timed out waiting for a peer' % e)

    def close(self):
        if self.slab is None:
            return
        torch.cuda.synchronize(self.device)
        for p in self.opened:
            self.lib.hetu_ipcar_close(p)
        self.opened = []
        self.lib.hetu_ipcar_free(self.slab)
        self.slab = None

    def __del__(self):
        try:
            self.close()
        except Exception:       # noqa: BLE001 -- interpreter shutdown
            pass
