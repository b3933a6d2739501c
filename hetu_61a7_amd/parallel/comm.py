"""RCCL communicators over xGMI (reference communicator/mpi_nccl_comm.py:24-342,
src/communication/mpi_nccl_communication.cu).

One process per GPU.  ``torch.distributed`` with backend ``nccl`` *is* RCCL on
ROCm; rendezvous uses the TCP store (``MASTER_ADDR``/``MASTER_PORT``) instead of
MPI, and ``RANK/WORLD_SIZE/LOCAL_RANK`` (or the ``OMPI_COMM_WORLD_*``
equivalents, so ``mpirun`` still works).  On CPU-only processes the same API
runs on gloo, which is what the multi-process CPU tests use.

Semantics kept from the reference: AllReduce is a SUM (users scale the lr),
AllToAll exchanges equal ``numel/nranks`` chunks, sub-group communicators are
cached per device/rank set.
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..context import dist_env

_GROUPS: Dict[Tuple[int, ...], 'Communicator'] = {}
_WORLD: Optional['Communicator'] = None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def backend_for_device(dev_is_gpu: bool) -> str:
    """The torch.distributed backend: gloo -- the TCP-store rendezvous, host-tensor
    collectives and host barriers only.  Every GPU collective runs on the in-house RCCL
    communicator (``parallel/rccl.py``), so torch never creates an RCCL communicator of its
    own (no ProcessGroupNCCL next to ours).  ``HETU_COMM=torch`` (A/B: torch's RCCL path)
    selects 'nccl'.  ``HETU_DIST_BACKEND=gloo`` forces gloo for GPU tensors too, without
    the native communicator: several ranks can then share one GPU (RCCL refuses duplicate
    devices), which rehearses the multi-rank GPU path on a one-GPU box."""
    forced = os.environ.get('HETU_DIST_BACKEND')
    if forced:
        return forced
    if dev_is_gpu and os.environ.get('HETU_COMM', 'native') == 'torch':
        return 'nccl'
    return 'gloo'


def native_gpu_comm(use_gpu: bool) -> bool:
    """GPU collectives on the in-house RCCL communicator (the default for GPU processes)"""
    return bool(use_gpu) and os.environ.get('HETU_COMM', 'native') != 'torch' and \
        not os.environ.get('HETU_DIST_BACKEND')


def init_process_group(use_gpu: Optional[bool] = None, timeout_s: Optional[int] = None) -> 'Communicator':
    """Initialise the global communicator (idempotent).

    Failure detection (SURVEY §5.3 "RCCL watchdog"): every GPU collective goes through
    the in-house communicator, whose completion events and ``ncclCommGetAsyncError``
    state the process's watchdog thread (``parallel/watchdog.py``) polls.  A collective
    older than ``timeout_s`` (env ``HETU_COMM_TIMEOUT``, default 1800 s) or an async
    error aborts every communicator and exits the process non-zero -- the launcher
    (``heturun --max-restarts``) then restarts the group, which resumes from the last
    checkpoint (``utils.checkpoint``).  The gloo bootstrap / host-tensor group keeps
    torch's own ``timeout``."""
    global _WORLD
    if timeout_s is None:
        timeout_s = int(os.environ.get('HETU_COMM_TIMEOUT', '1800'))
    os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '1')
    if _WORLD is not None:
        return _WORLD
    rank, world, local = dist_env()
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu:
        from .._base import set_device
        set_device(local % max(torch.cuda.device_count(), 1))
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'MASTER_PORT' not in os.environ:
            # a lone process picks a free port so concurrent single-rank jobs don't collide
            os.environ['MASTER_PORT'] = str(_free_port()) if world == 1 else '29517'
        os.environ.setdefault('RANK', str(rank))
        os.environ.setdefault('WORLD_SIZE', str(world))
        # gloo bootstrap (backend_for_device): one RCCL communicator per rank -- the
        # in-house one (parallel/rccl.py), created from this group's TCP store
        kw = dict(backend=backend_for_device(use_gpu), rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        dist.init_process_group(**kw)
    _WORLD = Communicator(None, use_gpu=use_gpu)
    return _WORLD


def world() -> Optional['Communicator']:
    return _WORLD


def is_initialized() -> bool:
    return _WORLD is not None


def new_group_comm(ranks: Optional[Sequence[int]] = None, local_sync: bool = False) -> 'Communicator':
    """Cached sub-group communicator.

    By default every rank of the world must call in the same order (static
    groups: TP/PP/DistGCN row and column groups).  ``local_sync=True`` creates
    the group with only its members participating -- what partial-reduce needs,
    whose partner sets are formed at run time (reference preduce.py:41-42 builds
    an NCCL group unique id among the partners only)."""
    w = init_process_group()
    if ranks is None:
        return w
    key = tuple(sorted(int(r) for r in ranks))
    if len(key) == w.nrank:
        return w
    if key not in _GROUPS:
        _GROUPS[key] = Communicator(key, use_gpu=w.use_gpu, local_sync=local_sync)
    return _GROUPS[key]


_RED = {'sum': dist.ReduceOp.SUM, 'max': dist.ReduceOp.MAX, 'min': dist.ReduceOp.MIN,
        'prod': dist.ReduceOp.PRODUCT}



# HETU_IPC_ALLREDUCE=1: small fp32 all-reduces through parallel/ipc_allreduce.py
_IPC_SMALL = os.environ.get('HETU_IPC_ALLREDUCE', '0') == '1'

class _CInt(object):
    __slots__ = ('value',)

    def __init__(self, v):
        self.value = int(v)


class Communicator(object):
    """A (sub-)group of ranks: collectives on the calling stream.

    All methods take torch tensors; ``async_op=True`` returns a work handle
    (RCCL runs on its own stream ordered after the current stream, so compute
    keeps flowing -- the overlap the reference gets from its nccl_stream).
    """

    def __init__(self, ranks: Optional[Tuple[int, ...]], use_gpu: bool = True, local_sync: bool = False):
        self.use_gpu = use_gpu
        self.ranks = ranks
        if ranks is None:
            self.group = None
        elif local_sync:
            self.group = dist.new_group(list(ranks), use_local_synchronization=True)
        else:
            self.group = dist.new_group(list(ranks))
        self.rank = dist.get_rank(self.group) if (ranks is None or dist.get_rank() in ranks) else -1
        self.nrank = dist.get_world_size(self.group) if ranks is None or self.rank >= 0 else len(ranks)
        self.global_rank = dist.get_rank()
        self.local_rank = dist_env()[2]
        self.device_id = self.local_rank
        self._bar = None
        # GPU collectives: the in-house RCCL communicator (csrc/comm/hetu_comm.cc) unless
        # HETU_COMM=torch; torch.distributed stays the bootstrap / host-tensor path.
        # Static sub-groups (created by every rank in the same order) are ncclCommSplit
        # children of the world communicator -- no new unique-id rendezvous or full
        # ncclCommInitRank per group; non-members take part in the split with no colour.
        # Partial-reduce groups (local_sync: only the members call) rendezvous by store.
        self.native = None
        if native_gpu_comm(use_gpu):
            from . import rccl
            if rccl.available():
                w = _WORLD.native if _WORLD is not None else None
                if ranks is None:
                    self.native = rccl.world_from_dist(None)
                elif not local_sync and w is not None:
                    sub = w.split(0 if self.rank >= 0 else -1, self.global_rank)
                    self.native = sub if self.rank >= 0 else None
                elif self.rank >= 0:
                    self.native = rccl.world_from_dist(self.group)
        self.group_backend = dist.get_backend(self.group) if self.rank >= 0 else None
        self.backend = 'hetu-rccl' if self.native is not None else \
            (dist.get_backend(self.group) if self.rank >= 0 else 'non-member')

    # reference MPI_NCCL_Communicator fields (ctypes c_int: read through .value),
    # used by manual-pipeline scripts (examples/runner/parallel/complex_pipeline_mlp.py)
    @property
    def myRank(self):
        return _CInt(self.rank)

    @property
    def nRanks(self):
        return _CInt(self.nrank)

    @property
    def localRank(self):
        return _CInt(self.local_rank)

    @property
    def dev_id(self):
        return _CInt(self.device_id)

    # -- helpers ------------------------------------------------------------------
    def _g(self, r):
        """group rank -> global rank"""
        return r if self.ranks is None else self.ranks[r]

    def _avg(self, t, op):
        if op == 'mean':
            t.div_(self.nrank)

    # -- collectives ------------------------------------------------------------------
    def _gloo_gpu(self, t) -> bool:
        # gloo rehearsal of the GPU path (HETU_DIST_BACKEND=gloo, ranks sharing one GPU):
        # device tensors are staged through host memory here, synchronously, instead of
        # gloo's asynchronous CUDA-tensor work (four ranks on one GPU stalled inside it,
        # every rank parked in work.wait() of the first step's buckets)
        return t.is_cuda and self.group_backend == 'gloo'

    def _exchange64(self, payload, device):
        """all-gather of a <= 64-byte payload per rank (list of bytes, rank order)"""
        buf = torch.zeros(64, dtype=torch.uint8)
        buf[:len(payload)] = torch.tensor(list(payload), dtype=torch.uint8)
        buf = buf.to(device)
        out = torch.empty(64 * self.nrank, dtype=torch.uint8, device=device)
        self.all_gather(out, buf)
        host = out.cpu().numpy().tobytes()
        return [host[64 * j:64 * (j + 1)] for j in range(self.nrank)]

    def _ipc_ar(self, device):
        """the one-shot IPC all-reduce of this communicator (built on first use: one handle
        exchange over the communicator itself), or False when the ranks are not all on
        this node (``hipIpcOpenMemHandle`` maps same-node peers only)"""
        ar = getattr(self, '_ipc', None)
        if ar is None:
            import hashlib
            import socket
            node = hashlib.sha256(socket.gethostname().encode()).digest()[:32]
            if any(h[:32] != node for h in self._exchange64(node, device)):
                self._ipc = False
                return False
            from .ipc_allreduce import IPCAllReduce
            ar = self._ipc = IPCAllReduce(self.rank, self.nrank, lambda hb: self._exchange64(hb, device),
                                          device=device)
        return ar

    def all_reduce(self, t: torch.Tensor, op: str = 'sum', async_op: bool = False):
        if _IPC_SMALL and self.nrank > 1 and not async_op and op in ('sum', 'max') and t.is_cuda \
                and t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= 4096 \
                and getattr(self, '_ipc', None) is not False:
            # opt-in: small fp32 reductions by the one-shot IPC kernel (no RCCL call);
            # a peer timeout of any earlier call raises here (and in barrier / the watchdog)
            ar = self._ipc_ar(t.device)
            if ar:
                ar.check()
                ar(t, op, out=t)
                return None
        if self.native is not None and t.is_cuda and t.is_contiguous():
            return self.native.all_reduce(t, op, async_op=async_op)
        if self._gloo_gpu(t):
            h = t.detach().to('cpu')
            self.all_reduce(h, op)
            t.copy_(h)
            return _Done() if async_op else None
        if op == 'mean':
            w = dist.all_reduce(t, dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            if async_op:
                return _PostDiv(w, t, self.nrank)
            t.div_(self.nrank)
            return None
        return dist.all_reduce(t, _RED[op], group=self.group, async_op=async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """out = concat over ranks along dim 0."""
        if self.native is not None and out.is_cuda and out.is_contiguous():
            return self.native.all_gather(out, inp, async_op=async_op)
        if self._gloo_gpu(out):
            h = torch.empty(out.shape, dtype=out.dtype)
            self.all_gather(h, inp.detach().to('cpu'))
            out.copy_(h)
            return _Done() if async_op else None
        return dist.all_gather_into_tensor(out, inp.contiguous(), group=self.group, async_op=async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = 'sum', async_op: bool = False):
        """out = this rank's 1/P chunk (dim 0) of the reduction of ``inp``."""
        if self.native is not None and out.is_cuda and out.is_contiguous():
            return self.native.reduce_scatter(out, inp, op, async_op=async_op)
        if not self.use_gpu:
            # gloo has no reduce-scatter: all-reduce a copy and keep our chunk
            t = inp.contiguous().clone()
            dist.all_reduce(t, _RED.get(op, dist.ReduceOp.SUM), group=self.group)
            out.copy_(t.reshape(self.nrank, -1)[self.rank].reshape(out.shape))
            return _Done() if async_op else None
        return dist.reduce_scatter_tensor(out, inp.contiguous(), _RED.get(op, dist.ReduceOp.SUM),
                                          group=self.group, async_op=async_op)

    def broadcast(self, t: torch.Tensor, root: int = 0, async_op: bool = False):
        if self.native is not None and t.is_cuda and t.is_contiguous():
            return self.native.broadcast(t, root, async_op=async_op)
        if self._gloo_gpu(t):
            h = t.detach().to('cpu')
            self.broadcast(h, root)
            t.copy_(h)
            return _Done() if async_op else None
        return dist.broadcast(t, self._g(root), group=self.group, async_op=async_op)

    def reduce(self, t: torch.Tensor, root: int = 0, op: str = 'sum', async_op: bool = False):
        if self.native is not None and t.is_cuda and t.is_contiguous():
            return self.native.reduce(t, root, op, async_op=async_op)
        return dist.reduce(t, self._g(root), _RED[op], group=self.group, async_op=async_op)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """Equal ``numel/nranks`` chunks along dim 0 (reference AllToAll semantics)."""
        if self.native is not None and out.is_cuda and out.is_contiguous():
            return self.native.all_to_all(out, inp, async_op=async_op)
        return dist.all_to_all_single(out, inp.contiguous(), group=self.group, async_op=async_op)

    def send(self, t: torch.Tensor, dst: int):
        if self.native is not None and t.is_cuda:
            return self.native.p2p([('send', t.contiguous(), dst)])
        return dist.isend(t.contiguous(), self._g(dst), group=self.group)

    def recv(self, t: torch.Tensor, src: int):
        if self.native is not None and t.is_cuda and t.is_contiguous():
            return self.native.p2p([('recv', t, src)])
        return dist.irecv(t, self._g(src), group=self.group)

    def all_reduce_bf16(self, t: torch.Tensor, async_op: bool = False):
        """SUM of an fp32 tensor with bf16 on the wire and fp32 accumulation (native
        RCCL path, 16-byte aligned tensor).  Elsewhere a plain fp32 all-reduce."""
        if self.native is not None and t.is_cuda and t.is_contiguous() and t.dtype == torch.float32 \
                and t.data_ptr() % 16 == 0:
            return self.native.all_reduce_bf16(t, async_op=async_op)
        return self.all_reduce(t, 'sum', async_op=async_op)

    def batch_p2p(self, ops):
        """ops: list of ('send'|'recv', tensor, peer) issued as one RCCL group
        (reference GroupStart/GroupEnd around pipeline send/recv)."""
        if not ops:
            return []
        if self.native is not None and all(t.is_cuda and t.is_contiguous() for _, t, _ in ops):
            return [self.native.p2p(ops)]
        p2p = [dist.P2POp(dist.isend if k == 'send' else dist.irecv, t, self._g(p), group=self.group)
               for k, t, p in ops]
        return dist.batch_isend_irecv(p2p)

    def barrier(self):
        """host barrier: a 1-element all-reduce on the native communicator, then the host
        waits for it under the watchdog's deadline (torch's barrier would create torch's
        own RCCL communicator)"""
        if self.native is not None:
            if self._bar is None:
                self._bar = torch.zeros(1, dtype=torch.float32, device='cuda')
            self.native.all_reduce(self._bar)
            from ..runtime import DeviceEvent
            from . import watchdog
            ev = DeviceEvent().record(None)
            if watchdog.enabled():
                watchdog.get().wait(ev, 'barrier', self)
            else:
                ev.synchronize()
            if getattr(self, '_ipc', None):
                self._ipc.check()
        elif self.use_gpu and dist.get_backend(self.group) == 'nccl':
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    def health(self):
        """RCCL watchdog probe: 0 when healthy, else the communicator's
        asynchronous error code."""
        return self.native.async_error() if self.native is not None else 0

    def __repr__(self):
        return 'Communicator(rank=%d, nrank=%d, ranks=%s, backend=%s)' % (self.rank, self.nrank, self.ranks,
                                                                          self.backend)


class _Done(object):
    def wait(self):
        return True


class _PostDiv(object):
    def __init__(self, work, t, n):
        self.work, self.t, self.n = work, t, n

    def wait(self):
        self.work.wait()
        self.t.div_(self.n)


def stats():
    """{'backend', 'world', 'communicators'}: what this rank's comm layer holds (bench JSON)"""
    from . import rccl
    w = _WORLD
    return {'backend': w.backend if w is not None else 'none', 'world': w.nrank if w is not None else 1,
            'native_communicators': rccl.NativeComm.created,
            'groups': len(_GROUPS)}


def destroy():
    global _WORLD
    from . import watchdog
    for c in list(_GROUPS.values()) + ([_WORLD] if _WORLD is not None else []):
        if getattr(c, 'native', None) is not None:
            torch.cuda.synchronize()
            c.native.destroy()
            c.native = None
        if getattr(c, '_ipc', None):
            c._ipc.close()
    watchdog.shutdown()
    _GROUPS.clear()
    _WORLD = None
    if dist.is_initialized():
        dist.destroy_process_group()
