"""Pipeline parallelism over RCCL point-to-point (xGMI): tensor send/recv with a
shape header, and the GPipe / PipeDream-1F1B / HetPipe sub-executors
(reference pipeline_subexecutor.py, gpipe_subexecutor.py,
pipedream_subexecutor.py)."""
from __future__ import annotations

import torch

_DT = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16, 3: torch.int64, 4: torch.int32}
_DT_INV = {v: k for k, v in _DT.items()}
HDR = 10


def _header(t):
    """(ndim, dtype, shape...) built on the host and moved to the device in one copy"""
    h = torch.zeros(HDR, dtype=torch.int64)
    h[0] = t.dim()
    h[1] = _DT_INV[t.dtype]
    h[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
    return h.to(t.device, non_blocking=False)


def send_tensor(comm, t, dst, state=None):
    """Payload to ``dst`` (one RCCL group), preceded by a shape header only when this channel
    has not described it yet: ``state`` (per-op dict) caches the (dtype, shape) already sent,
    as the reference exchanges shapes only when its buffers are (re)allocated
    (gpu_ops/executor.py:774-833).  A channel with ``state=None`` sends a header every time."""
    t = t.contiguous()
    sig = (t.dtype, tuple(t.shape))
    if state is None or state.get('sig') != sig:
        if state is not None and 'sig' in state and not state.get('dynamic', False):
            raise RuntimeError('pipeline_send: shape changed from %s to %s on a static channel (create the op with '
                               'dynamic_shapes=True to re-send headers)' % (state['sig'], sig))
        for w in comm.batch_p2p([('send', _header(t), dst)]):
            w.wait()
        if state is not None:
            state['sig'] = sig
    for w in comm.batch_p2p([('send', t, dst)]):
        w.wait()


def recv_tensor(comm, src, device, state=None):
    """Payload from ``src``; the header is received (one host read) only on the first message
    of the channel (``state`` caches the shape), or every time with ``state=None``."""
    sig = state.get('sig') if state is not None else None
    if sig is None:
        hdr = torch.zeros(HDR, dtype=torch.int64, device=device)
        for w in comm.batch_p2p([('recv', hdr, src)]):
            w.wait()
        h = hdr.tolist()
        nd, dt = int(h[0]), _DT[int(h[1])]
        sig = (dt, tuple(int(x) for x in h[2:2 + nd]))
        if state is not None:
            state['sig'] = sig
    from .. import native_array as _NA
    out = _NA.empty(sig[1], dtype=sig[0], device=device)
    for w in comm.batch_p2p([('recv', out, src)]):
        w.wait()
    return out


def make_pipeline_subexecutor(kind, name, nodes, config):
    from .pipeline_exec import PipelineSubExecutor
    return PipelineSubExecutor(kind, name, nodes, config)
