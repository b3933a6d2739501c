"""Pipeline parallelism over RCCL point-to-point (xGMI): tensor send/recv with a
shape header, and the GPipe / PipeDream-1F1B / HetPipe sub-executors
(reference pipeline_subexecutor.py, gpipe_subexecutor.py,
pipedream_subexecutor.py)."""
from __future__ import annotations

import torch

_DT = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16, 3: torch.int64, 4: torch.int32}
_DT_INV = {v: k for k, v in _DT.items()}
HDR = 10


def send_tensor(comm, t, dst):
    """Header (ndim, dtype, shape...) then payload, one RCCL group."""
    t = t.contiguous()
    hdr = torch.zeros(HDR, dtype=torch.int64, device=t.device)
    hdr[0] = t.dim()
    hdr[1] = _DT_INV[t.dtype]
    hdr[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
    for w in comm.batch_p2p([('send', hdr, dst)]):
        w.wait()
    for w in comm.batch_p2p([('send', t, dst)]):
        w.wait()


def recv_tensor(comm, src, device):
    hdr = torch.zeros(HDR, dtype=torch.int64, device=device)
    for w in comm.batch_p2p([('recv', hdr, src)]):
        w.wait()
    h = hdr.tolist()
    nd, dt = int(h[0]), _DT[int(h[1])]
    shape = tuple(int(x) for x in h[2:2 + nd])
    out = torch.empty(shape, dtype=dt, device=device)
    for w in comm.batch_p2p([('recv', out, src)]):
        w.wait()
    return out


def make_pipeline_subexecutor(kind, name, nodes, config):
    from .pipeline_exec import PipelineSubExecutor
    return PipelineSubExecutor(kind, name, nodes, config)
