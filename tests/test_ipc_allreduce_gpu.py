"""One-shot IPC all-reduce (parallel/ipc_allreduce.py): two processes on the same GPU
exchange their slab handles over a gloo group, then run sum / max reductions of random
sizes back to back; each must equal the reduction of both ranks' inputs (regenerated
from the seeds), and no call may time out."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W = 2


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(it, rank):
    rng = np.random.RandomState(1000 * it + rank)
    n = int(np.random.RandomState(it).randint(1, 4097))
    return rng.randn(n).astype(np.float32)


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=W)
    try:
        from hetu_61a7_amd.parallel.ipc_allreduce import IPCAllReduce
        torch.cuda.set_device(0)

        def exchange(hb):
            out = [None] * W
            dist.all_gather_object(out, hb)
            return out
        ar = IPCAllReduce(rank, W, exchange, device='cuda:0')
        bad = []
        for it in range(40):
            op = 'max' if it % 3 == 2 else 'sum'
            x = torch.tensor(_inputs(it, rank), device='cuda')
            y = ar(x, op).cpu().numpy()
            xs = [_inputs(it, r) for r in range(W)]
            ref = np.maximum.reduce(xs) if op == 'max' else np.sum(xs, 0)
            if not np.allclose(y, ref, rtol=1e-6, atol=1e-6):
                bad.append((it, op, float(np.abs(y - ref).max())))
        ar.check()
        dist.barrier()
        ar.close()
        q.put((rank, bad, None))
    except Exception as e:       # noqa: BLE001 -- reported to the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_ipc_allreduce_two_processes_one_gpu():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, bad, err in res:
        assert err is None, (rank, err)
        assert not bad, (rank, bad[:5])


def _comm_rank(rank, port, q, stall):
    # Communicator-level route: HETU_IPC_ALLREDUCE=1 sends small fp32 all-reduces through
    # the IPC kernel (ranks share the GPU over a gloo group; the handle exchange and the
    # same-node check run over the Communicator itself)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0',
                      HETU_IPC_ALLREDUCE='1', HETU_DIST_BACKEND='gloo', RANK=str(rank), WORLD_SIZE=str(W),
                      LOCAL_RANK='0', HETU_WATCHDOG='0')
    try:
        torch.cuda.set_device(0)
        from hetu_61a7_amd.parallel import comm, ipc_allreduce
        ipc_allreduce.SPIN_CAP = 1 << 18          # a missing peer times out quickly
        c = comm.init_process_group(use_gpu=True)
        bad = []
        for it in range(6):
            x = torch.tensor(_inputs(it, rank), device='cuda')
            c.all_reduce(x, 'sum')
            ref = np.sum([_inputs(it, r) for r in range(W)], 0)
            if not np.allclose(x.cpu().numpy(), ref, rtol=1e-6, atol=1e-6):
                bad.append(it)
        routed = bool(getattr(c, '_ipc', None))
        raised = None
        if stall:
            import torch.distributed as dist
            dist.barrier()
            if rank == 0:
                # rank 1 never joins this call: the kernel gives up, records the epoch,
                # and the next routed call raises instead of returning stale sums
                y = torch.ones(8, device='cuda')
                c.all_reduce(y, 'sum')
                torch.cuda.synchronize()
                try:
                    c.all_reduce(torch.ones(8, device='cuda'), 'sum')
                except RuntimeError as e:
                    raised = str(e)
            dist.barrier()
        q.put((rank, bad, routed, raised, None))
    except Exception as e:       # noqa: BLE001 -- reported to the parent
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.parametrize('stall', [False, True])
def test_ipc_allreduce_through_communicator(stall):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_comm_rank, args=(r, port, q, stall)) for r in range(W)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    for rank, bad, routed, raised, err in res:
        assert err is None, (rank, err)
        assert not bad, (rank, bad)
        assert routed, rank
        if stall and rank == 0:
            assert raised is not None and 'timed out' in raised, raised
