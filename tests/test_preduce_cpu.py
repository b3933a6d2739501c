"""Partial reduce: PS partner matching + member-only group all-reduce (mean).

Reference pattern: tests/test_ps_preduce.py (staggered workers, partner groups);
semantics from python/hetu/preduce.py:20-42.  Runs 1 PS server + 3 workers on
CPU (gloo)."""
import os
import socket
import time
import uuid

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _server(env):
    os.environ.update(env)
    os.environ['DMLC_ROLE'] = 'server'
    from hetu_61a7_amd.ps import server
    server.server_init()
    server.server_finish(timeout_s=120)


def _worker(rank, env, q):
    os.environ.update(env)
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), DMLC_ROLE='worker')
    from hetu_61a7_amd.ps import worker
    from hetu_61a7_amd.preduce import PartialReduce
    from hetu_61a7_amd.parallel import comm
    ag = worker.worker_init()
    world = comm.init_process_group(use_gpu=False)
    pr = PartialReduce(reduce_key=0, comm=world, ps_comm=ag)
    out = {}
    # round 1: everybody joins -> full set, mean of ranks
    p1 = pr.get_partner(max_worker=-1, wait_time=5000.0)
    t = torch.full((16,), float(world.rank))
    pr.preduce(t, p1)
    out['p1'], out['v1'] = p1, float(t[0])
    ag.BarrierWorker()
    # round 2: worker 2 arrives late; the first two close a set of size 2
    if world.rank == 2:
        time.sleep(1.5)
        p2 = pr.get_partner(max_worker=2, wait_time=200.0)
    else:
        p2 = pr.get_partner(max_worker=2, wait_time=5000.0)
    t = torch.full((4,), float(world.rank) * 2)
    pr.preduce(t, p2)
    out['p2'], out['v2'] = p2, float(t[0])
    ag.BarrierWorker()
    q.put((world.rank, out))
    worker.worker_finish()
    comm.destroy()


def test_partial_reduce_partner_groups():
    nw = 3
    port = 20000 + (uuid.uuid4().int % 20000)
    env = dict(DMLC_PS_ROOT_PORT=str(port), DMLC_NUM_WORKER=str(nw), DMLC_NUM_SERVER='1',
               HETU_PS_HEAP_GB='0.1', WORLD_SIZE=str(nw), MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(_free_port()))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    srv = ctx.Process(target=_server, args=(env,))
    srv.start()
    ws = [ctx.Process(target=_worker, args=(r, env, q)) for r in range(nw)]
    for w in ws:
        w.start()
    res = dict(q.get(timeout=120) for _ in ws)
    for w in ws:
        w.join(60)
        assert w.exitcode == 0
    srv.join(60)
    for r in range(nw):
        assert res[r]['p1'] == (0, 1, 2)
        assert res[r]['v1'] == pytest.approx(1.0)
    assert res[0]['p2'] == (0, 1) and res[1]['p2'] == (0, 1)
    assert res[0]['v2'] == pytest.approx(1.0)   # mean(0, 2)
    assert res[2]['p2'] == (2,)
    assert res[2]['v2'] == pytest.approx(4.0)   # alone: unchanged
