"""Piecewise hipGraph replay of a parameter-server step (utils/piecewise.py): pure-PS
Wide&Deep on the GPU -- PS lookups, gradient staging and the PS optimizer run eagerly, the
dense segments between them replay as captured graphs.  Under BSP the losses must equal
eager execution's; under ASP with prefetch (the bench default) the runner must replay and
train."""
import os
import uuid

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROWS, EMB, B = 2000, 16, 64


def _server(env):
    os.environ.update(env)
    from hetu_61a7_amd.ps import server
    server.server_init()
    server.server_finish(timeout_s=180)


def _worker(env, q, bsp, steps):
    os.environ.update(env)
    os.environ.update(RANK='0', LOCAL_RANK='0', DMLC_ROLE='worker')
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models.ctr import wdl_criteo, synthetic_criteo
    dense, sparse, labels = synthetic_criteo(B * 4, ROWS, seed=3)
    xd = ht.dataloader_op([ht.Dataloader(dense, B, 'train')])
    xs = ht.dataloader_op([ht.Dataloader(sparse, B, 'train')])
    y_ = ht.dataloader_op([ht.Dataloader(labels, B, 'train')])
    loss, y, _, train = wdl_criteo(xd, xs, y_, feature_dimension=ROWS, embedding_size=EMB, learning_rate=0.5)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), comm_mode='PS', cstable_policy=None,
                     bsp=bsp, prefetch=bsp < 0, seed=7)
    losses = [float(np.asarray(ex.run('train', convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
              for _ in range(steps)]
    sub = ex.subexecutor['train']
    pw = sub.piecewise
    info = None if pw is None else (pw.replays, pw.failed, sum(1 for s in pw.segments or () if not s.host),
                                    sum(1 for s in pw.segments or () if s.host))
    op = sub.opt_ops[0]
    if op.ps_dense is not None:
        op.ps_dense.drain()
    q.put((losses, info))
    ex.config.ps_comm.BarrierWorker()
    from hetu_61a7_amd.ps import worker
    worker.worker_finish()


def _run(bsp, piecewise, steps=12):
    env = dict(DMLC_PS_ROOT_PORT=str(20000 + uuid.uuid4().int % 30000), DMLC_NUM_WORKER='1',
               DMLC_NUM_SERVER='1', HETU_PS_HEAP_GB='0.2', WORLD_SIZE='1', HETU_USE_CONFIG='0',
               HSA_ENABLE_IPC_MODE_LEGACY='0', HETU_PIECEWISE_GRAPH='1' if piecewise else '0')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    srv = ctx.Process(target=_server, args=(env,))
    srv.start()
    w = ctx.Process(target=_worker, args=(env, q, bsp, steps))
    w.start()
    import queue
    import time
    t0 = time.time()
    while True:                       # fail as soon as the worker dies (no 240 s silent wait)
        try:
            res = q.get(timeout=5)
            break
        except queue.Empty:
            if not w.is_alive() or time.time() - t0 > 150:
                w.kill()
                srv.kill()
                raise AssertionError('worker exited %s without a result' % w.exitcode)
    w.join(60)
    srv.join(60)
    assert w.exitcode == 0 and srv.exitcode == 0
    return res


def test_piecewise_bsp_matches_eager():
    eager, info0 = _run(0, False)
    pw, info = _run(0, True)
    assert info0 is None
    replays, failed, dev_segs, host_segs = info
    assert not failed and dev_segs >= 2 and host_segs >= 2 and replays >= dev_segs * 9, info
    np.testing.assert_allclose(pw, eager, rtol=1e-5, atol=1e-6)


def test_piecewise_asp_prefetch_replays_and_trains():
    pw, info = _run(-1, True, steps=30)
    replays, failed, dev_segs, host_segs = info
    assert not failed and replays > 0, info
    assert np.isfinite(pw).all() and pw[-1] < pw[0], pw
