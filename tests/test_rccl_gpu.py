"""The in-house RCCL communicator (csrc/comm/hetu_comm.cc, parallel/rccl.py) and the
data-parallel gradient path on real RCCL, with one rank on the box's one GPU.

RCCL refuses two ranks on one device, so the multi-GPU path is rehearsed with a
single-rank communicator: every collective the DP / ZeRO / MoE / pipeline paths issue
goes through libhetu_comm.so -> RCCL on the communicator's own stream, and
``HETU_FORCE_DP=1`` runs the bucketed all-reduce machinery (async launch during the
backward pass, stream edges, bf16 wire with fp32 accumulation) for a one-rank job.
Each case runs in a fresh spawned process (process-group state is per process).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(port):
    os.environ.update(RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      HETU_USE_CONFIG='0')


def _primitives(port, q):
    try:
        _env(port)
        from hetu_61a7_amd.parallel import comm as C
        w = C.init_process_group(use_gpu=True)
        res = {'backend': w.backend}
        g = torch.Generator(device='cuda')
        g.manual_seed(3)
        t = torch.randn(1 << 20, device='cuda', generator=g)
        ref = t.clone()
        w.all_reduce(t, 'sum')
        res['sum'] = float((t - ref).abs().max())
        w.all_reduce(t, 'mean')
        res['mean'] = float((t - ref).abs().max())
        work = w.all_reduce(t, 'sum', async_op=True)
        work.wait()
        res['async'] = float((t - ref).abs().max())
        u = torch.randn(1000003, device='cuda', generator=g)   # not a multiple of 8: padded chunks
        uref = u.to(torch.bfloat16).float()
        w.all_reduce_bf16(u, async_op=True).wait()
        res['bf16'] = float((u - uref).abs().max())
        out = torch.empty(4096, device='cuda')
        w.reduce_scatter(out, ref[:4096])
        res['rs'] = float((out - ref[:4096]).abs().max())
        ag = torch.empty(4096, device='cuda')
        w.all_gather(ag, ref[:4096])
        res['ag'] = float((ag - ref[:4096]).abs().max())
        b = ref[:777].clone()
        w.broadcast(b, 0)
        res['bcast'] = float((b - ref[:777]).abs().max())
        a2a = torch.empty(8192, device='cuda')
        w.all_to_all(a2a, ref[:8192])
        res['a2a'] = float((a2a - ref[:8192]).abs().max())
        dst = torch.empty(513, device='cuda')
        works = w.batch_p2p([('send', ref[:513].contiguous(), 0), ('recv', dst, 0)])
        for x in works:
            x.wait()
        res['p2p'] = float((dst - ref[:513]).abs().max())
        res['health'] = w.health()
        torch.cuda.synchronize()
        C.destroy()
        q.put(res)
    except Exception as e:  # report, do not hang the parent
        q.put({'error': repr(e)})


def _spawn(target, *args):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=target, args=(_free_port(), q) + args)
    p.start()
    res = q.get(timeout=110)
    p.join(30)
    assert p.exitcode == 0, res
    assert 'error' not in res, res
    return res


def test_native_rccl_collectives_one_rank():
    res = _spawn(_primitives)
    assert res['backend'] == 'hetu-rccl', res
    for k in ('sum', 'mean', 'async', 'rs', 'ag', 'bcast', 'a2a', 'p2p'):
        assert res[k] == 0.0, (k, res)
    assert res['bf16'] == 0.0, res   # one rank: the bf16 wire rounds once, the fp32 sum is exact
    assert res['health'] == 0


def _mlp(X, Y, dp, wire, steps=6):
    import hetu_61a7_amd as ht
    rng = np.random.RandomState(5)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W1 = ht.Variable(name='w1', value=(rng.randn(64, 256) * 0.1).astype(np.float32))
    B1 = ht.Variable(name='b1', value=np.zeros(256, np.float32))
    W2 = ht.Variable(name='w2', value=(rng.randn(256, 256) * 0.1).astype(np.float32))
    W3 = ht.Variable(name='w3', value=(rng.randn(256, 16) * 0.1).astype(np.float32))
    h = ht.relu_op(ht.linear_op(x, W1, B1))
    h = ht.relu_op(ht.matmul_op(h, W2))
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(h, W3), y_), [0])
    train = ht.optim.MomentumOptimizer(0.05, 0.9).minimize(loss)
    kw = dict(bucket_mb=0.1, grad_wire=wire)
    if dp:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), **kw)
    out = [float(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]) for _ in range(steps)]
    info = dict(is_dp=bool(train.dp), buckets=len(train.buckets), backend=getattr(train.comm, 'backend', None))
    return out, info


def _forced_dp(port, q, wire):
    try:
        _env(port)
        os.environ['HETU_FORCE_DP'] = '1'
        rng = np.random.RandomState(0)
        X = rng.randn(128, 64).astype(np.float32)
        Y = np.eye(16, dtype=np.float32)[rng.randint(0, 16, 128)]
        dp_losses, info = _mlp(X, Y, True, wire)
        os.environ['HETU_FORCE_DP'] = '0'
        base, _ = _mlp(X, Y, False, 'fp32')
        torch.cuda.synchronize()
        from hetu_61a7_amd.parallel import comm as C
        C.destroy()
        q.put(dict(dp=dp_losses, base=base, **info))
    except Exception as e:
        q.put({'error': repr(e)})


@pytest.mark.parametrize('wire', ['fp32', 'bf16'])
def test_forced_single_rank_dp_on_rccl(wire):
    res = _spawn(_forced_dp, wire)
    assert res['is_dp'] and res['backend'] == 'hetu-rccl', res
    assert res['buckets'] >= 2, res          # several buckets launched during the backward pass
    dp, base = np.array(res['dp']), np.array(res['base'])
    assert np.all(np.isfinite(dp)) and dp[-1] < dp[0], res
    tol = 1e-5 if wire == 'fp32' else 2e-2   # bf16 wire rounds every gradient once
    np.testing.assert_allclose(dp, base, rtol=tol, atol=tol)


def _multi_device(port, q):
    try:
        from hetu_61a7_amd.parallel.rccl import MultiDeviceComm
        devs = list(range(torch.cuda.device_count()))
        mc = MultiDeviceComm(devs)
        ts = [torch.full((4096,), float(i + 1), device='cuda:%d' % d) for i, d in enumerate(devs)]
        mc.all_reduce(ts)
        want = float(sum(range(1, len(devs) + 1)))
        res = {'n': len(devs), 'ar': max(float((t - want).abs().max()) for t in ts)}
        n = len(devs)
        ins = [torch.arange(n * 8, dtype=torch.float32, device='cuda:%d' % d) + 100 * i for i, d in enumerate(devs)]
        outs = [torch.empty_like(x) for x in ins]
        mc.all_to_all(outs, ins)
        for d in devs:
            torch.cuda.synchronize(d)
        # chunk j of device i's output came from device j's chunk i
        err = 0.0
        for i in range(n):
            for j in range(n):
                err = max(err, float((outs[i][j * 8:(j + 1) * 8] - ins[j][i * 8:(i + 1) * 8]).abs().max()))
        res['a2a'] = err
        mc.destroy()
        q.put(res)
    except Exception as e:
        q.put({'error': repr(e)})


def test_single_process_multi_device_comm():
    """ncclCommInitAll communicator driving every visible GPU from one process (one on
    the test box): grouped all-reduce and all-to-all."""
    res = _spawn(_multi_device)
    assert res['n'] >= 1 and res['ar'] == 0.0 and res['a2a'] == 0.0, res


def _watchdog_step(port, q):
    try:
        _env(port)
        os.environ['HETU_FORCE_DP'] = '1'
        os.environ['HETU_WATCHDOG_POLL'] = '0.02'
        from hetu_61a7_amd.parallel import watchdog
        rng = np.random.RandomState(0)
        X = rng.randn(128, 64).astype(np.float32)
        Y = np.eye(16, dtype=np.float32)[rng.randint(0, 16, 128)]
        losses, info = _mlp(X, Y, True, 'fp32')
        wd = watchdog.get()
        from hetu_61a7_amd.parallel import comm as C
        C.world().barrier()                       # host wait under the deadline
        torch.cuda.synchronize()
        import time
        time.sleep(0.1)                           # a few polls after the last collective
        st = wd.stats()
        C.destroy()                               # stops the monitor thread
        q.put(dict(stats=st, losses=losses, after=watchdog._WD is None and not wd.running,
                   failed=wd.failed, **info))
    except Exception as e:
        q.put({'error': repr(e)})


def test_watchdog_monitors_training_step():
    """the watchdog starts with the native communicator, tracks the
    bucketed all-reduces of forced single-rank DP steps until they complete, polls the
    communicator's async error state, and stops cleanly at comm.destroy()."""
    res = _spawn(_watchdog_step)
    st = res['stats']
    assert res['backend'] == 'hetu-rccl', res
    assert st['running'] and st['polls'] >= 3 and st['communicators'] >= 1, st
    assert st['tracked'] >= res['buckets'] and st['in_flight'] == 0, st
    assert st['completed'] == st['tracked'], st
    assert res['failed'] is None and res['after'], res
