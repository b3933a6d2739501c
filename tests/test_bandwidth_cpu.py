"""Bandwidth tests in the reference's style (tests/test_nccl_bandwidth.py,
tests/pstests/test_bandwidth.py): collective bandwidth sweep through
NCCLProfiler on a 2-rank group, and PS dense push/pull throughput through the
shared-memory van (1 server + 2 workers under heturun).  On CPU these check
the plumbing and the busbw arithmetic and print the measured rates; on an
MI355X node the same NCCLProfiler runs over RCCL."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HETU_USE_CONFIG='0')
    from hetu_61a7_amd.parallel import comm as C
    from hetu_61a7_amd.utils.profiler import NCCLProfiler
    c = C.init_process_group(use_gpu=False)
    res = NCCLProfiler(c).bandwidth_sweep(sizes=(1 << 12, 1 << 18))
    p2p = NCCLProfiler(c).profile_sendrecv(1 << 16, iters=5)
    q.put((rank, res, p2p))
    C.destroy()


def test_collective_bandwidth_sweep():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, res, p2p in out:
        assert set(res) == {1 << 12, 1 << 18}
        for size, r in res.items():
            assert r['ms'] > 0 and r['algbw_GBps'] > 0
            assert abs(r['busbw_GBps'] - r['algbw_GBps']) < 1e-9 * max(1.0, r['algbw_GBps'])   # n=2: 2(n-1)/n = 1
        assert set(p2p) == {(0, 1), (1, 0)}
        print('rank', rank, {k: round(v['busbw_GBps'], 3) for k, v in res.items()})


def test_ps_push_pull_bandwidth(tmp_path):
    script = tmp_path / 'bw.py'
    script.write_text(textwrap.dedent('''
        import os, time, torch
        from hetu_61a7_amd.ps import worker
        ag = worker.worker_init()
        n = 1 << 20                                  # 4 MiB fp32 per transfer
        ag.InitTensor(11, 0, n, 1, 0, 0.0, 0.0, 0)
        ag.BarrierWorker()
        g, v = torch.ones(n), torch.zeros(n)
        iters = 10
        t0 = time.perf_counter()
        for _ in range(iters):
            ag.WaitTicket(ag.Push(11, g))
            ag.WaitTicket(ag.Pull(11, v))
        dt = time.perf_counter() - t0
        ag.BarrierWorker()
        ag.WaitTicket(ag.Pull(11, v))
        workers = int(os.environ['DMLC_NUM_WORKER'])
        assert float(v[0]) == float(iters * workers), float(v[0])   # every push landed
        print('BW rank %s %.3f GB/s' % (os.environ['RANK'], 2 * iters * n * 4 / dt / 1e9))
        worker.worker_finish()
    '''))
    env = dict(os.environ, PYTHONPATH=ROOT, HETU_PS_HEAP_GB='0.1')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bin', 'heturun'), '-w', '2', '-s', '1',
                        sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    rates = [float(l.split()[3]) for l in r.stdout.splitlines() if l.startswith('BW rank')]
    assert len(rates) == 2 and min(rates) > 0, r.stdout
