"""heturun launcher: 2 workers + 1 PS server on CPU (gloo)."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_heturun_workers_and_server(tmp_path):
    script = tmp_path / 'job.py'
    script.write_text(textwrap.dedent('''
        import os, torch
        import torch.distributed as dist
        from hetu_61a7_amd.parallel import comm
        from hetu_61a7_amd.ps import worker
        c = comm.init_process_group(use_gpu=False)
        t = torch.ones(4) * (c.rank + 1)
        c.all_reduce(t)
        ag = worker.worker_init()
        ag.InitTensor(5, 0, 8, 1, 0, 0.0, 0.0, 0)
        ag.WaitTicket(ag.Push(5, torch.ones(8)))
        ag.BarrierWorker()
        v = torch.zeros(8)
        ag.WaitTicket(ag.Pull(5, v))
        assert float(t[0]) == 3.0 and float(v[0]) == 2.0, (t, v)
        worker.worker_finish()
        comm.destroy()
        print('OK', os.environ['RANK'])
    '''))
    env = dict(os.environ, PYTHONPATH=ROOT, HETU_PS_HEAP_GB='0.05')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bin', 'heturun'), '-w', '2', '-s', '1',
                        sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'OK 0' in r.stdout and 'OK 1' in r.stdout
