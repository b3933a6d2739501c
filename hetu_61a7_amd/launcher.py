"""PS-role launcher (reference ``python/hetu/launcher.py:18-82``).

    python -m hetu_61a7_amd.launcher settings.yml -n 1 --sched

starts the scheduler (optional) and ``n`` server processes for a PS / Hybrid
job whose workers are launched separately; ``launch(target, args)`` runs
``target(args)`` in ``launch.worker`` local worker processes as well.  The
YAML file has the reference layout (``shared:`` env vars, ``launch:`` counts)
and is read with ``yaml.safe_load``.
"""
from __future__ import annotations

import argparse
import multiprocessing
import os
import signal

import yaml

_procs = []


def _settings(path):
    with open(path) as f:
        s = yaml.safe_load(f) or {}
    for k, v in (s.get('shared') or {}).items():
        os.environ[str(k)] = str(v)
    return s


def start_sched():
    os.environ['DMLC_ROLE'] = 'scheduler'
    from .ps import server
    server.scheduler_init()
    server.scheduler_finish()


def start_server():
    os.environ['DMLC_ROLE'] = 'server'
    from .ps import server
    server.run_server()


def start_worker(target, args):
    os.environ['DMLC_ROLE'] = 'worker'
    from .ps import worker
    worker.worker_init()
    target(args)
    worker.worker_finish()


def _stop(*_):
    for p in _procs:
        if p.is_alive():
            p.terminate()


def launch(target, args):
    s = _settings(args.config)
    ln = s.get('launch') or {}
    ctx = multiprocessing.get_context('spawn')
    for _ in range(int(ln.get('worker', 0))):
        _procs.append(ctx.Process(target=start_worker, args=(target, args)))
    for _ in range(int(ln.get('server', 0))):
        _procs.append(ctx.Process(target=start_server))
    if ln.get('scheduler'):
        _procs.append(ctx.Process(target=start_sched))
    signal.signal(signal.SIGINT, lambda *a: (_stop(), exit(0)))
    for p in _procs:
        p.start()
    for p in _procs:
        p.join()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('config')
    ap.add_argument('-n', type=int, default=1)
    ap.add_argument('--sched', action='store_true')
    a = ap.parse_args(argv)
    _settings(a.config)
    ctx = multiprocessing.get_context('spawn')
    if a.sched:
        _procs.append(ctx.Process(target=start_sched))
    for _ in range(a.n):
        _procs.append(ctx.Process(target=start_server))
    signal.signal(signal.SIGINT, lambda *x: (_stop(), exit(0)))
    for p in _procs:
        p.start()
    for p in _procs:
        p.join()


__all__ = ['launch']

if __name__ == '__main__':
    main()
