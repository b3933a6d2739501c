"""``heturun``: single-node job launcher (reference ``python/runner.py:25-252``,
``bin/heturun``).

    heturun -w 8 python train.py ...            # 8 GPU workers (one process per GPU)
    heturun -w 8 -s 1 python run_ctr.py ...     # + 1 PS server (Hybrid / PS jobs)
    heturun -c cluster.yml python train.py      # counts from a YAML spec
    heturun -w 8 --max-restarts 3 python train.py   # elastic: restart the group
                                                    # on a worker failure

Elastic recovery (SURVEY §5.3 "abort and restart from checkpoint", not
present in the reference): when a worker exits non-zero (an RCCL watchdog
abort, ``HETU_COMM_TIMEOUT``, a crash), every process of the group is stopped
and the whole group is relaunched on a fresh rendezvous port, up to
``max_restarts`` times.  Each attempt sees ``HETU_RESTART_COUNT``; the training
script resumes with ``utils.checkpoint.resume(ex, dir)`` from the last
atomically committed ``utils.checkpoint.save_resumable`` snapshot.

The reference wrapped ``mpirun`` and ssh; on one MI355X node every worker is a
local process with the torch.distributed environment (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) plus the ps-lite variables
(DMLC_ROLE, DMLC_PS_ROOT_URI/PORT, DMLC_NUM_WORKER/SERVER) -- RCCL rendezvous
goes through the TCP store, no MPI needed.  YAML spec (``yaml.safe_load``)::

    nodes:
      - host: localhost
        workers: 8
        servers: 1
    shared: {DMLC_PS_VAN_TYPE: shm}
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time

import yaml


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parse_config(path):
    with open(path) as f:
        spec = yaml.safe_load(f) or {}
    workers = servers = 0
    for node in spec.get('nodes', []):
        host = str(node.get('host', 'localhost'))
        if host not in ('localhost', '127.0.0.1', socket.gethostname()):
            raise SystemExit('heturun: multi-host specs are not supported on this build (%s)' % host)
        workers += int(node.get('workers', 0))
        servers += int(node.get('servers', 0))
    return workers, servers, {str(k): str(v) for k, v in (spec.get('shared') or {}).items()}


def launch(command, workers, servers=0, shared=None, env=None, poll=0.2, max_restarts=0):
    """Start servers then workers; returns the first non-zero worker exit code.

    With ``max_restarts > 0`` a failed group is torn down and relaunched (new
    MASTER_PORT / PS root port, ``HETU_RESTART_COUNT`` incremented) until it
    succeeds or the restarts are used up."""
    base = dict(os.environ if env is None else env)
    rc = 0
    for attempt in range(max_restarts + 1):
        e = dict(base, HETU_RESTART_COUNT=str(attempt))
        if attempt:
            e.pop('MASTER_PORT', None)
            e.pop('DMLC_PS_ROOT_PORT', None)
            print('heturun: worker group failed (rc=%d); restart %d/%d' % (rc, attempt, max_restarts),
                  file=sys.stderr, flush=True)
        rc = _launch_once(command, workers, servers, shared, e, poll)
        if rc == 0 or rc == 130:
            return rc
    return rc


def _launch_once(command, workers, servers, shared, base, poll):
    base = dict(base)
    base.update(shared or {})
    port = int(base.get('MASTER_PORT') or _free_port())
    base.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(workers),
                DMLC_PS_ROOT_URI='127.0.0.1', DMLC_NUM_WORKER=str(workers),
                DMLC_NUM_SERVER=str(max(servers, 1)))
    base.setdefault('DMLC_PS_ROOT_PORT', str(_free_port()))
    procs = []
    for i in range(servers):
        e = dict(base, DMLC_ROLE='server', DMLC_SERVER_ID=str(i))
        procs.append(('server', subprocess.Popen([sys.executable, '-m', 'hetu_61a7_amd.ps'], env=e)))
    ws = []
    for r in range(workers):
        e = dict(base, DMLC_ROLE='worker', RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(workers))
        p = subprocess.Popen(command, env=e)
        ws.append(p)
        procs.append(('worker', p))

    def stop(*_):
        for _, p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGINT, lambda *a: (stop(), sys.exit(130)))
    rc = 0
    while any(p.poll() is None for p in ws):
        for p in ws:
            c = p.poll()
            if c not in (None, 0):
                rc = rc or c
                stop()
        time.sleep(poll)
    rc = rc or next((p.returncode for p in ws if p.returncode), 0)
    for kind, p in procs:
        if kind == 'server':
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.terminate()
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(prog='heturun')
    ap.add_argument('-c', '--config', default=None, help='YAML cluster spec')
    ap.add_argument('-w', '--workers', type=int, default=0)
    ap.add_argument('-s', '--servers', type=int, default=0)
    ap.add_argument('--max-restarts', type=int, default=int(os.environ.get('HETU_MAX_RESTARTS', '0')),
                    help='relaunch the worker group this many times after a failure')
    ap.add_argument('command', nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    shared = {}
    w, s = a.workers, a.servers
    if a.config:
        cw, cs, shared = parse_config(a.config)
        w, s = w or cw, s or cs
    if not a.command:
        ap.error('no command given')
    return launch(a.command, max(w, 1), s, shared, max_restarts=a.max_restarts)


if __name__ == '__main__':
    sys.exit(main())
