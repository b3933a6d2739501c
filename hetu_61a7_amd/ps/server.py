"""PS server / scheduler roles (reference ps-lite server + launcher.py:18-82).

The server creates the shared-memory segment (``/hetu_ps_<port>``) that holds
every parameter table in host DRAM, then waits until every worker has
finalised.  The scheduler role has nothing to coordinate on one node beyond
what the segment's header does (barriers, heartbeats, SSP, PReduce) and simply
returns.

    python -m hetu_61a7_amd.ps                # DMLC_ROLE=server
"""
from __future__ import annotations

import os

from ._lib import lib, check
from .worker import shm_name

_ROLE = None


def _heap_bytes():
    gb = float(os.environ.get('HETU_PS_HEAP_GB', '8'))
    return int(gb * (1 << 30))


def server_init():
    global _ROLE
    nw = int(os.environ.get('DMLC_NUM_WORKER', '1'))
    ns = int(os.environ.get('DMLC_NUM_SERVER', '1'))
    check(lib('hps_init')(1, shm_name().encode(), nw, ns, _heap_bytes()), 'server init')
    _ROLE = 'server'


def server_finish(timeout_s=0.0):
    global _ROLE
    if _ROLE == 'server':
        lib('hps_server_wait_shutdown')(float(timeout_s))
        lib('hps_finalize')()
    _ROLE = None


def scheduler_init():
    global _ROLE
    _ROLE = 'scheduler'


def scheduler_finish():
    global _ROLE
    _ROLE = None


def run_server(poll_s=2.0):
    """Serve until all workers finalised; exits early if the launcher died
    (re-parented process), so a crashed job never leaves a server behind."""
    global _ROLE
    server_init()
    parent = os.getppid()
    while lib('hps_server_wait_shutdown')(float(poll_s)) != 0:
        if os.getppid() != parent:
            break
    lib('hps_finalize')()
    _ROLE = None


if __name__ == '__main__':
    role = os.environ.get('DMLC_ROLE', 'server')
    if role == 'server':
        run_server()
    else:
        scheduler_init()
        scheduler_finish()
