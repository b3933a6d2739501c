"""Process bootstrap entry points (reference executor.py:60-131).

``wrapped_mpi_nccl_init`` brings up the global RCCL communicator (TCP-store
rendezvous; honours ``mpirun``'s OMPI_* variables); the PS role functions start
the C++ parameter-server roles (``ps`` package).
"""
from __future__ import annotations


def wrapped_mpi_nccl_init(init_nccl=True, devices=None):
    from .parallel import comm
    return comm.init_process_group()


def get_worker_communicate():
    from .ps import worker
    return worker.get_agent()


def worker_init():
    from .ps import worker
    return worker.worker_init()


def worker_finish():
    from .ps import worker
    return worker.worker_finish()


def server_init():
    from .ps import server
    return server.server_init()


def server_finish():
    from .ps import server
    return server.server_finish()


def scheduler_init():
    from .ps import server
    return server.scheduler_init()


def scheduler_finish():
    from .ps import server
    return server.scheduler_finish()
