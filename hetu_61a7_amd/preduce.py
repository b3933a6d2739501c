"""Partial reduce (reference ``python/hetu/preduce.py:8-42``; server side
``ps-lite/src/preduce_handler.cc:6-56``).

A worker asks the parameter server for a *partner set*: the server groups the
workers that arrive within ``wait_time`` ms (up to ``max_worker``) and hands
every member the same sorted rank tuple.  The partners then average a tensor
with one all-reduce on a communicator built for exactly that set (RCCL over
xGMI on GPUs, gloo on CPU).  Partner sets are dynamic, so their communicators
are created with member-only synchronisation and cached per set.

    pr = PartialReduce(reduce_key=stage_id)
    partner = pr.get_partner(max_worker=-1, wait_time=1.0)
    pr.preduce(weight_tensor, partner)          # in place, mean over partners
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch


class PartialReduce(object):
    def __init__(self, reduce_key=0, comm=None, ps_comm=None):
        from .launcher_api import get_worker_communicate, wrapped_mpi_nccl_init
        self._reduce_key = int(reduce_key)
        self.ps_comm = ps_comm if ps_comm is not None else get_worker_communicate()
        self.comm = comm if comm is not None else wrapped_mpi_nccl_init()
        self._comm_map: Dict[Tuple[int, ...], object] = {}
        self.rank = self.comm.rank
        self.nrank = self.comm.nrank

    def get_partner(self, max_worker=-1, wait_time=1.0) -> Tuple[int, ...]:
        """Block until the server closes this worker's partner set.

        ``wait_time`` is in milliseconds; ``max_worker`` closes the set early
        once that many workers joined (``-1``: all workers)."""
        if max_worker < 0:
            max_worker = self.nrank
        members = self.ps_comm.preduce_get_partner(self._reduce_key, self.rank, max_worker, float(wait_time))
        return tuple(sorted(int(r) for r in members))

    def preduce(self, array, partner, stream=None):
        """In-place mean of ``array`` over ``partner`` (a rank tuple)."""
        partner = tuple(sorted(int(r) for r in partner))
        if len(partner) <= 1:
            return array
        t = array.tensor if hasattr(array, 'tensor') else array
        comm = self._get_comm(partner)
        if stream is not None and hasattr(stream, 'torch_stream') and stream.torch_stream is not None:
            from .runtime import use_stream
            with use_stream(stream):
                comm.all_reduce(t, 'mean')
        else:
            comm.all_reduce(t, 'mean')
        return array

    def _get_comm(self, partner):
        c = self._comm_map.get(partner)
        if c is None:
            from .parallel.comm import new_group_comm
            c = new_group_comm(partner, local_sync=True)
            self._comm_map[partner] = c
        return c

    _create_partial_comm = _get_comm
