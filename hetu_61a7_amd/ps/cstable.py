"""HET cache table (reference ``python/hetu/cstable.py:19-211``) over the C++
cache (csrc/cache/het_cache.cc).  Keys are int64 (no float-encoded ids)."""
from __future__ import annotations

import numpy as np
import torch

from ._lib import lib, ptr
from .worker import get_agent

POLICIES = {'lru': 0, 'lfu': 1, 'lfuopt': 2}


class CacheSparseTable(object):
    def __init__(self, limit, length, width, node_id, policy='LRU', bound=100):
        self.agent = get_agent()
        self.width = width
        self.node_id = node_id
        self.handle = lib('hc_create')(POLICIES[policy.lower()], int(limit), int(length), int(width),
                                       int(node_id), int(bound), int(bound))
        self.keep = {}
        self.agent.BarrierWorker()

    @property
    def pull_bound(self):
        return self._pull

    def set_bounds(self, pull, push):
        lib('hc_set_bounds')(self.handle, int(pull), int(push))

    def _k(self, keys):
        if isinstance(keys, np.ndarray):
            keys = torch.from_numpy(np.ascontiguousarray(keys.astype(np.int64)))
        return keys.reshape(-1).long().contiguous()

    def embedding_lookup(self, keys, dest, sync=False):
        k = self._k(keys)
        assert dest.numel() == k.numel() * self.width
        t = lib('hc_async_lookup')(self.handle, ptr(k), k.numel(), ptr(dest))
        self.keep[t] = (k, dest)
        if sync:
            self.wait(t)
            return None
        return t

    def embedding_update(self, keys, grads, sync=False):
        k = self._k(keys)
        g = grads.reshape(-1, self.width).float().contiguous()
        t = lib('hc_async_update')(self.handle, ptr(k), k.numel(), ptr(g))
        self.keep[t] = (k, g)
        if sync:
            self.wait(t)
            return None
        return t

    def embedding_push_pull(self, pullkeys, dest, pushkeys, grads, sync=False):
        pk = self._k(pullkeys)
        uk = self._k(pushkeys)
        g = grads.reshape(-1, self.width).float().contiguous()
        t = lib('hc_async_push_pull')(self.handle, ptr(pk), pk.numel(), ptr(dest), ptr(uk), uk.numel(), ptr(g))
        self.keep[t] = (pk, dest, uk, g)
        if sync:
            self.wait(t)
            return None
        return t

    def wait(self, ticket):
        lib('hc_wait')(int(ticket))
        self.keep.pop(ticket, None)

    def flush(self):
        lib('hc_flush')(self.handle)

    def size(self):
        return lib('hc_size')(self.handle)

    def clear(self):
        """Drop every cached line without pushing it (the server's table was
        replaced, e.g. by a checkpoint load); later lookups re-pull."""
        lib('hc_clear')(self.handle)

    def bypass(self, on=True):
        lib('hc_set_bypass')(self.handle, int(on))

    @property
    def perf_enabled(self):
        return getattr(self, '_perf', False)

    @perf_enabled.setter
    def perf_enabled(self, v):
        self._perf = bool(v)
        lib('hc_set_perf')(self.handle, int(v))

    @property
    def perf(self):
        out = np.zeros(10, dtype=np.float64)
        lib('hc_get_perf')(self.handle, out.ctypes.data)
        keys = ['calls', 'unique', 'miss', 'transfer', 'evict', 'pushed', 't_unique', 't_sync', 't_copy', 't_push']
        return dict(zip(keys, out.tolist()))
