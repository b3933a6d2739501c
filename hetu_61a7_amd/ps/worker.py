"""PS worker agent (reference ps-lite worker + python_binding.cc:6-151, and
executor.py:60-131 role bootstrap).

Environment (ps-lite compatible): ``DMLC_ROLE``, ``DMLC_PS_ROOT_PORT`` (names
the shared-memory segment ``/hetu_ps_<port>``), ``DMLC_NUM_WORKER``,
``DMLC_NUM_SERVER``; fault knobs ``PS_DROP_MSG``, ``PS_RESEND``,
``PS_RESEND_TIMEOUT``, ``PS_HEARTBEAT_INTERVAL``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._lib import lib, ptr, check

PARAM_DENSE, PARAM_SPARSE, PARAM_CACHE = 0, 1, 2
INIT_TYPES = {'ConstantInit': 0, 'ZerosInit': 0, 'OnesInit': 0, 'UniformInit': 1,
              'GeneralXavierUniformInit': 1, 'XavierUniformInit': 1, 'HeUniformInit': 1,
              'LecunUniformInit': 1, 'NormalInit': 2, 'GeneralXavierNormalInit': 2,
              'XavierNormalInit': 2, 'HeNormalInit': 2, 'LecunNormalInit': 2,
              'TruncatedNormalInit': 3}
PSF_NAMES = ['DensePull', 'DensePush', 'DDPushPull', 'SparsePull', 'SparsePush', 'SDPushPull',
             'SSPushPull', 'PushEmbedding', 'SyncEmbedding', 'ParamInit', 'SaveParam', 'LoadParam',
             'SSPSync', 'PReduceGetPartner', 'Barrier', 'ParamClear']

_AGENT = None


def shm_name():
    return '/hetu_ps_%s' % os.environ.get('DMLC_PS_ROOT_PORT', '13100')


class PSAgent(object):
    """Worker-side PS API; method names follow the reference C ABI."""

    def __init__(self):
        nw = int(os.environ.get('DMLC_NUM_WORKER', '1'))
        ns = int(os.environ.get('DMLC_NUM_SERVER', '1'))
        check(lib('hps_init')(2, shm_name().encode(), nw, ns, 0), 'init')
        self.pending = {}
        self.keepalive = {}
        self.keys = []   # node ids this worker registered (save_params / load_params)

    # ---- identity --------------------------------------------------------------------
    def rank(self):
        return lib('hps_rank')()

    def nrank(self):
        return lib('hps_nrank')()

    # ---- parameters ------------------------------------------------------------------
    def InitTensor(self, node_id, ptype, length, width, init_type, init_a, init_b, seed, opt=None):
        rows = length // width if ptype == PARAM_DENSE and width > 1 else length
        if ptype == PARAM_DENSE:
            rows, width = length, 1
        check(lib('hps_param_init')(int(node_id), int(ptype), int(rows), int(width), int(init_type),
                                    float(init_a), float(init_b), int(seed)), 'ParamInit')
        self._register(node_id)

    def init_tensor(self, node_id, param_type, shape, initializer, seed, opt=None):
        name = type(initializer).__name__
        it = INIT_TYPES.get(name, 2)
        a, b = 0.0, 0.0
        if it == 0:
            a = getattr(initializer, 'constant', 0.0)
        elif it == 1:
            a, b = initializer.low, initializer.high
        else:
            a, b = initializer.mean, initializer.stddev
        if param_type == PARAM_DENSE:
            length, width = int(np.prod(shape)), 1
        else:
            length, width = int(shape[0]), int(np.prod(shape[1:]))
        check(lib('hps_param_init')(int(node_id), int(param_type), length, width, it, float(a),
                                    float(b), int(seed)), 'ParamInit')
        self._register(node_id)

    def _register(self, node_id):
        if int(node_id) not in self.keys:
            self.keys.append(int(node_id))

    def Clear(self, node_id):
        check(lib('hps_param_clear')(int(node_id)), 'Clear')

    ClearOnServer = Clear

    def SaveParam(self, node_id, path):
        os.makedirs(path, exist_ok=True)
        check(lib('hps_save_param')(int(node_id), path.encode()), 'SaveParam')

    def LoadParam(self, node_id, path):
        check(lib('hps_load_param')(int(node_id), path.encode()), 'LoadParam')

    # ---- PSFs (async; buffers must stay alive until Wait) -------------------------------
    def _issue(self, key, ticket, *ts):
        if ticket < 0:
            raise RuntimeError('PS request on key %d failed: %d' % (key, ticket))
        self.keepalive[ticket] = (key, ts)
        return ticket

    def Pull(self, node_id, arr):
        return self._issue(node_id, lib('hps_async_dense_pull')(int(node_id), ptr(arr), arr.numel()), arr)

    def Push(self, node_id, arr):
        return self._issue(node_id, lib('hps_async_dense_push')(int(node_id), ptr(arr), arr.numel()), arr)

    def DDPushPull(self, node_id, in_arr, out_arr):
        return self._issue(node_id, lib('hps_async_dd_pushpull')(int(node_id), ptr(in_arr), ptr(out_arr),
                                                                   in_arr.numel()), in_arr, out_arr)

    def SparsePull(self, node_id, index, value):
        return self._issue(node_id, lib('hps_async_sparse_pull')(int(node_id), ptr(index), index.numel(),
                                                                   ptr(value)), index, value)

    def SparsePush(self, node_id, index, value):
        return self._issue(node_id, lib('hps_async_sparse_push')(int(node_id), ptr(index), index.numel(),
                                                                   ptr(value)), index, value)

    def SDPushPull(self, node_id, index, in_arr, out_arr):
        return self._issue(node_id, lib('hps_async_sd_pushpull')(int(node_id), ptr(index), index.numel(),
                                                                   ptr(in_arr), ptr(out_arr), out_arr.numel()),
                           index, in_arr, out_arr)

    def SSPushPull(self, node_id, in_index, in_arr, out_index, out_arr):
        return self._issue(node_id, lib('hps_async_ss_pushpull')(int(node_id), ptr(in_index), in_index.numel(),
                                                                   ptr(in_arr), ptr(out_index), out_index.numel(),
                                                                   ptr(out_arr)),
                           in_index, in_arr, out_index, out_arr)

    def Wait(self, node_id):
        lib('hps_wait_key')(int(node_id))
        for t in [t for t, (k, _) in self.keepalive.items() if k == node_id]:
            del self.keepalive[t]

    def wait(self, node_id):
        self.Wait(node_id)

    def WaitTicket(self, ticket):
        r = lib('hps_wait')(int(ticket))
        self.keepalive.pop(ticket, None)
        return r

    # ---- sync versions (used by the HET cache glue and tests) ---------------------------
    def pull_sync(self, node_id, arr):
        check(lib('hps_dense_pull')(int(node_id), ptr(arr), arr.numel()), 'DensePull')

    def push_sync(self, node_id, arr):
        check(lib('hps_dense_push')(int(node_id), ptr(arr), arr.numel()), 'DensePush')

    # ---- coordination -----------------------------------------------------------------------
    def BarrierWorker(self):
        lib('hps_barrier_worker')()

    def ssp_init(self, key, group_size, tolerance):
        lib('hps_ssp_init')(int(key), int(group_size), int(tolerance))

    def ssp_sync(self, key, version):
        lib('hps_ssp_sync')(int(key), int(version))

    def preduce_get_partner(self, key, rank, required_worker_num, wait_time):
        out = np.full(257, -1, dtype=np.int32)
        lib('hps_preduce_get_partner')(int(key), int(rank), int(required_worker_num), float(wait_time),
                                       out.ctypes.data)
        return [int(x) for x in out[:np.argmax(out < 0)]]

    def heartbeat(self):
        lib('hps_heartbeat')()

    def fault_stats(self):
        """Reliable-delivery counters of this process (PS_DROP_MSG / PS_RESEND): dropped
        requests, dropped acks, resends, duplicates suppressed, plus the number of
        workers that took over a dead rank (node recovery)."""
        out = np.zeros(5, dtype=np.int64)
        lib('hps_fault_stats')(out.ctypes.data)
        keys = ('dropped_requests', 'dropped_acks', 'resends', 'duplicates_suppressed', 'recovered_workers')
        return dict(zip(keys, (int(x) for x in out)))

    def dead_nodes(self, timeout_s=None):
        timeout_s = timeout_s or float(os.environ.get('PS_HEARTBEAT_TIMEOUT', '60'))
        out = np.zeros(256, dtype=np.int32)
        n = lib('hps_dead_nodes')(float(timeout_s), out.ctypes.data, 256)
        return out[:n].tolist()

    # ---- load recording (reference executor.py:351-355, kvworker.h:39-51) --------------------
    def startRecord(self, dirpath):
        self.record_dir = dirpath
        os.makedirs(dirpath, exist_ok=True)
        lib('hps_start_record')(dirpath.encode())

    def getLoads(self):
        c = np.zeros(16, dtype=np.int64)
        b = np.zeros(16, dtype=np.int64)
        n = lib('hps_get_loads')(c.ctypes.data, b.ctypes.data, 16)
        return {PSF_NAMES[i]: (int(c[i]), int(b[i])) for i in range(n) if c[i]}

    def record_loads(self):
        loads = self.getLoads()
        d = getattr(self, 'record_dir', '.')
        with open(os.path.join(d, 'loads_%d.txt' % self.rank()), 'a') as f:
            f.write(repr(loads) + '\n')

    def save_params(self, path, keys=None):
        """SaveParam for every table this worker registered (or ``keys``): one
        ``<key>_<part>.dat`` per server partition under ``path``."""
        keys = self.keys if keys is None else keys
        if not keys:
            raise ValueError('save_params: no PS tables registered on this worker')
        for k in keys:
            self.SaveParam(k, path)
        return list(keys)

    def load_params(self, path, keys=None):
        """LoadParam counterpart of :meth:`save_params`."""
        keys = self.keys if keys is None else keys
        if not keys:
            raise ValueError('load_params: no PS tables registered on this worker')
        for k in keys:
            self.LoadParam(k, path)
        return list(keys)

    def finalize(self):
        lib('hps_finalize')()


def worker_init():
    global _AGENT
    if _AGENT is None:
        _AGENT = PSAgent()
    return _AGENT


def get_agent():
    return worker_init()


def worker_finish():
    global _AGENT
    if _AGENT is not None:
        from .table import close_all
        close_all()
        _AGENT.finalize()
        _AGENT = None


def get_worker(config):
    return worker_init()
