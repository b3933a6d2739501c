"""ctypes bindings of ``libhetu_runtime.so``: shared-memory PS (``hps_*``) and
HET cache (``hc_*``) C ABIs (csrc/ps/shm_ps.h, csrc/cache/het_cache.cc)."""
from __future__ import annotations

import ctypes

from .._base import runtime_lib

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
U64 = ctypes.c_uint64
F32 = ctypes.c_float
F64 = ctypes.c_double
S = ctypes.c_char_p

_SIGS = {
    'hps_init': ([I32, S, I32, I32, U64], I32),
    'hps_finalize': ([], I32),
    'hps_rank': ([], I32),
    'hps_nrank': ([], I32),
    'hps_server_wait_shutdown': ([F64], I32),
    'hps_param_init': ([I32, I32, I64, I64, I32, F64, F64, U64], I32),
    'hps_param_clear': ([I32], I32),
    'hps_param_rows': ([I32], I64),
    'hps_param_width': ([I32], I64),
    'hps_dense_pull': ([I32, P, I64], I32),
    'hps_dense_push': ([I32, P, I64], I32),
    'hps_dd_pushpull': ([I32, P, P, I64], I32),
    'hps_sparse_pull': ([I32, P, I64, P], I32),
    'hps_sparse_push': ([I32, P, I64, P], I32),
    'hps_sd_pushpull': ([I32, P, I64, P, P, I64], I32),
    'hps_ss_pushpull': ([I32, P, I64, P, P, I64, P], I32),
    'hps_push_embedding': ([I32, P, I64, P, P], I32),
    'hps_sync_embedding': ([I32, P, I64, P, I64, P, P, P], I64),
    'hps_async_dense_pull': ([I32, P, I64], I64),
    'hps_async_dense_push': ([I32, P, I64], I64),
    'hps_async_dd_pushpull': ([I32, P, P, I64], I64),
    'hps_async_sparse_pull': ([I32, P, I64, P], I64),
    'hps_async_sparse_push': ([I32, P, I64, P], I64),
    'hps_async_sd_pushpull': ([I32, P, I64, P, P, I64], I64),
    'hps_async_ss_pushpull': ([I32, P, I64, P, P, I64, P], I64),
    'hps_wait': ([I64], I32),
    'hps_wait_key': ([I32], I32),
    'hps_barrier_worker': ([], I32),
    'hps_ssp_init': ([I32, I32, I64], I32),
    'hps_ssp_sync': ([I32, I64], I32),
    'hps_preduce_get_partner': ([I32, I32, I32, F32, P], I32),
    'hps_heartbeat': ([], I32),
    'hps_dead_nodes': ([F64, P, I32], I32),
    'hps_fault_stats': ([P], I32),
    'hps_save_param': ([I32, S], I32),
    'hps_load_param': ([I32, S], I32),
    'hps_start_record': ([S], I32),
    'hps_get_loads': ([P, P, I32], I32),
    'hc_create': ([I32, I64, I64, I64, I32, I64, I64], I32),
    'hc_lookup': ([I32, P, I64, P], I32),
    'hc_update': ([I32, P, I64, P], I32),
    'hc_async_lookup': ([I32, P, I64, P], I64),
    'hc_async_update': ([I32, P, I64, P], I64),
    'hc_async_push_pull': ([I32, P, I64, P, P, I64, P], I64),
    'hc_wait': ([I64], I32),
    'hc_flush': ([I32], I32),
    'hc_clear': ([I32], I32),
    'hc_size': ([I32], I64),
    'hc_set_bounds': ([I32, I64, I64], I32),
    'hc_set_bypass': ([I32, I32], I32),
    'hc_set_perf': ([I32, I32], I32),
    'hc_get_perf': ([I32, P], I32),
}

_fns = {}


def lib(name):
    f = _fns.get(name)
    if f is None:
        f = getattr(runtime_lib(), name)
        f.argtypes, f.restype = _SIGS[name]
        _fns[name] = f
    return f


def ptr(t):
    """Host pointer of a CPU tensor / numpy array."""
    if t is None:
        return None
    if hasattr(t, 'data_ptr'):
        assert not t.is_cuda, 'PS buffers live in host memory'
        assert t.is_contiguous()
        return t.data_ptr()
    return t.ctypes.data


def check(ret, what):
    if ret < 0:
        raise RuntimeError('PS call %s failed: %d' % (what, ret))
    return ret
