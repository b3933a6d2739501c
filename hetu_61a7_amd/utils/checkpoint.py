"""Checkpoint / resume.

Format-compatible with the reference (``executor.py:457-537``): a pickle of
``{param.name: np.float32 ndarray}`` written by rank 0 for every parameter the
worker holds; PS-held parameters (embedding tables in PS/Hybrid mode, the flat
dense buffer in pure PS mode) are written by the server as raw float32
``<dir>/<node_id>_<partition>.dat`` (reference ``PSAgent.h:447-476``,
``PSFHandle.h:389-427``): workers drain their pending pushes, meet at a
worker barrier, worker 0 issues SaveParam/LoadParam per PS key, and a second
barrier releases everyone.  After a load every HET cache is invalidated and
PS-held dense parameters are re-pulled.

Extension (opt-in, ``save_optimizer=True``): ``<file>.ext`` holds optimizer
states (flat m/v/velocity, per-table sparse states), step counters, BN running
statistics and LR-scheduler state -- none of which the reference saves
(SURVEY §5.4).  With ZeRO-1 each rank owns a 1/P shard of the flat optimizer
state; it is written by that rank to ``<file>.ext.rank<r>`` and read back by
the same rank.

Loading uses a restricted unpickler that only reconstructs numpy arrays and
builtin containers/scalars, so a foreign checkpoint cannot run code.
Every file is fsynced before it becomes reachable, and resumable snapshots
are published by an atomic rename of ``<dir>/latest`` followed by a
directory fsync.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np
import torch


# ---------------------------------------------------------------------------
# safe (de)serialisation

_SAFE_GLOBALS = {
    ('builtins', n) for n in ('dict', 'list', 'tuple', 'set', 'frozenset', 'int', 'float', 'bool',
                              'str', 'bytes', 'bytearray', 'complex', 'slice', 'range')
} | {
    ('collections', 'OrderedDict'),
    ('_codecs', 'encode'),             # protocol-2 pickles spell bytes this way
    ('numpy', 'ndarray'), ('numpy', 'dtype'),
    ('numpy.core.multiarray', '_reconstruct'), ('numpy.core.multiarray', 'scalar'),
    ('numpy._core.multiarray', '_reconstruct'), ('numpy._core.multiarray', 'scalar'),
    ('numpy.core.numeric', '_frombuffer'), ('numpy._core.numeric', '_frombuffer'),   # protocol 5
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _SAFE_GLOBALS:
            return super().find_class(module, name)
        if module == 'numpy' and name.endswith('DType'):
            return super().find_class(module, name)
        if module in ('numpy.dtypes',) and name.endswith('DType'):
            return super().find_class(module, name)
        raise pickle.UnpicklingError('checkpoint refers to %s.%s, which a checkpoint may not '
                                     'contain (only numpy arrays and builtin values)' % (module, name))


def safe_load(f):
    """Unpickle ``f`` allowing only numpy arrays and builtin values."""
    return _SafeUnpickler(f).load()


def _fsync_dir(path):
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def _write_durable(path, obj):
    """Pickle ``obj`` to ``path`` via a temporary file: written, fsynced, renamed."""
    tmp = '%s.tmp.%d' % (path, os.getpid())
    with open(tmp, 'wb') as f:
        pickle.dump(obj, f, protocol=4)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _read(path):
    with open(path, 'rb') as f:
        return safe_load(io.BufferedReader(f))


# ---------------------------------------------------------------------------
# parameter views

def _params(ex):
    from ..ops.variable import PlaceholderOp
    return [n for n in ex.config.placeholder_to_arr_map if isinstance(n, PlaceholderOp) and n.trainable]


def _ps_tables(ex):
    from ..ps.table import PSTable
    return [(n, t) for n, t in ex.config.placeholder_to_arr_map.items() if isinstance(t, PSTable)]


def _opt_ops(ex):
    return [op for sub in ex.subexecutor.values() for op in getattr(sub, 'opt_ops', [])]


def _ps_dense(ex):
    return [op.ps_dense for op in _opt_ops(ex) if getattr(op, 'ps_dense', None) is not None]


def state_dict(ex):
    """``{name: float32 ndarray}`` of every worker-held trainable parameter (PS
    tables are saved by the server, not here)."""
    out = {}
    for n in _params(ex):
        t = ex.config.placeholder_to_arr_map[n]
        if not isinstance(t, torch.Tensor):
            continue
        out[n.name] = t.detach().float().cpu().numpy().astype(np.float32)
    return out


def _zero_rank(ex):
    for op in _opt_ops(ex):
        if getattr(op, 'zero', False) and op.comm is not None:
            return op.comm.rank
    return None


# ---------------------------------------------------------------------------
# save

def _ps_save(ex, file_path):
    """Reference executor.py:465-481: drain, barrier, worker 0 -> SaveParam per
    PS key, barrier."""
    agent = ex.config.ps_comm
    tables = _ps_tables(ex)
    for _, t in tables:
        t.close()                      # flush staged grads, wait pushes, flush cache lines
    for d in _ps_dense(ex):
        d.drain()                      # the overlapped dense exchange in flight (ASP prefetch)
    agent.BarrierWorker()
    if agent.rank() == 0:
        os.makedirs(file_path, exist_ok=True)
        for _, t in tables:
            agent.SaveParam(t.key, file_path)
        for d in _ps_dense(ex):
            agent.SaveParam(d.key, file_path)
        for name in os.listdir(file_path):
            if name.endswith('.dat'):
                with open(os.path.join(file_path, name), 'rb') as f:
                    os.fsync(f.fileno())
        _fsync_dir(file_path)
    agent.BarrierWorker()


def _ext_state(ex, zero_rank):
    ext = {'optimizers': [], 'bn': {}}
    for op in _opt_ops(ex):
        fl = op.flat
        d = {'step': op.step, 'name': op.name, 'zero': bool(getattr(op, 'zero', False))}
        if fl is not None:
            d['order'] = [p.name for p in fl.params]
            # where each parameter's moments sit in the flat buffers: the segment alignment
            # (optimizer.SEG_ALIGN) and the parameter set may differ at load time
            d['layout'] = [(p.name, int(fl.offsets[p][0]), int(fl.offsets[p][1])) for p in fl.params]
            if not d['zero']:   # ZeRO shards go to the per-rank file
                d['s1'] = fl.s1.cpu().numpy() if fl.s1 is not None else None
                d['s2'] = fl.s2.cpu().numpy() if fl.s2 is not None else None
        d['sparse'] = {p.name: {k: v.detach().float().cpu().numpy() for k, v in st.items()}
                       for p, st in op.sparse_state.items()}
        lr = op.optimizer.learning_rate
        if hasattr(lr, 'state_dict'):
            d['lr_sched'] = lr.state_dict()
        ext['optimizers'].append(d)
    for sub in ex.subexecutor.values():
        for n in sub.topo_order:
            if getattr(n, 'running_mean', None) is not None:
                ext['bn'][n.name] = (n.running_mean.cpu().numpy(), n.running_var.cpu().numpy())
    return ext


def _zero_shards(ex):
    out = []
    for op in _opt_ops(ex):
        fl = op.flat
        if not getattr(op, 'zero', False) or fl is None:
            out.append(None)
            continue
        out.append({'s1': fl.s1.cpu().numpy() if fl.s1 is not None else None,
                    's2': fl.s2.cpu().numpy() if fl.s2 is not None else None,
                    'nrank': op.comm.nrank, 'rank': op.comm.rank})
    return out


def save(ex, file_path, file_name='checkpoint.pkl', save_optimizer=False):
    """Write the checkpoint; every rank must call it (PS barriers, ZeRO shards).
    Returns the pickle path on the rank that wrote it, else None."""
    cfg = ex.config
    if cfg.ps_comm is not None:
        _ps_save(ex, file_path)
    path = os.path.join(file_path, file_name)
    zr = _zero_rank(ex) if save_optimizer else None
    if zr is not None:
        os.makedirs(file_path, exist_ok=True)
        _write_durable('%s.ext.rank%d' % (path, zr), _zero_shards(ex))
    writer = not (cfg.nrank > 1 and cfg.rank != 0 and cfg.comm_mode in ('AllReduce', 'Hybrid'))
    if cfg.ps_comm is not None and cfg.comm_mode == 'PS':
        writer = cfg.ps_comm.rank() == 0
    if not writer:
        return None
    os.makedirs(file_path, exist_ok=True)
    _write_durable(path, state_dict(ex))
    if save_optimizer:
        _write_durable(path + '.ext', _ext_state(ex, zr))
    _fsync_dir(file_path)
    return path


# ---------------------------------------------------------------------------
# load

def load_dict(ex, state, consider_splits=False):
    cfg = ex.config
    for n in _params(ex):
        if n.name not in state:
            continue
        t = cfg.placeholder_to_arr_map[n]
        if not isinstance(t, torch.Tensor):
            continue
        v = np.asarray(state[n.name], dtype=np.float32)
        src = torch.from_numpy(v)
        if consider_splits and n.mp_split is not None:
            src = n.mp_split.slice_tensor(src)
        t.copy_(src.reshape(t.shape).to(t.device))
        cv = cfg.compute_values.get(n)
        if cv is not None:
            cv.copy_(t)
    for op in _opt_ops(ex):   # refresh the bf16 shadow of the flat master
        if op.flat is not None and op.flat.shadow is not None:
            op.flat.shadow.copy_(op.flat.param)


def _ps_load(ex, file_path):
    agent = ex.config.ps_comm
    tables = _ps_tables(ex)
    for _, t in tables:
        t.close()
    for d in _ps_dense(ex):
        d.drain()
    agent.BarrierWorker()
    if agent.rank() == 0:
        for _, t in tables:
            agent.LoadParam(t.key, file_path)
        for d in _ps_dense(ex):
            agent.LoadParam(d.key, file_path)
    agent.BarrierWorker()
    for _, t in tables:
        t.invalidate()
    for d in _ps_dense(ex):
        d.repull()


def _full_moments(d, fl, op=None):
    """the (non-ZeRO) optimizer record ``d`` holds whole flat s1 / s2 buffers: every
    bucket's owned range of this rank lies inside them"""
    if fl is None or op is None or not getattr(op, 'buckets', None) or d.get('zero'):
        return False
    arrs = [d.get(k) for k in ('s1', 's2') if getattr(fl, k) is not None]
    return bool(arrs) and all(a is not None and getattr(a, 'size', 0) >= fl.numel for a in arrs)


def _owned_moments(op, d):
    """this rank's ZeRO-1 shard (bucket by bucket, the owned 1/P of each) of full moments"""
    import numpy as np
    out = {}
    for k in ('s1', 's2'):
        full = d.get(k)
        if full is None:
            continue
        full = np.asarray(full).reshape(-1)
        end = max(b.own[1] for b in op.buckets)
        if full.size < end:      # the ZeRO flat pads to 64 x ranks; the padding has zero state
            full = np.concatenate([full, np.zeros(end - full.size, full.dtype)])
        pieces = [full[b.own[0]:b.own[1]] for b in op.buckets]
        out[k] = np.concatenate(pieces) if pieces else full[:0]
    out['nrank'] = op.comm.nrank
    return out


def _load_flat_moments(fl, d, i):
    """copy whole-buffer moments (s1 / s2) of optimizer record ``d`` into ``fl``
    parameter by parameter, through the saved layout (name, offset, numel).  A record
    without a layout (written before layouts were saved) is taken only when its order
    and buffer size match this flat buffer exactly; anything else is refused rather
    than loaded under the wrong offsets."""
    import numpy as np
    layout = d.get('layout')
    for k in ('s1', 's2'):
        buf = getattr(fl, k)
        arr = d.get(k)
        if arr is None or buf is None:
            continue
        arr = np.asarray(arr).reshape(-1)
        if layout is None:
            order = d.get('order')
            if order != [p.name for p in fl.params] or arr.size != buf.numel():
                raise ValueError('optimizer %d: checkpoint moments have no layout and do not match this '
                                 'flat buffer (%d saved elements, %d here, parameter order %s); '
                                 're-save the checkpoint with this version' %
                                 (i, arr.size, buf.numel(), 'matches' if order == [p.name for p in fl.params]
                                  else 'differs'))
            buf.copy_(torch.from_numpy(arr).to(buf.device))
            continue
        saved = {name: (o, n) for name, o, n in layout}
        host = buf.detach().cpu().numpy().copy()
        for p in fl.params:
            o, n, _ = fl.offsets[p]
            if p.name not in saved:
                continue
            so, sn = saved[p.name]
            if sn != n:
                raise ValueError('optimizer %d: parameter %s has %d elements, the checkpoint %d'
                                 % (i, p.name, n, sn))
            host[o:o + n] = arr[so:so + sn]
        buf.copy_(torch.from_numpy(host).to(buf.device))


def load(ex, file_path, file_name='checkpoint.pkl', consider_splits=False):
    cfg = ex.config
    path = os.path.join(file_path, file_name)
    load_dict(ex, _read(path), consider_splits)
    if cfg.ps_comm is not None:
        _ps_load(ex, file_path)
    ext_path = path + '.ext'
    if not os.path.exists(ext_path):
        return
    ext = _read(ext_path)
    ops = _opt_ops(ex)
    zr = _zero_rank(ex)
    shards = None
    if zr is not None and os.path.exists('%s.ext.rank%d' % (path, zr)):
        shards = _read('%s.ext.rank%d' % (path, zr))
    for i, (op, d) in enumerate(zip(ops, ext.get('optimizers', []))):
        op.step = d['step']
        fl = op.flat
        src = d
        if getattr(op, 'zero', False):
            if shards is None or i >= len(shards) or shards[i] is None:
                if _full_moments(d, fl, op):
                    # a checkpoint written without ZeRO carries the full moments: take this
                    # rank's owned range of every bucket
                    src = _owned_moments(op, d)
                else:
                    # a ZeRO-1 resume without this rank's moments would keep the restored
                    # step count with zeroed state (Adam bias correction off): refuse
                    raise FileNotFoundError('ZeRO-1 optimizer shard %s.ext.rank%s (optimizer %d) missing'
                                            % (path, zr, i))
            else:
                src = shards[i]
            if src.get('nrank', op.comm.nrank) != op.comm.nrank:
                raise ValueError('ZeRO checkpoint was written with %s ranks, resuming with %d'
                                 % (src.get('nrank'), op.comm.nrank))
        if fl is not None:
            if src is d:
                _load_flat_moments(fl, d, i)
            else:
                for k in ('s1', 's2'):
                    buf = getattr(fl, k)
                    if src.get(k) is not None and buf is not None:
                        buf.copy_(torch.from_numpy(src[k]).to(buf.device))
        by_name = {p.name: st for p, st in op.sparse_state.items()}
        for name, st in d.get('sparse', {}).items():
            if name in by_name:
                for k, v in st.items():
                    if k in by_name[name]:
                        by_name[name][k].copy_(torch.from_numpy(v).to(by_name[name][k].device))
        lr = op.optimizer.learning_rate
        if 'lr_sched' in d and hasattr(lr, 'load_state_dict'):
            lr.load_state_dict(d['lr_sched'])
    for sub in ex.subexecutor.values():
        for n in sub.topo_order:
            if n.name in ext.get('bn', {}):
                m, v = ext['bn'][n.name]
                dev = cfg.device
                n.running_mean = torch.from_numpy(m).to(dev)
                n.running_var = torch.from_numpy(v).to(dev)


# ---------------------------------------------------------------------------
# Resumable snapshots for elastic restarts (heturun --max-restarts).
# A snapshot is a directory ``<dir>/step_<N>/`` holding the reference-format
# pickle plus the ``.ext`` optimizer/BN/scheduler state; it becomes visible
# only when ``<dir>/latest`` (a one-line text file, replaced by an atomic
# rename) names it.  Every snapshot file and the snapshot directory are
# fsynced before ``latest`` moves, and ``<dir>`` is fsynced after, so a crash
# never leaves ``latest`` naming a torn snapshot.  Every rank calls it.

def _barrier(ex):
    cfg = ex.config
    if cfg.nrank > 1 and cfg.comm_mode in ('AllReduce', 'Hybrid'):
        from ..parallel import comm
        comm.world().barrier()
    elif cfg.ps_comm is not None:
        cfg.ps_comm.BarrierWorker()


def save_resumable(ex, ckpt_dir, step, keep=2):
    """Commit a full snapshot (weights + optimizer state) taken after ``step``
    completed steps.  Returns the snapshot path on the writing rank."""
    sub = os.path.join(ckpt_dir, 'step_%d' % step)
    path = save(ex, sub, save_optimizer=True)
    _barrier(ex)                      # every rank's ZeRO shard is durable
    if path is not None:
        _fsync_dir(sub)
        tmp = os.path.join(ckpt_dir, '.latest.%d' % os.getpid())
        with open(tmp, 'w') as f:
            f.write('step_%d\n' % step)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, os.path.join(ckpt_dir, 'latest'))
        _fsync_dir(ckpt_dir)
        snaps = sorted((d for d in os.listdir(ckpt_dir) if d.startswith('step_')),
                       key=lambda d: int(d[5:]))
        for d in snaps[:-keep] if keep else []:
            if d != 'step_%d' % step:
                import shutil
                shutil.rmtree(os.path.join(ckpt_dir, d), ignore_errors=True)
    _barrier(ex)
    return path


def latest_step(ckpt_dir):
    """Step count of the last committed snapshot, or 0 if there is none."""
    try:
        with open(os.path.join(ckpt_dir, 'latest')) as f:
            name = f.read().strip()
    except FileNotFoundError:
        return 0
    return int(name[5:]) if name.startswith('step_') else 0


def resume(ex, ckpt_dir):
    """Load the last committed snapshot into ``ex``; returns the number of
    completed steps it holds (0: nothing to resume, ``ex`` untouched)."""
    step = latest_step(ckpt_dir)
    if step:
        load(ex, os.path.join(ckpt_dir, 'step_%d' % step))
    return step
