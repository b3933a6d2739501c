"""Checkpoint / resume.

Format-compatible with the reference (``executor.py:457-537``): a pickle of
``{param.name: np.float32 ndarray}`` written by rank 0; PS-held parameters are
written by the servers as raw float32 ``<dir>/<node_id>_<partition>.dat``.

Extension (opt-in, ``save_optimizer=True``): ``<file>.ext`` holds optimizer
states (flat m/v/velocity), step counters, BN running statistics and LR
scheduler state -- none of which the reference saves.
Loading never unpickles foreign files with code execution beyond plain numpy
arrays (``numpy`` arrays inside a dict; use trusted checkpoints only).
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch


def _params(ex):
    from ..ops.variable import PlaceholderOp
    return [n for n in ex.config.placeholder_to_arr_map if isinstance(n, PlaceholderOp) and n.trainable]


def state_dict(ex):
    out = {}
    for n in _params(ex):
        t = ex.config.placeholder_to_arr_map[n]
        out[n.name] = t.detach().float().cpu().numpy().astype(np.float32)
    return out


def save(ex, file_path, file_name='checkpoint.pkl', save_optimizer=False):
    cfg = ex.config
    if cfg.ps_comm is not None:
        cfg.ps_comm.save_params(file_path)
    if cfg.nrank > 1 and cfg.rank != 0 and cfg.comm_mode in ('AllReduce', 'Hybrid'):
        return None
    os.makedirs(file_path, exist_ok=True)
    st = state_dict(ex)
    path = os.path.join(file_path, file_name)
    with open(path, 'wb') as f:
        pickle.dump(st, f)
    if save_optimizer:
        ext = {'optimizers': [], 'bn': {}}
        for sub in ex.subexecutor.values():
            for op in getattr(sub, 'opt_ops', []):
                fl = op.flat
                d = {'step': op.step, 'name': op.name}
                if fl is not None:
                    d['order'] = [p.name for p in fl.params]
                    d['s1'] = fl.s1.cpu().numpy() if fl.s1 is not None else None
                    d['s2'] = fl.s2.cpu().numpy() if fl.s2 is not None else None
                lr = op.optimizer.learning_rate
                if hasattr(lr, 'state_dict'):
                    d['lr_sched'] = lr.state_dict()
                ext['optimizers'].append(d)
            for n in sub.topo_order:
                if getattr(n, 'running_mean', None) is not None:
                    ext['bn'][n.name] = (n.running_mean.cpu().numpy(), n.running_var.cpu().numpy())
        with open(path + '.ext', 'wb') as f:
            pickle.dump(ext, f)
    return path


def load_dict(ex, state, consider_splits=False):
    cfg = ex.config
    for n in _params(ex):
        if n.name not in state:
            continue
        v = np.asarray(state[n.name], dtype=np.float32)
        t = cfg.placeholder_to_arr_map[n]
        src = torch.from_numpy(v)
        if consider_splits and n.mp_split is not None:
            src = n.mp_split.slice_tensor(src)
        t.copy_(src.reshape(t.shape).to(t.device))
        cv = cfg.compute_values.get(n)
        if cv is not None:
            cv.copy_(t)


def load(ex, file_path, file_name='checkpoint.pkl', consider_splits=False):
    cfg = ex.config
    path = os.path.join(file_path, file_name)
    with open(path, 'rb') as f:
        st = pickle.load(f)
    load_dict(ex, st, consider_splits)
    if cfg.ps_comm is not None:
        cfg.ps_comm.load_params(file_path)
    ext_path = path + '.ext'
    if os.path.exists(ext_path):
        with open(ext_path, 'rb') as f:
            ext = pickle.load(f)
        ops = [op for sub in ex.subexecutor.values() for op in getattr(sub, 'opt_ops', [])]
        for op, d in zip(ops, ext.get('optimizers', [])):
            op.step = d['step']
            if op.flat is not None and d.get('s1') is not None and op.flat.s1 is not None:
                op.flat.s1.copy_(torch.from_numpy(d['s1']))
            if op.flat is not None and d.get('s2') is not None and op.flat.s2 is not None:
                op.flat.s2.copy_(torch.from_numpy(d['s2']))
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
# rename) names it, so a worker killed mid-write never leaves a torn
# checkpoint behind.  Rank 0 writes; every rank reads.

def save_resumable(ex, ckpt_dir, step, keep=2):
    """Commit a full snapshot (weights + optimizer state) taken after ``step``
    completed steps.  Returns the snapshot path on the writing rank."""
    cfg = ex.config
    sub = os.path.join(ckpt_dir, 'step_%d' % step)
    path = save(ex, sub, save_optimizer=True)
    if path is not None:
        tmp = os.path.join(ckpt_dir, '.latest.%d' % os.getpid())
        with open(tmp, 'w') as f:
            f.write('step_%d\n' % step)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, os.path.join(ckpt_dir, 'latest'))
        snaps = sorted((d for d in os.listdir(ckpt_dir) if d.startswith('step_')),
                       key=lambda d: int(d[5:]))
        for d in snaps[:-keep] if keep else []:
            if d != 'step_%d' % step:
                import shutil
                shutil.rmtree(os.path.join(ckpt_dir, d), ignore_errors=True)
    if cfg.nrank > 1 and cfg.comm_mode in ('AllReduce', 'Hybrid'):
        from ..parallel import comm
        comm.world().barrier()
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
