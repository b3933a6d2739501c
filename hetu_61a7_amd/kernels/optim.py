"""Flat multi-tensor optimizer kernels (``optimizer.hip``) and sparse row updates."""
from __future__ import annotations

import torch

from . import fn, native, stream_ptr, check, P, I64, I32, F32

MODES = dict(sgd=0, momentum=1, nesterov=2, adagrad=3, adam=4, adamw=5, lamb=6)


def optimizer_flat(mode, p, g, s1=None, s2=None, shadow=None, lr=0.01, l2=0.0, mu=0.9,
                   beta1=0.9, beta2=0.999, beta1t=1.0, beta2t=1.0, eps=1e-7, wd=0.0,
                   gscale=1.0, seg_off=None, seg_off_host=None, norms_ws=None, dyn=None):
    """Update flat fp32 ``p`` in place from flat fp32 ``g``.

    ``seg_off`` (device int64, LAMB only) holds per-tensor offsets.  ``shadow``
    (bf16, same numel) receives the updated weights for mixed precision.
    """
    m = MODES[mode]
    from . import deterministic
    # deterministic LAMB: the per-tensor norms as ordered torch reductions below
    # instead of the fused kernel's cross-block atomics
    if native(p) and not (mode == 'lamb' and deterministic()):
        f = fn('hetu_optimizer_flat', [I32, P, P, P, P, P, I64, F32, F32, F32, F32, F32, F32, F32,
                                       F32, F32, F32, P, I32, P, P, P])
        nseg = (seg_off.numel() - 1) if seg_off is not None else 0
        check(f(m, p.data_ptr(), g.data_ptr(), s1.data_ptr() if s1 is not None else None,
                s2.data_ptr() if s2 is not None else None,
                shadow.data_ptr() if shadow is not None else None, p.numel(), lr, l2, mu, beta1,
                beta2, beta1t, beta2t, eps, wd, gscale,
                seg_off.data_ptr() if seg_off is not None else None, nseg,
                norms_ws.data_ptr() if norms_ws is not None else None,
                dyn.data_ptr() if dyn is not None else None, stream_ptr()), 'optimizer')
        return
    if dyn is not None:
        lr, beta1t, beta2t, gscale = [float(v) for v in dyn.tolist()]
    from . import cpu_native
    if mode != 'lamb' and cpu_native.active(p, g) and p.is_contiguous() and g.is_contiguous():
        cpu_native.optimizer(mode, p, g, s1, s2, lr, l2, mu, beta1, beta2, beta1t, beta2t, eps, wd, gscale)
        if shadow is not None:
            shadow.copy_(p)
        return
    gr = g * gscale + l2 * p if (gscale != 1.0 or l2) else g
    if mode == 'sgd':
        p.sub_(lr * gr)
    elif mode == 'momentum':
        s1.mul_(mu).sub_(lr * gr)
        p.add_(s1)
    elif mode == 'nesterov':
        t = lr * gr
        s1.sub_(t).mul_(mu)
        p.add_(s1 - t)
    elif mode == 'adagrad':
        s1.add_(gr * gr)
        p.sub_(lr * gr / (torch.sqrt(s1) + eps))
    else:
        s1.mul_(beta1).add_((1 - beta1) * gr)
        s2.mul_(beta2).add_((1 - beta2) * gr * gr)
        u = (s1 / (1 - beta1t)) / (torch.sqrt(s2 / (1 - beta2t)) + eps)
        if mode == 'adam':
            p.sub_(lr * u)
        elif mode == 'adamw':
            p.sub_(lr * (u + wd * p))
        else:  # lamb, per segment
            offs = seg_off_host
            for i in range(len(offs) - 1):
                a, b = offs[i], offs[i + 1]
                pn = torch.linalg.vector_norm(p[a:b])
                un = torch.linalg.vector_norm(u[a:b])
                ratio = (pn / un) if (pn > 0 and un > 0) else torch.tensor(1.0)
                p[a:b].sub_(lr * ratio * (u[a:b] + wd * p[a:b]))
    if shadow is not None:
        shadow.copy_(p)


SPARSE_MODES = dict(sgd=0, momentum=1, nesterov=2, adagrad=3, adam=4, adamw=5)


def sparse_update(mode, table, ids, grads, s1=None, s2=None, lr=0.01, l2=0.0, mu=0.9,
                  beta1=0.9, beta2=0.999, beta1t=1.0, beta2t=1.0, eps=1e-7, wd=0.0):
    """Row-sparse update of ``table`` (fp32 [rows, dim]) at UNIQUE ``ids``."""
    dim = table.shape[-1]
    g = grads.reshape(-1, dim).float().contiguous()
    ids = ids.reshape(-1).long().contiguous()
    if native(table):
        f = fn('hetu_sparse_opt', [I32, P, P, P, P, P, I64, I64, I64, F32, F32, F32, F32, F32,
                                   F32, F32, F32, F32, P])
        check(f(SPARSE_MODES[mode], table.data_ptr(), s1.data_ptr() if s1 is not None else None,
                s2.data_ptr() if s2 is not None else None, ids.data_ptr(), g.data_ptr(),
                ids.numel(), dim, table.shape[0], lr, l2, mu, beta1, beta2, beta1t, beta2t, eps,
                wd, stream_ptr()), 'sparse_opt')
        return
    # ids < 0 mark rows the dense de-duplication left untouched (optimizer.py);
    # the native kernel skips them, the torch path must too (table[-1] is a real row)
    keep = ids >= 0
    if not bool(keep.all()):
        ids, g = ids[keep], g[keep]
    p = table[ids]
    gr = g + l2 * p if l2 else g
    if mode == 'sgd':
        p = p - lr * gr
    elif mode == 'momentum':
        v = mu * s1[ids] - lr * gr
        s1[ids] = v
        p = p + v
    elif mode == 'nesterov':
        t = lr * gr
        v = mu * (s1[ids] - t)
        s1[ids] = v
        p = p + v - t
    elif mode == 'adagrad':
        a = s1[ids] + gr * gr
        s1[ids] = a
        p = p - lr * gr / (torch.sqrt(a) + eps)
    else:
        m = beta1 * s1[ids] + (1 - beta1) * gr
        v = beta2 * s2[ids] + (1 - beta2) * gr * gr
        s1[ids] = m
        s2[ids] = v
        u = (m / (1 - beta1t)) / (torch.sqrt(v / (1 - beta2t)) + eps)
        p = p - lr * u if mode == 'adam' else p - lr * (u + wd * p)
    table[ids] = p
