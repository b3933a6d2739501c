"""Masked-LM row compaction (``mlm_gather.hip``): the labelled rows of a BERT batch into
C slots per sequence, their gather and its adjoint.  CPU: the same semantics in torch."""
from __future__ import annotations

import torch

from .. import native_array as _NA
from . import fn, native, stream_ptr, check, record_native, P, I32, I64


def masked_positions(labels, C, overflow):
    """labels [B, S] int64 (-1 = no label) -> idx [B*C] int64: slot k of sequence b holds
    the k-th labelled row b*S + s in position order, or -1.  A sequence with more than C
    labels sets overflow[0] (device int32) to its count."""
    B, S = labels.shape
    kind = {torch.int64: 0, torch.int32: 1, torch.float32: 2}.get(labels.dtype)
    if labels.is_cuda and native(labels) and kind is not None:
        lab = labels
        if not lab.is_contiguous():
            from .tensor import copy_into
            lab = copy_into(_NA.empty((B, S), dtype=lab.dtype, device=lab.device), lab)
        idx = _NA.empty((B * C,), dtype=torch.int64, device=labels.device)
        f = fn('hetu_masked_positions', [P, I32, I32, I32, I32, P, P, P])
        check(f(lab.data_ptr(), kind, B, S, C, idx.data_ptr(), overflow.data_ptr(), stream_ptr()), 'masked_positions')
        record_native('masked_positions')
        return idx
    lab = labels.reshape(B, S)
    idx = torch.full((B, C), -1, dtype=torch.int64)
    for b in range(B):
        pos = torch.nonzero(lab[b] != -1).reshape(-1)
        if pos.numel() > C:
            overflow[0] = max(int(overflow[0]), int(pos.numel()))
        pos = pos[:C]
        idx[b, :pos.numel()] = pos + b * S
    return idx.reshape(-1)


def take_rows(x, idx, fill_neg1=False):
    """out[j] = x[idx[j]] (rows of a [R, H] or [R] tensor), fill (0, or -1 for int64
    labels) where idx[j] < 0"""
    x2 = x.reshape(x.shape[0], -1)
    H = x2.shape[1]
    n = idx.numel()
    if x.is_cuda and native(x):
        x2 = x2.contiguous()
        out = _NA.empty((n, H), dtype=x.dtype, device=x.device)
        mode = 0 if not fill_neg1 else (2 if x.is_floating_point() else 1)
        f = fn('hetu_take_rows', [P, P, I64, I32, I32, I32, P, P])
        check(f(x2.data_ptr(), idx.data_ptr(), n, H, x2.element_size(), mode, out.data_ptr(), stream_ptr()),
              'take_rows')
        record_native('take_rows')
    else:
        safe = idx.clamp_min(0)
        out = x2[safe].clone()
        out[idx < 0] = -1 if fill_neg1 else 0
    return out.reshape((n,) + tuple(x.shape[1:]))


def put_rows(g, idx, rows):
    """the adjoint of take_rows: out [rows, H] zero except out[idx[j]] = g[j] (idx unique)"""
    g2 = g.reshape(g.shape[0], -1)
    H = g2.shape[1]
    if g.is_cuda and native(g):
        from .tensor import zeros
        g2 = g2.contiguous()
        out = zeros((rows, H), g.dtype, g.device)
        f = fn('hetu_put_rows', [P, P, I64, I32, I32, P, P])
        check(f(g2.data_ptr(), idx.data_ptr(), idx.numel(), H, g2.element_size(), out.data_ptr(), stream_ptr()),
              'put_rows')
        record_native('put_rows')
    else:
        out = torch.zeros((rows, H), dtype=g.dtype)
        keep = idx >= 0
        out[idx[keep]] = g2[keep]
    return out.reshape((rows,) + tuple(g.shape[1:]))
