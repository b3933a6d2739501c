"""MoE routing kernels: top-k gating, dispatch (layout transform) and combine
(reverse layout transform) -- ``moe.hip``.

Reference LayoutTransform.cu scatters token i into slot
``expert(i) * capacity + location(i)`` (dropped when location >= capacity) and
combines with gate weights through atomicAdd; its gate-gradient uses a
hard-coded 32-lane shuffle.  Here dispatch and combine are gathers keyed by a
per-slot source index (deterministic, no atomics) with wave64 dot products.
"""
from __future__ import annotations

import torch

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32


def topk(x, k):
    v, i = torch.topk(x, k, dim=-1)
    return v, i


def layout_transform(x, indices, locations, capacity, num_experts):
    """x [T, d]; indices/locations [T, k] -> out [E*capacity, d] (zero padded)."""
    T, d = x.shape
    k = indices.shape[1] if indices.dim() == 2 else 1
    idx = indices.reshape(T, k).long()
    loc = locations.reshape(T, k).long()
    out = torch.zeros((num_experts * capacity, d), dtype=x.dtype, device=x.device)
    valid = loc < capacity
    slots = idx * capacity + loc
    tok = torch.arange(T, device=x.device).unsqueeze(1).expand(T, k)
    s, t = slots[valid], tok[valid]
    out[s] = x[t]
    return out


def layout_transform_backward(g, indices, locations, capacity):
    """grad wrt x: sum over the k slots each token was written to."""
    T = indices.shape[0]
    k = indices.shape[1] if indices.dim() == 2 else 1
    idx = indices.reshape(T, k).long()
    loc = locations.reshape(T, k).long()
    valid = (loc < capacity)
    slots = torch.where(valid, idx * capacity + loc, torch.zeros_like(idx))
    gathered = g[slots.reshape(-1)].reshape(T, k, -1) * valid.unsqueeze(-1).to(g.dtype)
    return gathered.sum(1)


def reverse_layout_transform(y, indices, locations, gates, capacity):
    """combine: out[t] = sum_j gates[t, j] * y[slot(t, j)] (dropped slots -> 0)."""
    T = indices.shape[0]
    k = indices.shape[1] if indices.dim() == 2 else 1
    idx = indices.reshape(T, k).long()
    loc = locations.reshape(T, k).long()
    valid = loc < capacity
    slots = torch.where(valid, idx * capacity + loc, torch.zeros_like(idx))
    rows = y[slots.reshape(-1)].reshape(T, k, -1).float()
    w = (gates.reshape(T, k).float() * valid.float()) if gates is not None else valid.float()
    return (rows * w.unsqueeze(-1)).sum(1).to(y.dtype)


def reverse_layout_transform_backward_data(g, indices, locations, gates, capacity, num_slots):
    T = indices.shape[0]
    k = indices.shape[1] if indices.dim() == 2 else 1
    idx = indices.reshape(T, k).long()
    loc = locations.reshape(T, k).long()
    valid = loc < capacity
    slots = idx * capacity + loc
    w = (gates.reshape(T, k).float() * valid.float()) if gates is not None else valid.float()
    out = torch.zeros((num_slots, g.shape[-1]), dtype=torch.float32, device=g.device)
    contrib = g.float().unsqueeze(1) * w.unsqueeze(-1)
    sv = slots[valid]
    out.index_add_(0, sv, contrib[valid])
    return out.to(g.dtype)


def reverse_layout_transform_backward_gate(g, y, indices, locations, capacity):
    T = indices.shape[0]
    k = indices.shape[1] if indices.dim() == 2 else 1
    idx = indices.reshape(T, k).long()
    loc = locations.reshape(T, k).long()
    valid = loc < capacity
    slots = torch.where(valid, idx * capacity + loc, torch.zeros_like(idx))
    rows = y[slots.reshape(-1)].reshape(T, k, -1).float()
    d = (rows * g.float().unsqueeze(1)).sum(-1) * valid.float()
    return d.reshape(indices.shape)


def balanced_assignment(scores, max_iterations=100):
    """Auction-based balanced assignment (BASE layers): every expert receives
    exactly T/E tokens; returns token ids grouped by expert, flattened [T].

    Bertsekas auction with a fixed epsilon run as batched device ops: each
    unassigned token bids for its best expert at price increments; every
    expert keeps its T/E highest bids.
    """
    s = scores.float()
    T, E = s.shape
    cap = T // E
    prices = torch.zeros(E, device=s.device)
    eps = 1e-4 * (s.max() - s.min()).clamp_min(1e-6)
    assign = torch.full((T,), -1, dtype=torch.long, device=s.device)
    for _ in range(max_iterations):
        free = assign < 0
        if not bool(free.any()):
            break
        val = s[free] - prices
        top2 = torch.topk(val, min(2, E), dim=1)
        best = top2.indices[:, 0]
        incr = (top2.values[:, 0] - (top2.values[:, 1] if E > 1 else top2.values[:, 0])) + eps
        bids = torch.full((T, E), -float('inf'), device=s.device)
        fidx = torch.nonzero(free).reshape(-1)
        bids[fidx, best] = (prices[best] + incr)
        # keep current owners with their price
        own = ~free
        bids[own, assign[own]] = prices[assign[own]]
        # each expert keeps top-cap bidders
        kv, ki = torch.topk(bids.t(), cap, dim=1)
        new_assign = torch.full((T,), -1, dtype=torch.long, device=s.device)
        valid = torch.isfinite(kv)
        e_ids = torch.arange(E, device=s.device).unsqueeze(1).expand(E, cap)
        new_assign[ki[valid]] = e_ids[valid]
        assign = new_assign
        full = valid.all(1)
        prices = torch.where(full, kv[:, -1], prices)
    # fall back: greedily place any leftovers
    free = torch.nonzero(assign < 0).reshape(-1)
    if free.numel():
        counts = torch.bincount(assign[assign >= 0], minlength=E)
        for t in free.tolist():
            e = int(torch.argmin(counts))
            assign[t] = e
            counts[e] += 1
    return torch.argsort(assign, stable=True)
