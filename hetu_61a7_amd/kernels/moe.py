"""MoE routing kernels: top-k gating, dispatch (layout transform) and combine
(reverse layout transform) -- ``moe.hip``.

Reference LayoutTransform.cu scatters token i into slot
``expert(i) * capacity + location(i)`` (dropped when location >= capacity) and
combines with gate weights through atomicAdd; its gate-gradient uses a
hard-coded 32-lane shuffle.  Here dispatch and combine are gathers keyed by a
per-slot source index (deterministic, no atomics) with wave64 dot products, and
the top-k gate is fused (softmax + top-k + capacity slots + balance terms).
"""
from __future__ import annotations

import ctypes

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32


def _dc(t, dtype=None):
    """contiguous (optionally re-typed) tensor; device copies / casts on the native
    kernels, no copy when it already is one"""
    dtype = dtype or t.dtype
    if t.is_contiguous() and t.dtype == dtype:
        return t
    if t.is_cuda:
        from .tensor import copy_into
        return copy_into(_NA.empty(t.shape, dtype=dtype, device=t.device), t)
    return t.to(dtype).contiguous()


def _ik(t, T):
    return t.reshape(T, -1).long().contiguous()


def _io_ok(*ts):
    return native(ts[0]) and all(supported_float(t) for t in ts) and len({t.dtype for t in ts}) == 1


def topk(x, k, softmax=False):
    """(values, indices) of the k largest entries per row; ``softmax=True``
    ranks softmax(x) and also returns the probabilities (wave-per-row kernel)."""
    R, E = x.reshape(-1, x.shape[-1]).shape
    if native(x) and supported_float(x) and E <= 512 and k <= min(8, E):
        x2 = x.reshape(R, E).contiguous()
        probs = _NA.empty((R, E) if softmax else (1,), dtype=torch.float32, device=x.device)
        idx = _NA.empty((R, k), dtype=torch.int64, device=x.device)
        val = _NA.empty((R, k), dtype=torch.float32, device=x.device)
        f = fn('hetu_moe_gate_topk', [P, P, P, P, I32, I32, I32, I32, I32, P])
        check(f(x2.data_ptr(), probs.data_ptr(), idx.data_ptr(), val.data_ptr(), R, E, k, int(softmax),
                is_bf16(x2), stream_ptr()), 'moe_gate_topk')
        return (val, idx, probs) if softmax else (val, idx)
    if softmax:
        p = torch.softmax(x.reshape(R, E).float(), -1)
        v, i = torch.topk(p, k, dim=-1)
        return v, i, p
    v, i = torch.topk(x, k, dim=-1)
    return v, i


def locations(idx, num_experts, probs=None, inactive=False):
    """Slot of every (token, choice) inside its expert, choice-major (the
    reference's cumsum chain, moe_layer.py / TopGate.py), plus per-expert routed
    counts and column sums of ``probs`` (balance loss terms)."""
    T, k = idx.shape
    E = num_experts
    if native(idx):
        idx = idx.long().contiguous()
        loc = _NA.empty((T, k), dtype=torch.int64, device=idx.device)
        if inactive:   # choices with idx -1 (dense-to-sparse gate) keep loc -1: dropped everywhere
            from .tensor import fill_
            fill_(loc, -1)
        counts = _NA.empty((E,), dtype=torch.int32, device=idx.device)
        psum = _NA.empty((E,), dtype=torch.float32, device=idx.device) if probs is not None else None
        # per-segment hit counts of the segmented scan (an int32 workspace from the pool)
        nws = int(fn('hetu_moe_locations_ws', [I32, I32, I32], I64)(T, k, E))
        ws = _NA.empty((nws,), dtype=torch.int32, device=idx.device) if nws > 0 else None
        f = fn('hetu_moe_locations2', [P, P, P, P, P, I32, I32, I32, P, P])
        check(f(idx.data_ptr(), probs.contiguous().data_ptr() if probs is not None else None, loc.data_ptr(),
                counts.data_ptr(), psum.data_ptr() if psum is not None else None, T, k, E,
                ws.data_ptr() if ws is not None else None, stream_ptr()), 'moe_locations')
        return loc, counts, psum
    il = idx.long()
    on = (il >= 0).t().reshape(-1)
    oh = torch.nn.functional.one_hot(il.clamp_min(0).t().reshape(-1), E) * on.unsqueeze(1)   # [(j, t), E]
    cum = torch.cumsum(oh, 0) - 1
    loc = torch.where(on, (cum * oh).sum(1), torch.full_like(on, -1, dtype=torch.int64))
    loc = loc.reshape(k, T).t().contiguous()
    counts = oh.sum(0).int()
    psum = probs.float().sum(0) if probs is not None else None
    return loc, counts, psum


def aux_terms(counts, psum, T):
    """(coef [E] = counts / T, l_aux [] = E * sum_e psum_e / T * coef_e): one native launch"""
    E = counts.numel()
    if native(psum) and counts.dtype == torch.int32 and psum.dtype == torch.float32:
        coef = _NA.empty((E,), dtype=torch.float32, device=psum.device)
        l_aux = _NA.empty((), dtype=torch.float32, device=psum.device)
        f = fn('hetu_moe_aux', [P, P, P, P, I32, I32, P])
        check(f(counts.contiguous().data_ptr(), psum.contiguous().data_ptr(), coef.data_ptr(), l_aux.data_ptr(),
                int(T), int(E), stream_ptr()), 'moe_aux')
        return coef, l_aux
    coef = counts.float() / float(T)
    return coef, (psum / float(T) * coef).sum() * float(E)


MAX_K = 16   # choices per token the kernels take (moe.hip kMaxK)


def gate_backward(probs, idx, dgate, aux_coef, scale=1.0):
    """d logits of (gate values [T, k] = probs[t, idx], balance term sum_e c_e * sum_t probs[t, e]),
    times ``scale`` (1 / tau of a tempered softmax); choices with idx < 0 carry no gradient."""
    T, E = probs.shape
    k = idx.shape[1]
    if native(probs) and E <= 512 and k <= MAX_K:
        out = _NA.empty((T, E), dtype=torch.float32, device=probs.device)
        dg = _dc(dgate.reshape(T, k), torch.float32) if dgate is not None else None
        ac = _dc(aux_coef, torch.float32) if aux_coef is not None else None
        f = fn('hetu_moe_gate_backward', [P, P, P, P, P, I32, I32, I32, ctypes.c_float, P])
        check(f(probs.contiguous().data_ptr(), idx.long().contiguous().data_ptr(), ptr_or_none(dg), ptr_or_none(ac),
                out.data_ptr(), T, E, k, float(scale), stream_ptr()), 'moe_gate_backward')
        return out
    dp = _NA.zeros((T, E), dtype=torch.float32, device=probs.device)
    if dgate is not None:
        il = idx.long()
        on = il >= 0
        dp.scatter_add_(1, torch.where(on, il, _NA.zeros_like(il)),
                        torch.where(on, dgate.float().reshape(T, k), _NA.zeros((T, k), device=probs.device)))
    if aux_coef is not None:
        dp = dp + aux_coef.float().unsqueeze(0)
    p = probs.float()
    return scale * p * (dp - (p * dp).sum(-1, keepdim=True))


# ---- dense-to-sparse gate ------------------------------------------------------------------
def _philox_x(seed, counter):
    """first 32-bit output of Philox4x32-10 (common.h Philox::gen(...).x) for uint64 arrays of
    counters -- the CPU reference path draws the same Gumbel noise as the HIP kernel"""
    return philox4(seed, counter)[0]


def philox4(seed, counter):
    """the four 32-bit outputs (x, y, z, w) of Philox4x32-10 (common.h Philox::gen) for a
    uint64 array of counters: host references of the kernels' random streams"""
    import numpy as np
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    m32 = np.uint64(0xFFFFFFFF)
    c = np.asarray(counter, dtype=np.uint64)
    c0 = c & m32
    c1 = c >> np.uint64(32)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & m32
        hi1, lo1 = p1 >> np.uint64(32), p1 & m32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & m32, lo1, (hi0 ^ c3 ^ k1) & m32, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & m32
        k1 = (k1 + np.uint64(0xBB67AE85)) & m32
    return c0, c1, c2, c3


def dts_gate(logits, k, inv_tau, threshold, seed, noise=True):
    """Dense-to-sparse gate forward (moe.hip dts_gate_k): y = softmax((logits + gumbel) * inv_tau);
    the k largest choices per token, choice j > 0 active only while y >= threshold (inactive:
    idx -1, value 0).  Returns (val [T, k] fp32, idx [T, k] int64, probs [T, E] fp32,
    hist [k + 1] int32: tokens by number of active choices)."""
    T, E = logits.shape
    seed = int(seed) & ((1 << 64) - 1)
    if native(logits) and supported_float(logits) and E <= 512 and 1 <= k <= min(MAX_K, E):
        x = logits.contiguous()
        probs = _NA.empty((T, E), dtype=torch.float32, device=x.device)
        idx = _NA.empty((T, k), dtype=torch.int64, device=x.device)
        val = _NA.empty((T, k), dtype=torch.float32, device=x.device)
        hist = _NA.empty((k + 1,), dtype=torch.int32, device=x.device)
        f = fn('hetu_moe_dts_gate', [P, P, P, P, P, I32, I32, I32, ctypes.c_float, ctypes.c_float, ctypes.c_uint64,
                                     I32, I32, P])
        check(f(x.data_ptr(), probs.data_ptr(), idx.data_ptr(), val.data_ptr(), hist.data_ptr(), T, E, k,
                float(inv_tau), float(threshold), seed, int(bool(noise)), is_bf16(x), stream_ptr()), 'moe_dts_gate')
        return val, idx, probs, hist
    if logits.is_cuda:
        raise RuntimeError('dts_gate: no hand-written kernel for E=%d k=%d %s' % (E, k, logits.dtype))
    import numpy as np
    z = logits.float()
    if noise:
        cnt = (np.arange(T, dtype=np.uint64)[:, None] * np.uint64(E) + np.arange(E, dtype=np.uint64)[None, :])
        u = (_philox_x(seed, cnt) >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0) + 0.5 / 16777216.0
        z = z - torch.from_numpy(np.log(-np.log(u)).astype(np.float32))
    probs = torch.softmax(z * float(inv_tau), -1)
    v, i = torch.topk(probs, k, dim=-1)           # ties: torch order; the kernel takes the lowest id
    on = torch.ones_like(v, dtype=torch.bool)
    on[:, 1:] = v[:, 1:] >= threshold
    idx = torch.where(on, i, torch.full_like(i, -1))
    val = torch.where(on, v, _NA.zeros_like(v))
    hist = torch.bincount(on.sum(1), minlength=k + 1).to(torch.int32)
    return val, idx, probs, hist


def ptr_or_none(t):
    return t.data_ptr() if t is not None else None


def _slot_map(idx, loc, capacity, nslots):
    Tk = idx.numel()
    m = _NA.empty((nslots,), dtype=torch.int32, device=idx.device)
    f = fn('hetu_moe_slot_map', [P, P, P, I32, I32, I32, P])
    check(f(idx.data_ptr(), loc.data_ptr(), m.data_ptr(), Tk, capacity, nslots, stream_ptr()), 'moe_slot_map')
    return m


def layout_transform(x, indices, locations, capacity, num_experts):
    """x [T, d]; indices/locations [T, k] -> out [E*capacity, d] (zero padded)."""
    T, d = x.shape
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    nslots = num_experts * capacity
    if _io_ok(x):
        x = _dc(x)
        smap = _slot_map(idx, loc, capacity, nslots)
        out = _NA.empty((nslots, d), dtype=x.dtype, device=x.device)
        f = fn('hetu_moe_gather_slots', [P, P, P, P, I32, I32, I32, I32, P])
        check(f(x.data_ptr(), smap.data_ptr(), None, out.data_ptr(), nslots, d, k, is_bf16(x), stream_ptr()),
              'moe_gather_slots')
        return out
    out = _NA.zeros((nslots, d), dtype=x.dtype, device=x.device)
    valid = (loc < capacity) & (loc >= 0) & (idx >= 0)
    slots = idx * capacity + loc
    tok = torch.arange(T, device=x.device).unsqueeze(1).expand(T, k)
    out[slots[valid]] = x[tok[valid]]
    return out


def _combine(y, idx, loc, w, capacity, T):
    d = y.shape[-1]
    k = idx.shape[1]
    y = _dc(y)
    out = _NA.empty((T, d), dtype=y.dtype, device=y.device)
    wf = _dc(w.reshape(T, k), torch.float32) if w is not None else None
    f = fn('hetu_moe_combine', [P, P, P, P, P, I32, I32, I32, I32, I32, P])
    check(f(y.data_ptr(), idx.data_ptr(), loc.data_ptr(), ptr_or_none(wf), out.data_ptr(), T, k, capacity, d,
            is_bf16(y), stream_ptr()), 'moe_combine')
    return out


def layout_transform_backward(g, indices, locations, capacity):
    """grad wrt x: sum over the k slots each token was written to."""
    T = indices.shape[0]
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    if _io_ok(g) and k <= MAX_K:
        return _combine(g, idx, loc, None, capacity, T)
    valid = (loc < capacity) & (loc >= 0) & (idx >= 0)
    slots = torch.where(valid, idx * capacity + loc, _NA.zeros_like(idx))
    gathered = g[slots.reshape(-1)].reshape(T, k, -1) * valid.unsqueeze(-1).to(g.dtype)
    return gathered.sum(1)


def reverse_layout_transform(y, indices, locations, gates, capacity):
    """combine: out[t] = sum_j gates[t, j] * y[slot(t, j)] (dropped slots -> 0)."""
    T = indices.shape[0]
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    if _io_ok(y) and k <= MAX_K:
        return _combine(y, idx, loc, gates, capacity, T)
    valid = (loc < capacity) & (loc >= 0) & (idx >= 0)
    slots = torch.where(valid, idx * capacity + loc, _NA.zeros_like(idx))
    rows = y[slots.reshape(-1)].reshape(T, k, -1).float()
    w = (gates.reshape(T, k).float() * valid.float()) if gates is not None else valid.float()
    return (rows * w.unsqueeze(-1)).sum(1).to(y.dtype)


def reverse_layout_transform_backward_data(g, indices, locations, gates, capacity, num_slots):
    T = indices.shape[0]
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    d = g.shape[-1]
    if _io_ok(g):
        g = _dc(g)
        smap = _slot_map(idx, loc, capacity, num_slots)
        wf = _dc(gates.reshape(T, k), torch.float32) if gates is not None else None
        out = _NA.empty((num_slots, d), dtype=g.dtype, device=g.device)
        f = fn('hetu_moe_gather_slots', [P, P, P, P, I32, I32, I32, I32, P])
        check(f(g.data_ptr(), smap.data_ptr(), ptr_or_none(wf), out.data_ptr(), num_slots, d, k, is_bf16(g),
                stream_ptr()), 'moe_gather_slots')
        return out
    valid = (loc < capacity) & (loc >= 0) & (idx >= 0)
    slots = idx * capacity + loc
    w = (gates.reshape(T, k).float() * valid.float()) if gates is not None else valid.float()
    out = _NA.zeros((num_slots, d), dtype=torch.float32, device=g.device)
    contrib = g.float().unsqueeze(1) * w.unsqueeze(-1)
    out.index_add_(0, slots[valid], contrib[valid])
    return out.to(g.dtype)


def reverse_layout_transform_backward_fused(g, y, indices, locations, gates, capacity, num_slots):
    """(``reverse_layout_transform_backward_data``, ``reverse_layout_transform_backward_gate``)
    -- on the GPU one kernel reading the token gradient once"""
    T = indices.shape[0]
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    d = g.shape[-1]
    if _io_ok(g, y) and tuple(y.shape) == (num_slots, d):
        g, y = _dc(g), _dc(y)
        smap = _slot_map(idx, loc, capacity, num_slots)
        wf = _dc(gates.reshape(T, k), torch.float32) if gates is not None else None
        out = _NA.empty((num_slots, d), dtype=g.dtype, device=g.device)
        gout = _NA.empty((T, k), dtype=torch.float32, device=g.device)
        f = fn('hetu_moe_gather_slots_gate', [P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, P])
        check(f(g.data_ptr(), y.data_ptr(), smap.data_ptr(), ptr_or_none(wf), loc.data_ptr(), out.data_ptr(),
                gout.data_ptr(), num_slots, T * k, d, k, capacity, is_bf16(g), stream_ptr()), 'moe_gather_slots_gate')
        return out, gout.reshape(indices.shape)
    return (reverse_layout_transform_backward_data(g, indices, locations, gates, capacity, num_slots),
            reverse_layout_transform_backward_gate(g, y, indices, locations, capacity))


def reverse_layout_transform_backward_gate(g, y, indices, locations, capacity):
    T = indices.shape[0]
    idx, loc = _ik(indices, T), _ik(locations, T)
    k = idx.shape[1]
    d = g.shape[-1]
    if _io_ok(g, y):
        g, y = _dc(g), _dc(y)
        out = _NA.empty((T, k), dtype=torch.float32, device=g.device)
        f = fn('hetu_moe_gate_grad', [P, P, P, P, P, I32, I32, I32, I32, I32, P])
        check(f(g.data_ptr(), y.data_ptr(), idx.data_ptr(), loc.data_ptr(), out.data_ptr(), T * k, k, capacity, d,
                is_bf16(g), stream_ptr()), 'moe_gate_grad')
        return out.reshape(indices.shape)
    valid = (loc < capacity) & (loc >= 0) & (idx >= 0)
    slots = torch.where(valid, idx * capacity + loc, _NA.zeros_like(idx))
    rows = y[slots.reshape(-1)].reshape(T, k, -1).float()
    dd = (rows * g.float().unsqueeze(1)).sum(-1) * valid.float()
    return dd.reshape(indices.shape)


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
    prices = _NA.zeros(E, device=s.device)
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
