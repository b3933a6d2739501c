"""Embedding gather / row scatter-add / dedup (``embedding.hip``)."""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32


def gather_rows(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """out[..., :] = table[ids[...], :]; out-of-range ids give zero rows."""
    dim = table.shape[-1]
    idx = ids.reshape(-1).long()
    out_shape = tuple(ids.shape) + (dim,)
    if native(table) and supported_float(table) and table.is_contiguous():
        idx = idx.contiguous()
        out = _NA.empty(out_shape, dtype=table.dtype, device=table.device)
        f = fn('hetu_gather_rows', [P, P, P, I64, I64, I64, I32, P])
        check(f(table.data_ptr(), idx.data_ptr(), out.data_ptr(), idx.numel(), dim,
                table.shape[0], is_bf16(table), stream_ptr()), 'gather_rows')
        return out
    valid = (idx >= 0) & (idx < table.shape[0])
    safe = torch.where(valid, idx, _NA.zeros_like(idx))
    out = table[safe] * valid.unsqueeze(1).to(table.dtype)
    return out.reshape(out_shape)


def scatter_add_rows(dst: torch.Tensor, ids: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst[ids[r], :] += src[r, :] (fp32 dst).  Deterministic mode: rows sorted by
    destination (stable) and summed per destination in order by one wave."""
    dim = dst.shape[-1]
    idx = ids.reshape(-1).long()
    src2 = src.reshape(-1, dim)
    from . import deterministic
    if native(dst) and dst.dtype == torch.float32 and supported_float(src2) and dst.is_contiguous() \
            and deterministic():
        idx = idx.contiguous()
        src2 = src2.contiguous()
        sidx, perm = torch.sort(idx, stable=True)
        seg_row, counts = torch.unique_consecutive(sidx, return_counts=True)
        off = _NA.zeros(seg_row.numel() + 1, dtype=torch.int64, device=idx.device)
        torch.cumsum(counts, 0, out=off[1:])
        f = fn('hetu_segment_sum_rows', [P, P, P, P, P, I64, I64, I64, I32, P])
        check(f(dst.data_ptr(), seg_row.data_ptr(), off.data_ptr(), perm.data_ptr(), src2.data_ptr(),
                seg_row.numel(), dim, dst.shape[0], is_bf16(src2), stream_ptr()), 'segment_sum_rows')
        return dst
    if native(dst) and dst.dtype == torch.float32 and supported_float(src2) and dst.is_contiguous():
        idx = idx.contiguous()
        src2 = src2.contiguous()
        f = fn('hetu_scatter_add_rows', [P, P, P, I64, I64, I64, I32, P])
        check(f(dst.data_ptr(), idx.data_ptr(), src2.data_ptr(), idx.numel(), dim, dst.shape[0],
                is_bf16(src2), stream_ptr()), 'scatter_add_rows')
        return dst
    valid = (idx >= 0) & (idx < dst.shape[0])
    dst.index_add_(0, idx[valid], src2[valid].to(dst.dtype))
    return dst


def dedup_rows(idx: torch.Tensor, vals: torch.Tensor):
    """Unique ids and the per-unique-id sum of their rows (fp32).

    Heavily duplicated ids (BERT's token-type embedding: 8192 rows onto 2; the
    position embedding: onto 128) would serialise thousands of fp32 atomics on
    each destination element.  Rows are then spread over K private replicas of
    the destination (row r -> replica r % K, at most ~16 rows per replica row),
    scattered with little contention, and the replicas summed."""
    uniq, inv = torch.unique(idx, sorted=True, return_inverse=True)
    nu, n, dim = uniq.numel(), inv.numel(), vals.shape[-1]
    from . import deterministic
    K = min(64, n // max(nu * 16, 1))
    if K > 1 and vals.is_cuda and not deterministic():
        rep = torch.arange(n, device=inv.device) % K
        scratch = _NA.zeros((K * nu, dim), dtype=torch.float32, device=vals.device)
        scatter_add_rows(scratch, inv.reshape(-1) + rep * nu, vals.reshape(n, dim))
        return uniq, scratch.view(K, nu, dim).sum(0)
    merged = _NA.zeros((nu, dim), dtype=torch.float32, device=vals.device)
    scatter_add_rows(merged, inv, vals)
    return uniq, merged


def dedup_rows_dense(idx: torch.Tensor, vals: torch.Tensor, nrows: int):
    """Sync-free dedup for a small table: (ids, merged) over ALL ``nrows`` rows --
    merged[r] = sum of the rows with id r, ids[r] = r where some row hit r, else
    -1 (the row-sparse optimizer kernel skips those, so untouched rows keep
    exact sparse-update semantics).  Unlike ``dedup_rows`` nothing depends on
    the number of distinct ids, so the host never waits for the GPU (BERT's
    position and token-type embeddings).  Duplicates are spread over private
    replicas as in ``dedup_rows``; out-of-range ids are dropped."""
    n, dim = idx.numel(), vals.shape[-1]
    idx = idx.reshape(-1).long()
    from . import deterministic
    K = 1 if deterministic() else max(1, min(64, n // max(nrows * 16, 1)))
    v2 = vals.reshape(n, dim)
    if native(vals) and supported_float(v2) and v2.is_contiguous() and not deterministic():
        from .tensor import zeros
        idx = idx.contiguous()
        scratch = zeros((K * nrows * dim,), torch.float32, vals.device)
        hit = zeros((nrows,), torch.int32, vals.device)
        merged = _NA.empty((nrows, dim), dtype=torch.float32, device=vals.device)
        ids = _NA.empty((nrows,), dtype=torch.int64, device=vals.device)
        f = fn('hetu_dedup_rows_dense', [P, P, I32, I64, I64, I64, I32, P, P, P, P, P])
        check(f(idx.data_ptr(), v2.data_ptr(), is_bf16(v2), n, dim, nrows, K, scratch.data_ptr(), hit.data_ptr(),
                merged.data_ptr(), ids.data_ptr(), stream_ptr()), 'dedup_rows_dense')
        from . import record_native
        record_native('dedup_rows_dense')
        return ids, merged
    valid = (idx >= 0) & (idx < nrows)
    tgt = idx if K == 1 else idx + (torch.arange(n, device=idx.device) % K) * nrows
    tgt = torch.where(valid, tgt, torch.full_like(tgt, -1))
    scratch = _NA.zeros((K * nrows, dim), dtype=torch.float32, device=vals.device)
    scatter_add_rows(scratch, tgt, vals.reshape(n, dim))
    merged = scratch if K == 1 else scratch.view(K, nrows, dim).sum(0)
    hit = _NA.zeros(nrows + 1, dtype=torch.int64, device=idx.device)
    hit.scatter_(0, torch.where(valid, idx, torch.full_like(idx, nrows)), 1)
    rows = torch.arange(nrows, device=idx.device)
    ids = torch.where(hit[:nrows] > 0, rows, torch.full_like(rows, -1))
    return ids, merged
