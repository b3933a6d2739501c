"""CSR sparse x dense products (reference CuSparseCsrmv.cu / CuSparseCsrmm.cu).

Sparse matrices are ``ND_Sparse_Array`` (CSR: indptr ``row``, indices ``col``,
fp32 ``data``).  On a ROCm device the hand-written wave-per-row kernels of
``csrc/kernels/sparse.hip`` run; the transposed product uses an explicitly
transposed CSR built once per matrix and cached on it (deterministic, no
atomics).  The CPU backend uses torch's sparse kernels.

``col_window=(c0, c1)`` restricts A to columns ``[c0, c1)`` and indexes B rows
relative to ``c0`` -- the DistGCN-1.5D stage product (reference
``DistGCN_15d.py:61-63`` passes ``start_pos/end_pos`` to ``CuSparse_Csrmm``).
"""
from __future__ import annotations

import numpy as np
import torch
from .. import native_array as _NA

from . import native, fn, stream_ptr, check, is_bf16, P, I32, I64, F32


def _np_parts(a):
    return (a.row.asnumpy().astype(np.int64), a.col.asnumpy().astype(np.int64),
            a.data.asnumpy().astype(np.float32))


def _dev_parts(a, device):
    key = ('dev', str(device))
    c = a.cache.get(key)
    if c is None:
        rp, ci, v = _np_parts(a)
        c = (torch.from_numpy(rp.astype(np.int32)).to(device), torch.from_numpy(ci.astype(np.int32)).to(device),
             torch.from_numpy(v).to(device))
        a.cache[key] = c
    return c


def transposed(a):
    """CSR of A^T (cached on ``a``)."""
    t = a.cache.get('T')
    if t is None:
        import scipy.sparse
        from ..ndarray import ND_Sparse_Array, array
        rp, ci, v = _np_parts(a)
        m = scipy.sparse.csr_matrix((v, ci, rp), shape=(a.nrow, a.ncol)).T.tocsr()
        t = ND_Sparse_Array(array(m.data.astype(np.float32)), array(m.indptr, dtype=np.int32),
                            array(m.indices, dtype=np.int32), a.ncol, a.nrow)
        t.cache['T'] = a
        a.cache['T'] = t
    return t


def _torch_csr(a, dtype=torch.float32):
    if isinstance(a, torch.Tensor):
        return a
    rp, ci, v = _np_parts(a)
    return torch.sparse_csr_tensor(torch.from_numpy(rp), torch.from_numpy(ci), torch.from_numpy(v),
                                   size=(a.nrow, a.ncol)).to(dtype)


def csrmm(a, b, trans_A=False, trans_B=False, col_window=None, out=None, accumulate=False, alpha=1.0):
    """op(A) @ op(B) with A sparse CSR [m, k], B dense."""
    if isinstance(a, torch.Tensor):  # torch sparse input (tests / interop)
        mm = a.to_sparse_coo() if a.is_sparse_csr else a
        if trans_A:
            mm = mm.t()
        bb = b.t() if trans_B else b
        return torch.sparse.mm(mm.float(), bb.float()).to(b.dtype)
    A = transposed(a) if trans_A else a
    B = b.t() if trans_B else b
    c0, c1 = col_window if col_window is not None else (0, A.ncol)
    M, N = A.nrow, B.shape[1]
    if native(b) and b.dtype in (torch.float32, torch.bfloat16):
        B = B.contiguous()
        if out is None:
            out = (torch.zeros if accumulate else torch.empty)((M, N), dtype=b.dtype, device=b.device)
        rp, ci, v = _dev_parts(A, b.device)
        f = fn('hetu_csrmm', [P, P, P, P, P, I32, I32, I64, I64, I32, I32, F32, I32, I32, P])
        check(f(rp.data_ptr(), ci.data_ptr(), v.data_ptr(), B.data_ptr(), out.data_ptr(), M, N,
                B.stride(0), out.stride(0), int(c0), int(c1), float(alpha), int(accumulate),
                is_bf16(b), stream_ptr()), 'csrmm')
        return out
    csr = _torch_csr(A)
    if col_window is not None:
        dense_rows = _NA.zeros((A.ncol, N), dtype=torch.float32)
        dense_rows[c0:c1] = B.float()[:c1 - c0]
        r = torch.sparse.mm(csr.to_sparse_coo(), dense_rows)
    else:
        r = torch.sparse.mm(csr.to_sparse_coo(), B.float())
    r = (alpha * r).to(b.dtype)
    if out is not None:
        if accumulate:
            out.add_(r)
        else:
            out.copy_(r)
        return out
    return r


def csrmv(a, x, trans=False):
    if isinstance(a, torch.Tensor):
        m = a.to_sparse_coo() if a.is_sparse_csr else a
        if trans:
            m = m.t()
        return torch.mv(m.float(), x.float()).to(x.dtype)
    A = transposed(a) if trans else a
    if native(x) and x.dtype in (torch.float32, torch.bfloat16):
        xc = x.contiguous()
        y = _NA.empty(A.nrow, dtype=x.dtype, device=x.device)
        rp, ci, v = _dev_parts(A, x.device)
        f = fn('hetu_csrmv', [P, P, P, P, P, I32, I32, P])
        check(f(rp.data_ptr(), ci.data_ptr(), v.data_ptr(), xc.data_ptr(), y.data_ptr(), A.nrow,
                is_bf16(x), stream_ptr()), 'csrmv')
        return y
    return torch.mv(_torch_csr(A).to_sparse_coo(), x.float()).to(x.dtype)
