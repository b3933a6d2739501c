"""CSR sparse x dense products (reference CuSparseCsrmv.cu / CuSparseCsrmm.cu).

Sparse matrices are ``ND_Sparse_Array`` (CSR).  torch's CSR kernels serve as
the implementation here; the DistGCN path uses ``csrmm`` with row-split
partitions.
"""
from __future__ import annotations

import torch


def _csr(a):
    if hasattr(a, 'to_torch'):
        return a.to_torch()
    return a


def csrmv(a, x, trans=False):
    m = _csr(a).to(x.dtype) if not hasattr(a, 'to_torch') else _csr(a)
    if trans:
        m = m.to_dense().t() if not m.is_sparse_csr else m.to_sparse_coo().t()
    return torch.mv(m if not m.is_sparse_csr else m.to_sparse_coo(), x.float()).to(x.dtype)


def csrmm(a, b, trans_A=False, trans_B=False):
    m = _csr(a)
    bb = b.t() if trans_B else b
    mm = m.to_sparse_coo() if m.is_sparse_csr else m
    if trans_A:
        mm = mm.t()
    return torch.sparse.mm(mm.float(), bb.float()).to(b.dtype)
