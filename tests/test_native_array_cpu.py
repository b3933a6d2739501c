"""Framework-owned strided arrays (csrc/runtime/array.cc, hetu_61a7_amd/native_array.py):
the reference's DLArray C ABI (src/common/dlarray.h:18-66; c_runtime_api.cc:93-142
DLArrayAlloc / Free / CopyFromTo) -- allocation, zero-copy views (reshape, transpose,
broadcast with stride 0, slice), copies, DLPack export to torch (non-owning) and import
(borrowing), and reference counting back to zero."""
import gc

import numpy as np
import pytest
import torch

from hetu_61a7_amd import native_array as NA


def _live():
    gc.collect()
    return NA.stats()['live_allocations']


def test_array_views_share_memory_and_free_at_last_reference():
    base = _live()
    a = NA.Array.empty((4, 6), torch.float32, 'cpu')
    t = a.torch()
    t.copy_(torch.arange(24.).reshape(4, 6))
    tr = a.view((6, 4), (1, 6)).torch()                      # transpose
    np.testing.assert_array_equal(tr.numpy(), np.arange(24.).reshape(4, 6).T)
    sl = a.view((2, 3), (6, 1), byte_offset=4 * (6 + 2)).torch()   # rows 1..2, cols 2..4
    np.testing.assert_array_equal(sl.numpy(), np.arange(24.).reshape(4, 6)[1:3, 2:5])
    bc = a.reshape((24,)).reshape((4, 6)).view((1, 6), (0, 1)).broadcast_to((5, 6)).torch()
    assert bc.stride() == (0, 1) and bc.shape == (5, 6)
    np.testing.assert_array_equal(bc.numpy()[3], np.arange(6.))
    t[0, 0] = 100.
    assert tr[0, 0] == 100. and bc[4, 0] == 100.          # one allocation under every view
    with pytest.raises(ValueError):
        a.view((5, 6), (6, 1))                             # past the allocation
    assert _live() == base + 1
    del a, t, tr, sl, bc
    assert _live() == base


def test_copy_contiguous_and_rows():
    a = NA.Array.empty((3, 8), torch.float32, 'cpu')
    a.torch().copy_(torch.randn(3, 8))
    b = NA.Array.empty((3, 8), torch.float32, 'cpu')
    b.copy_from(a)
    assert torch.equal(a.torch(), b.torch())
    c = NA.Array.empty((3, 16), torch.float32, 'cpu')
    c.torch().zero_()
    c.view((3, 8), (16, 1), byte_offset=4 * 4).copy_from(a)    # strided rows (2-D copy)
    assert torch.equal(c.torch()[:, 4:12], a.torch()) and float(c.torch()[:, :4].abs().sum()) == 0


def test_empty_family_matches_torch_semantics():
    x = NA.empty(2, 3, 4, 5, dtype=torch.bfloat16, memory_format=torch.channels_last)
    assert x.shape == (2, 3, 4, 5) and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
    y = NA.empty_like(x, dtype=torch.float32)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.float32
    z = NA.zeros((7,), dtype=torch.int64)
    assert z.dtype == torch.int64 and int(z.abs().sum()) == 0
    w = NA.empty(5, dtype=torch.float32)
    assert w.shape == (5,)
    assert NA.zeros_like(x).is_contiguous(memory_format=torch.channels_last)


def test_dlpack_import_borrows_torch_memory():
    base = _live()
    src = torch.arange(12, dtype=torch.float32).reshape(3, 4)
    a = NA.Array.from_torch(src)
    v = a.view((4, 3), (1, 4)).torch()
    np.testing.assert_array_equal(v.numpy(), src.numpy().T)
    src[1, 1] = -5.
    assert v[1, 1] == -5.
    assert NA.Array.from_torch(src).info()['shape'] == (3, 4)
    del a, v
    assert _live() == base


def test_ndarray_api_is_backed_by_native_arrays():
    import hetu_61a7_amd as ht
    before = NA.stats()['created']
    e = ht.empty((3, 4), ctx=ht.cpu(0))
    a = ht.array(np.ones((2, 5), np.float32), ctx=ht.cpu(0))
    assert NA.stats()['created'] >= before + 2
    assert a.asnumpy().sum() == 10 and e.shape == (3, 4)
    r = a.reshape((5, 2))
    assert r.shape == (5, 2) and r.tensor.data_ptr() == a.tensor.data_ptr()
    h = a.handle.info()
    assert h['shape'] == (2, 5) and h['data'] == a.tensor.data_ptr()
