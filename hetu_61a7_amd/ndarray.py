"""Device contexts and array containers.

Parity target: reference ``python/hetu/ndarray.py`` (DLContext ``:10-57``,
NDArray ``:140-402``, ``array``/``empty`` ``:405-444``, CSR ``:460-504``,
IndexedSlices ``:507-618``).

MI355X design: the memory behind an ``NDArray`` is a framework-owned native array
(``csrc/runtime/array.cc``: refcounted strided header over a BFC-pool allocation -- HBM
of ``gpu(i)``, pinned host DRAM for PS / cache staging, or plain host memory), allocated
stream-ordered on the framework's current HIP stream (``runtime.use_stream``).  The
Python-side handle is a non-owning ``torch.Tensor`` view of it (DLPack, zero copy), used
as the op vocabulary of the CPU reference paths; torch owns neither the memory nor the
streams.  Unlike the reference (fp32 only, float-encoded indices) arrays carry a real
dtype: fp32 / bf16 / fp16 / int32 / int64.
"""
from __future__ import annotations

import socket
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
from . import native_array as _NA

_HOSTNAME = socket.gethostname()


class DLContext(object):
    """A device context: (device_type, device_id, hostname).

    device_type 1 = cpu, 2 = gpu (same encoding as the reference so YAML/configs
    written for Hetu keep working).
    """

    MASK2STR = {1: 'cpu', 2: 'gpu'}

    __slots__ = ('device_id', 'device_type', 'hostname', 'local')

    def __init__(self, device_id: int, device_type: int, hostname: str = 'localhost'):
        self.device_id = int(device_id)
        self.device_type = int(device_type)
        if hostname in ('localhost', _HOSTNAME, '127.0.0.1'):
            self.hostname = _HOSTNAME
            self.local = True
        else:
            self.hostname = hostname
            self.local = False

    def __repr__(self) -> str:
        if self.local:
            return "%s(%d)" % (DLContext.MASK2STR[self.device_type], self.device_id)
        return "%s:%s(%d)" % (self.hostname, DLContext.MASK2STR[self.device_type], self.device_id)

    def full_repr(self) -> str:
        return "%s:%s:%d" % (self.hostname, DLContext.MASK2STR[self.device_type], self.device_id)

    def relocalize(self) -> None:
        self.local = self.hostname in ('localhost', _HOSTNAME)

    def __hash__(self):
        if self.local:
            return hash((self.device_type, self.device_id))
        return hash((self.hostname, self.device_type, self.device_id))

    def __eq__(self, other):
        return isinstance(other, DLContext) and hash(self) == hash(other)

    def __ne__(self, other):
        return not self.__eq__(other)

    # --- MI355X mapping -------------------------------------------------
    @property
    def torch_device(self) -> torch.device:
        if self.device_type == 2:
            return torch.device('cuda', self.device_id)
        return torch.device('cpu')

    def __getstate__(self):
        return (self.device_id, self.device_type, self.hostname)

    def __setstate__(self, st):
        self.device_id, self.device_type, self.hostname = st
        self.relocalize()


def cpu(dev_id: int = 0) -> DLContext:
    return DLContext(dev_id, 1)


def gpu(dev_id: int = 0) -> DLContext:
    return DLContext(dev_id, 2)


def rcpu(hostname: str, dev_id: int = 0) -> DLContext:
    return DLContext(dev_id, 1, hostname=hostname)


def rgpu(hostname: str, dev_id: int = 0) -> DLContext:
    return DLContext(dev_id, 2, hostname=hostname)


def is_gpu_ctx(ctx) -> bool:
    return bool(ctx) and isinstance(ctx, DLContext) and ctx.device_type == 2


def shape_to_stride(shape: Sequence[int]) -> Tuple[int, ...]:
    stride = [1] * len(shape)
    for i in range(len(shape) - 1, 0, -1):
        stride[i - 1] = stride[i] * shape[i]
    return tuple(stride)


_NP2TORCH = {
    np.dtype(np.float32): torch.float32,
    np.dtype(np.float64): torch.float64,
    np.dtype(np.float16): torch.float16,
    np.dtype(np.int32): torch.int32,
    np.dtype(np.int64): torch.int64,
    np.dtype(np.int8): torch.int8,
    np.dtype(np.uint8): torch.uint8,
    np.dtype(np.bool_): torch.bool,
}


def to_torch_dtype(dtype) -> torch.dtype:
    if dtype is None:
        return torch.float32
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, str):
        return {'bf16': torch.bfloat16, 'bfloat16': torch.bfloat16, 'fp16': torch.float16,
                'float16': torch.float16, 'fp32': torch.float32, 'float32': torch.float32,
                'int32': torch.int32, 'int64': torch.int64}[dtype]
    return _NP2TORCH[np.dtype(dtype)]


def ctx_of(t: torch.Tensor) -> DLContext:
    if t.is_cuda:
        return gpu(t.device.index or 0)
    return cpu(0)


class NDArray(object):
    """An array of the framework (reference ``ndarray.py:140``): a native strided array
    header (``native_array.Array``, the C ABI of ``csrc/runtime/array.cc``) plus its torch
    view for the kernel wrappers.  Arrays made by ``array`` / ``empty`` own framework
    memory; an NDArray wrapped around a tensor from elsewhere borrows it (the native
    header is created on first use of ``handle``)."""

    __slots__ = ('tensor', 'ctx', '_handle')

    def __init__(self, tensor: torch.Tensor, ctx: Optional[DLContext] = None, handle=None):
        self.tensor = tensor
        self.ctx = ctx if ctx is not None else ctx_of(tensor)
        self._handle = handle

    @property
    def handle(self):
        """the native array header (DLPack-borrowed from the tensor when not framework-made)"""
        if self._handle is None:
            from .native_array import Array
            self._handle = Array.from_torch(self.tensor)
        return self._handle

    # shape / metadata -------------------------------------------------
    @property
    def shape(self) -> Tuple[int, ...]:
        return tuple(self.tensor.shape)

    @property
    def stride(self) -> Tuple[int, ...]:
        return tuple(self.tensor.stride())

    @property
    def dtype(self):
        return self.tensor.dtype

    @property
    def lazy(self) -> bool:
        return not self.tensor.is_contiguous()

    def __repr__(self):
        return 'NDArray(%s, shape=%s, dtype=%s)' % (self.ctx, self.shape, self.tensor.dtype)

    def __len__(self):
        return self.tensor.shape[0]

    # data movement ----------------------------------------------------
    def asnumpy(self) -> np.ndarray:
        t = self.tensor.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()

    def __setitem__(self, in_slice, value):
        if not isinstance(in_slice, slice) or in_slice.start is not None or in_slice.stop is not None:
            raise ValueError('Array only support set from numpy array')
        if isinstance(value, NDArray):
            self.tensor.copy_(value.tensor)
        elif isinstance(value, (np.ndarray, np.generic)):
            self.tensor.copy_(torch.from_numpy(np.ascontiguousarray(value)).to(self.tensor.dtype))
        else:
            self.tensor.fill_(value)

    def copyto(self, target):
        if isinstance(target, DLContext):
            return NDArray(self.tensor.to(target.torch_device, copy=True), target)
        target.tensor.copy_(self.tensor, non_blocking=True)
        return target

    def async_h2d(self, source, stream_handle=None, event_handle=None):
        """Copy a host array into this device array on ``stream_handle``."""
        src = source.tensor if isinstance(source, NDArray) else source
        from .runtime import use_stream
        with use_stream(stream_handle if stream_handle is not None and stream_handle.torch_stream is not None
                        else None):
            self.tensor.copy_(src, non_blocking=True)
            if event_handle is not None:
                event_handle.record(stream_handle)

    def async_d2h(self, source, stream_handle=None, event_handle=None):
        src = source.tensor if isinstance(source, NDArray) else source
        from .runtime import use_stream
        with use_stream(stream_handle if stream_handle is not None and stream_handle.torch_stream is not None
                        else None):
            self.tensor.copy_(src, non_blocking=True)
            if event_handle is not None:
                event_handle.record(stream_handle)

    # zero-copy views (reference ndarray.py:298-381) ----------------------
    def reshape(self, shape, target=None):
        if self._handle is not None and self.tensor.is_contiguous():
            h = self._handle.reshape(tuple(shape))       # native zero-copy view
            v = h.torch()
        else:
            h, v = None, self.tensor.reshape(shape)
        if target is not None:
            target.tensor, target._handle = v, h
            return target
        return NDArray(v, self.ctx, h)

    def broadcast_to(self, shape, target=None):
        if self._handle is not None:
            h = self._handle.broadcast_to(tuple(shape))   # stride-0 native view
            v = h.torch()
        else:
            h, v = None, self.tensor.expand(shape)
        if target is not None:
            target.tensor, target._handle = v, h
            return target
        return NDArray(v, self.ctx, h)

    def inplace_copy(self, target):
        target.tensor.copy_(self.tensor)
        return target


class _null(object):
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def array(arr, ctx: Optional[DLContext] = None, data_type=np.float32, dtype=None) -> NDArray:
    """Create an NDArray from numpy (reference ``ndarray.py:405``)."""
    ctx = ctx or cpu(0)
    if isinstance(arr, NDArray):
        arr = arr.asnumpy()
    if isinstance(arr, torch.Tensor):
        t = arr
    else:
        arr = np.asarray(arr)
        if dtype is None and data_type is not None and arr.dtype.kind == 'f':
            arr = arr.astype(data_type)
        t = torch.from_numpy(np.ascontiguousarray(arr))
    if dtype is not None:
        t = t.to(to_torch_dtype(dtype))
    out = empty(tuple(t.shape), ctx, t.dtype)      # framework memory, filled from the source
    out.tensor.copy_(t)
    return out


def empty(shape, ctx: Optional[DLContext] = None, dtype=np.float32) -> NDArray:
    """a new framework array (reference DLArrayAlloc): HBM from the device BFC pool, host
    arrays pinned when a GPU is present (the reference's cudaMallocHost CPU arrays)"""
    ctx = ctx or cpu(0)
    dt = to_torch_dtype(dtype)
    from . import native_array
    dev = ctx.torch_device
    if native_array.available() and native_array._device_ok(dev):
        h = native_array.Array.empty(tuple(shape), dt, dev, pinned=dev.type == 'cpu' and torch.cuda.is_available())
        return NDArray(h.torch(), ctx, h)
    return NDArray(_NA.empty(tuple(shape), dtype=dt, device=dev), ctx)


def numpyasdlarrayhandle(data: np.ndarray) -> NDArray:
    return NDArray(torch.from_numpy(np.ascontiguousarray(data)), cpu(0))


def pinned_empty(shape, dtype=torch.float32) -> torch.Tensor:
    """Pinned host buffer used for async staging: carved from the native
    pinned-DRAM BFC pool (``memory_pool.pinned_pool``, hipHostMalloc regions),
    or torch's pinned allocator when the pool library is not built."""
    if torch.cuda.is_available():
        from . import memory_pool
        if memory_pool.available():
            return memory_pool.pinned_pool().tensor(tuple(shape), dtype)
        return _NA.empty(tuple(shape), dtype=dtype).pin_memory()
    return _NA.empty(tuple(shape), dtype=dtype)


class ND_Sparse_Array(object):
    """CSR sparse matrix (reference ``ndarray.py:460-504``)."""

    __slots__ = ('data', 'row', 'col', 'nrow', 'ncol', 'lazy', 'cache')

    def __init__(self, data: NDArray, row: NDArray, col: NDArray, nrow: int, ncol: int):
        self.data = data
        self.row = row
        self.col = col
        self.nrow = nrow
        self.ncol = ncol
        self.lazy = False
        self.cache = {}  # device CSR parts / transposed CSR (kernels.spmm)

    @property
    def shape(self):
        return (self.nrow, self.ncol)

    @property
    def ctx(self):
        return self.data.ctx

    def to_torch(self) -> torch.Tensor:
        return torch.sparse_csr_tensor(self.row.tensor.long(), self.col.tensor.long(),
                                       self.data.tensor, size=(self.nrow, self.ncol))

    def asnumpy(self):
        import scipy.sparse
        return scipy.sparse.csr_matrix((self.data.asnumpy(), self.col.asnumpy(), self.row.asnumpy()),
                                       shape=(self.nrow, self.ncol)).toarray()


def sparse_array(values, indices, shape, ctx: Optional[DLContext] = None) -> ND_Sparse_Array:
    """Build a CSR array from COO (values, (row, col)) like the reference."""
    import scipy.sparse
    ctx = ctx or cpu(0)
    mat = scipy.sparse.csr_matrix((values, indices), shape=shape)
    return ND_Sparse_Array(array(mat.data, ctx), array(mat.indptr, ctx, dtype=np.int32),
                           array(mat.indices, ctx, dtype=np.int32), shape[0], shape[1])


class IndexedSlices(object):
    """Row-sparse gradient: ``values[i]`` belongs to row ``indices[i]``.

    Reference ``ndarray.py:507-618``.  Indices are int64 here (the reference
    stores them as float32 and loses precision above 2^24).
    """

    __slots__ = ('indices', 'values', 'dense_shape', 'deduplicated', 'lazy',
                 'to_dense_flag', 'dense_arr')

    def __init__(self, indices=None, values=None, dense_shape=None):
        self.indices = indices
        self.values = values
        self.dense_shape = tuple(dense_shape) if dense_shape is not None else None
        self.deduplicated = False
        self.lazy = False
        self.to_dense_flag = False
        self.dense_arr = None

    def _t(self, x):
        return x.tensor if isinstance(x, NDArray) else x

    def get_dense_shape(self):
        return self.dense_shape

    def get_sparse_shape(self):
        return tuple(self._t(self.values).shape)

    def update(self, indices, values, dense_shape):
        self.indices = indices
        self.values = values
        self.dense_shape = tuple(dense_shape)
        self.deduplicated = False

    def deduplicate(self):
        """Merge duplicate rows (device-side sort + segment-sum)."""
        if self.deduplicated:
            return self
        from .kernels import sparse as ksparse
        idx = self._t(self.indices).reshape(-1).long()
        vals = self._t(self.values)
        width = vals.shape[-1]
        vals = vals.reshape(-1, width)
        uniq, merged = ksparse.dedup_rows(idx, vals)
        self.indices, self.values = uniq, merged
        self.deduplicated = True
        return self

    def to_dense(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        from .kernels import sparse as ksparse
        idx = self._t(self.indices).reshape(-1).long()
        vals = self._t(self.values)
        width = self.dense_shape[-1]
        vals = vals.reshape(-1, width)
        if out is None:
            out = _NA.zeros(self.dense_shape, dtype=vals.dtype, device=vals.device)
        elif out.is_cuda:
            from .kernels.tensor import fill_
            fill_(out, 0)
        else:
            out.zero_()
        ksparse.scatter_add_rows(out.view(-1, width), idx, vals)
        return out

    def merge(self, other: 'IndexedSlices') -> 'IndexedSlices':
        """concatenated (indices, values) of two sparse gradients of one table (framework
        arrays filled by the native strided copy: no torch.cat kernel)"""
        a_i, b_i = self._t(self.indices).reshape(-1), self._t(other.indices).reshape(-1)
        w = self.dense_shape[-1]
        a_v, b_v = self._t(self.values).reshape(-1, w), self._t(other.values).reshape(-1, w)
        if b_i.dtype != a_i.dtype:
            b_i = b_i.to(a_i.dtype)
        if b_v.dtype != a_v.dtype:
            b_v = b_v.to(a_v.dtype)
        na, nb = a_i.numel(), b_i.numel()
        i = _NA.empty(na + nb, dtype=a_i.dtype, device=a_i.device)
        v = _NA.empty((na + nb, w), dtype=a_v.dtype, device=a_v.device)
        if a_i.is_cuda:
            from .kernels.tensor import copy_into
            copy_into(i[:na], a_i)
            copy_into(i[na:], b_i)
            copy_into(v[:na], a_v)
            copy_into(v[na:], b_v)
        else:
            i[:na].copy_(a_i)
            i[na:].copy_(b_i)
            v[:na].copy_(a_v)
            v[na:].copy_(b_v)
        return IndexedSlices(i, v, self.dense_shape)

    def cpu(self):
        return IndexedSlices(self._t(self.indices).cpu(), self._t(self.values).cpu(), self.dense_shape)

    def asnumpy(self):
        return self.to_dense().float().cpu().numpy()
