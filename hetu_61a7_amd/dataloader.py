"""Dataloaders (reference ``python/hetu/dataloader.py:11-257``).

A ``Dataloader`` owns one split of host data; ``dataloader_op([...])`` is the
graph source that yields the batch for the split being run.  Batches are
staged in a ring of pinned host buffers and copied to HBM with
``hipMemcpyAsync`` on a side stream one step ahead (prefetch depth 2), the
consumer stream waits on an event.  Under data parallelism each rank reads its
own shard (the reference's ``set_dp_rank`` hook is never called, SURVEY §0.2;
here the executor calls it).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .ops.node import Op
from . import ndarray


_TORCH_DT = {'<f4': torch.float32, '<i8': torch.int64, '<i4': torch.int32, '<f8': torch.float64,
             '|u1': torch.uint8, '<f2': torch.float16, '|b1': torch.bool}


class Dataloader(object):
    def __init__(self, raw_data, batch_size, name='default', func=None, drop_last=True,
                 shuffle=False, dtype=None):
        self.func = func if func else (lambda x: x)
        data = self.func(raw_data)
        if isinstance(data, torch.Tensor):
            data = data.numpy()
        data = np.asarray(data)
        if dtype is not None:
            data = data.astype(dtype)
        elif data.dtype == np.float64:
            data = data.astype(np.float32)
        self.raw_data = data
        self.batch_size = batch_size
        self.drop_last = drop_last
        self.shuffle = shuffle
        self.name = str(name)
        self.dp_rank, self.dp_nrank = 0, None
        self.parts = None
        self.cur_part = None
        self.slices = None
        self.initialized = False
        self.device = None
        self._stream = None

    def set_dp_rank(self, dp_rank, dp_nrank):
        self.dp_rank, self.dp_nrank = dp_rank, dp_nrank

    def set_mp_parts(self, cur_part, parts):
        self.cur_part, self.parts = cur_part, parts

    def init_states(self, device=None):
        if self.initialized:
            return
        data = self.raw_data
        if self.dp_nrank is not None and self.dp_nrank > 1:
            cur = data.shape[0] // self.dp_nrank
            data = data[cur * self.dp_rank: cur * (self.dp_rank + 1)]
        self.data = data
        self.samples_num = len(data)
        if self.drop_last:
            self.batch_num = self.samples_num // self.batch_size
        else:
            self.batch_num = (self.samples_num + self.batch_size - 1) // self.batch_size
        self.batch_num = max(self.batch_num, 1)
        self.shape = (self.batch_size,) + tuple(data.shape[1:])
        self.set_slices()
        self.device = device
        self.batch_index = 0
        self.order = np.arange(self.samples_num)
        self._ring = []
        self._pending = None
        # pinned staging ring: batch i goes through host slot i % 3 (no pin_memory call and
        # no event creation per batch; a slot is rewritten two batches after its H2D copy
        # was queued, and its event is waited for before that)
        self._pin = [None] * 3
        self._pev = [None] * 3
        self._slot = 0
        self._resident = None
        budget = float(os.environ.get('HETU_DATALOADER_RESIDENT_MB', '4096')) * (1 << 20)
        if device is not None and device.type == 'cuda' and not self.shuffle and self.slices is None \
                and self.data.nbytes <= budget:
            # HBM-resident split (288 GB per GPU): copied once, then every batch is a view of
            # it -- no per-step staging copy, event or kernel; the host rows ride along for
            # the PS / HET-cache lookups of sparse ids
            host = torch.from_numpy(np.ascontiguousarray(self.data))
            from . import native_array as _NA
            dev = _NA.empty(tuple(host.shape), dtype=host.dtype, device=device)
            dev.copy_(host.pin_memory() if host.numel() else host)
            torch.cuda.synchronize(device)
            self._resident = (dev, host)
            self._resident_cast = {}
        if device is not None and device.type == 'cuda':
            from .runtime import DeviceStream
            self._dstream = DeviceStream(torch.device(device).index, persistent=True)   # framework-created prefetch stream
            self._stream = self._dstream.torch
        self.initialized = True

    def set_slices(self):
        if self.parts is None:
            return
        new_shape, slcs = [], []
        for i, d in enumerate(self.shape):
            if i in self.parts:
                part = d // self.parts[i]
                st = part * self.cur_part[i]
                en = st + part
            else:
                st, en = 0, d
            slcs.append(slice(st, en))
            new_shape.append(en - st)
        self.slices = tuple(slcs)
        self.shape = tuple(new_shape)

    def reshape_tensor(self, tensor):
        return tensor if self.slices is None else tensor[self.slices]

    def _host_batch(self, idx):
        if idx == 0 and self.shuffle:
            np.random.shuffle(self.order)
        st = idx * self.batch_size
        en = min(st + self.batch_size, self.samples_num)
        sel = self.order[st:en] if self.shuffle else slice(st, en)
        b = self.data[sel]
        if self.slices is not None:
            b = b[(slice(None),) + self.slices[1:]]
        return np.ascontiguousarray(b)

    def _stage(self, idx):
        if self.device is None or self.device.type != 'cuda':
            return (torch.from_numpy(self._host_batch(idx)), None)
        from .runtime import DeviceEvent, use_stream
        from . import native_array as _NA
        src = self._host_src(idx)
        k = self._slot = (self._slot + 1) % 3
        buf, ev = self._pin[k], self._pev[k]
        n = int(np.prod(src.shape))
        if buf is None or buf.numel() < n or buf.dtype != _TORCH_DT.get(src.dtype.str, buf.dtype):
            buf = self._pin[k] = torch.from_numpy(np.ascontiguousarray(src)).reshape(-1).pin_memory()
        if ev is None:
            ev = self._pev[k] = DeviceEvent()
        else:
            ev.synchronize()                   # the last H2D copy out of this slot is done
        hb = buf[:n].view(src.shape)
        np.copyto(hb.numpy(), src)
        with use_stream(self._stream):
            db = _NA.empty(tuple(src.shape), dtype=hb.dtype, device=self.device)
            db.copy_(hb, non_blocking=True)
            ev.record(self._stream)
        # the host batch rides along: a consumer that needs the values on the host (PS /
        # HET-cache lookups of sparse ids, ``ps.table.host_ids``) reads it instead of a
        # device-to-host copy that would wait for the GPU
        db.hetu_host = hb
        return (db, ev, hb)

    def _host_src(self, idx):
        """the rows of batch idx as a numpy view when possible (copied once, into the
        pinned slot), else a gathered copy"""
        if self.shuffle or self.slices is not None:
            return self._host_batch(idx)
        st = idx * self.batch_size
        return self.data[st:min(st + self.batch_size, self.samples_num)]

    def _resident_batch(self, idx):
        dev, host = self._resident
        st = idx * self.batch_size
        en = min(st + self.batch_size, self.samples_num)
        t = dev[st:en]
        t.hetu_host = host[st:en]
        return t

    def resident_cast(self, dtype):
        """the resident split in ``dtype`` (cast once: mixed-precision feeds)"""
        c = self._resident_cast.get(dtype)
        if c is None:
            from .kernels.elementwise import cast
            c = self._resident_cast[dtype] = cast(self._resident[0], dtype)
        return c

    def get_arr(self):
        """Current batch on the device; prefetches the next one."""
        if self._resident is not None:
            t = self._resident_batch(self.batch_index)
            self.batch_index = (self.batch_index + 1) % self.batch_num
            return t
        if self._pending is None:
            self._pending = self._stage(self.batch_index)
        cur = self._pending
        nxt = (self.batch_index + 1) % self.batch_num
        self._pending = self._stage(nxt)
        self.batch_index = nxt
        t = cur[0]
        if len(cur) > 1 and cur[1] is not None:
            cur[1].wait(None)                       # the framework's current stream
            from .memory_pool import record_stream
            from ._base import cur_stream
            record_stream(t, cur_stream())
        return t

    def get_next_arr(self):
        return self.get_arr()

    def peek_next_arr(self):
        """The batch the next ``get_arr`` will return (already staged), without
        advancing; None before the first batch."""
        if self.initialized and self._resident is not None:
            st = self.batch_index * self.batch_size
            return self._resident[1][st:min(st + self.batch_size, self.samples_num)]
        if not self.initialized or self._pending is None:
            return None
        return self._pending[2] if len(self._pending) > 2 else self._pending[0]

    def get_cur_shape(self):
        return self.shape


class DataloaderOp(Op):
    def __init__(self, dataloaders):
        super().__init__(DataloaderOp, [], ndarray.cpu(0))
        self.dataloaders = {dl.name: dl for dl in dataloaders}
        self.name = 'DataloaderOp%d(%s)' % (self.id, '_'.join(self.dataloaders.keys()))
        self.keep_fp32 = False

    @property
    def desc(self):
        return self.name

    def set_dp_rank(self, dp_rank, dp_nrank):
        for d in self.dataloaders.values():
            d.set_dp_rank(dp_rank, dp_nrank)

    def set_mp_parts(self, cur_part, parts):
        for d in self.dataloaders.values():
            d.set_mp_parts(cur_part, parts)

    def get_batch_num(self, name):
        dl = self.dataloaders.get(name)
        if dl is None:
            return None
        if not dl.initialized:
            dl.init_states(None)
        return dl.batch_num

    def get_arr(self, name, config=None):
        dl = self.dataloaders[name]
        if not dl.initialized:
            dev = config.device if config is not None else None
            if getattr(self, 'host_feed', False):
                dev = torch.device('cpu')
            dl.init_states(dev)
        if getattr(dl, '_resident', None) is not None and config is not None and config.mixed_precision and \
                dl._resident[0].dtype == torch.float32 and not self.keep_fp32:
            # a resident fp32 split is cast once; batches are views of the bf16 copy
            i = dl.batch_index
            t = dl.get_arr()
            c = dl.resident_cast(torch.bfloat16)
            st = i * dl.batch_size
            v = c[st:st + t.shape[0]]
            v.hetu_host = t.hetu_host
            return v
        t = dl.get_arr()
        if config is not None and config.mixed_precision and t.is_cuda and t.dtype == torch.float32 \
                and not self.keep_fp32:
            from .kernels.elementwise import cast
            t = cast(t, torch.bfloat16)          # native cast kernel
        return t

    def get_next_arr(self, name):
        return self.get_arr(name)

    def peek_next_arr(self, name):
        dl = self.dataloaders.get(name)
        return None if dl is None else dl.peek_next_arr()

    def get_cur_shape(self, name):
        return self.dataloaders[name].get_cur_shape()

    def compute(self, input_vals, output_val=None, stream_handle=None):
        raise AssertionError('dataloader values are provided by the executor')

    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        raise NotImplementedError

    def forward_hook(self, config):
        self.ctx = config.context
        self.on_gpu = ndarray.is_gpu_ctx(self.ctx)
        self.on_cpu = not self.on_gpu

    def backward_hook(self, config):
        if config.comm_mode in ('AllReduce', 'Hybrid', 'PS') and config.nrank > 1:
            self.set_dp_rank(config.rank, config.nrank)
        for d in self.dataloaders.values():
            if d.initialized:
                continue
            d.init_states(config.device)


def dataloader_op(dataloaders):
    """``dataloaders``: Dataloader objects, or their constructor arguments as
    ``[data, batch_size, name, ...]`` lists or keyword dicts (reference
    dataloader.py:243-257)."""
    dls = []
    for dl in dataloaders:
        if isinstance(dl, Dataloader):
            dls.append(dl)
        elif isinstance(dl, (list, tuple)):
            dls.append(Dataloader(*dl))
        elif isinstance(dl, dict):
            dls.append(Dataloader(**dl))
        else:
            raise TypeError('dataloader_op: expected Dataloader, list or dict, got %r' % type(dl))
    return DataloaderOp(dls)


class GNNDataLoaderOp(Op):
    """Graph-sampling source (GraphMix hook in the reference; GraphMix itself is
    not shipped).  Feeds batches produced by a user ``handler``."""

    graph = None        # the sampled graph this step trains on
    nxt_graph = None    # the one after it (prefetchable)

    def __init__(self, handler, ctx=None):
        super().__init__(GNNDataLoaderOp, [], ctx or ndarray.cpu(0))
        self.handler = handler

    def get_batch_num(self, name):
        return None

    def get_arr(self, name, config=None):
        return self.handler(GNNDataLoaderOp.graph)

    def get_next_arr(self, name):
        return self.handler(GNNDataLoaderOp.nxt_graph)

    def get_cur_shape(self, name):
        return self.handler(GNNDataLoaderOp.graph).shape

    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        raise NotImplementedError

    @classmethod
    def step(cls, graph):
        """Two-deep queue (reference dataloader.py:180-183): the graph given now
        is trained on one step later, so its sampling overlaps the current step.
        Call it twice before the first run."""
        cls.graph = cls.nxt_graph
        cls.nxt_graph = graph
