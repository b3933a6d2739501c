"""Optimizers and the OptimizerOp (reference ``python/hetu/optimizer.py:13-555``).

MI355X design:

* All dense trainable parameters of one ``OptimizerOp`` live in ONE flat fp32
  buffer (parameters are views into it) laid out in *gradient arrival order*
  (reverse topological order of the backward pass).  Gradients are written into a
  matching flat fp32 buffer as soon as they are produced.
* Data parallel: the flat gradient buffer is cut into contiguous buckets
  (default 32 MB); a bucket's RCCL SUM all-reduce is launched asynchronously the
  moment its last gradient lands, so communication overlaps the rest of the
  backward pass.  The reference issues one blocking NCCL call per parameter with
  a host-side event sync (``optimizer.py:145-163``, ``executor.py:1034-1036``).
* The update is ONE fused HIP launch over the whole flat buffer
  (``kernels/optimizer.hip``), which can also emit the bf16 compute copy of the
  weights (mixed precision: fp32 master weights, bf16 MFMA operands).
* Row-sparse (embedding) gradients are de-duplicated on device and applied with
  the row-sparse update kernels; parameters named ``expert*`` are excluded from
  the data-parallel all-reduce (MoE expert parallelism, reference
  ``optimizer.py:150-152``).
* Update rules and the AllReduce SUM semantics match the reference exactly.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import numpy as np

import torch
from . import native_array as _NA

from .ops.node import Op
from . import ndarray
from .kernels import optim as KO
from .kernels import sparse as KSP


class Optimizer(object):
    def __init__(self, learning_rate, l2reg=0):
        self.learning_rate = learning_rate
        self.l2reg = l2reg
        self.params = None
        self.tensors = None
        self.initiated = False
        self.name = 'Optimizer'
        self.betats_updated = False

    # reference API -----------------------------------------------------------------
    @staticmethod
    def get_var_list(loss):
        from .ops.variable import PlaceholderOp
        from .ops.executor import find_topo_sort
        return [n for n in find_topo_sort([loss]) if isinstance(n, PlaceholderOp) and n.trainable]

    def get_config(self):
        """Wire format for the PS server optimizer (reference optimizer.py:91-101)."""
        return (0, (self.learning_rate,), 1)

    def minimize(self, loss, var_list=None):
        from .ops.executor import gradients
        from .graph_opt import fuse_forward
        from .parallel.lowering import lower_dispatch
        lower_dispatch([loss])
        fuse_forward([loss])
        self.loss = loss
        if not var_list:
            var_list = self.get_var_list(loss)
        self.params = var_list
        grads, self.backward2forward, self.forward2backward = gradients(loss, self.params, return_all=True)
        from .graph_opt import fuse_backward
        fuse_backward([g for g in grads if g is not None])
        return OptimizerOp(grads, self)

    def get_learning_rate(self):
        lr = self.learning_rate
        if hasattr(lr, 'get'):
            return lr.get()
        return lr

    # flat update -------------------------------------------------------------------
    mode = 'sgd'
    n_states = 0

    def hyper(self, step):
        return dict(lr=self.get_learning_rate(), l2=self.l2reg)

    def dense_update(self, flat, step, dyn=None):
        KO.optimizer_flat(self.mode, flat.param, flat.grad, flat.s1, flat.s2, flat.shadow,
                          gscale=flat.gscale, seg_off=flat.seg_off, seg_off_host=flat.seg_host,
                          norms_ws=flat.norms_ws, dyn=dyn, **self.hyper(step))

    def sparse_update(self, table, state, ids, grads, step):
        h = self.hyper(step)
        h.pop('seg_off', None)
        KO.sparse_update(self.mode if self.mode != 'lamb' else 'adamw', table, ids, grads,
                         state.get('s1'), state.get('s2'), **h)

    def __deepcopy__(self, memo):
        return self


class SGDOptimizer(Optimizer):
    def __init__(self, learning_rate=0.01, l2reg=0):
        super().__init__(learning_rate, l2reg)
        self.name = 'SGD'

    def get_config(self):
        return (0, (self.get_learning_rate(),), 1)


class MomentumOptimizer(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.9, nesterov=False, l2reg=0):
        super().__init__(learning_rate, l2reg)
        self.momentum, self.nesterov = momentum, nesterov
        self.name = 'Momentum'
        self.mode = 'nesterov' if nesterov else 'momentum'
        self.n_states = 1

    def hyper(self, step):
        return dict(lr=self.get_learning_rate(), l2=self.l2reg, mu=self.momentum)

    def get_config(self):
        return (1, (self.get_learning_rate(), self.momentum, float(self.nesterov)), 3)


class AdaGradOptimizer(Optimizer):
    def __init__(self, learning_rate=0.01, initial_accumulator_value=0.0, eps=1e-7, l2reg=0):
        super().__init__(learning_rate, l2reg)
        self.initial_accumulator_value, self.eps = initial_accumulator_value, eps
        self.name = 'AdaGrad'
        self.mode = 'adagrad'
        self.n_states = 1
        self.state_init = (initial_accumulator_value, 0.0)

    def hyper(self, step):
        return dict(lr=self.get_learning_rate(), l2=self.l2reg, eps=self.eps)

    def get_config(self):
        return (2, (self.get_learning_rate(), self.initial_accumulator_value, self.eps), 3)


class AdamOptimizer(Optimizer):
    def __init__(self, learning_rate=0.01, beta1=0.9, beta2=0.999, epsilon=1e-7, l2reg=0):
        super().__init__(learning_rate, l2reg)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon
        self.name = 'Adam'
        self.mode = 'adam'
        self.n_states = 2

    def hyper(self, step):
        return dict(lr=self.get_learning_rate(), l2=self.l2reg, beta1=self.beta1, beta2=self.beta2,
                    beta1t=self.beta1 ** step, beta2t=self.beta2 ** step, eps=self.epsilon)

    def get_config(self):
        return (3, (self.get_learning_rate(), self.beta1, self.beta2, self.epsilon), 4)


class AdamWOptimizer(AdamOptimizer):
    def __init__(self, learning_rate=0.01, beta1=0.9, beta2=0.999, epsilon=1e-7, weight_decay=0):
        super().__init__(learning_rate, beta1, beta2, epsilon, 0)
        self.weight_decay = weight_decay
        self.name = 'AdamW'
        self.mode = 'adamw'

    def hyper(self, step):
        h = super().hyper(step)
        h['wd'] = self.weight_decay
        return h


class LambOptimizer(AdamWOptimizer):
    def __init__(self, learning_rate=0.01, beta1=0.9, beta2=0.999, epsilon=1e-7, weight_decay=0):
        super().__init__(learning_rate, beta1, beta2, epsilon, weight_decay)
        self.name = 'Lamb'
        self.mode = 'lamb'


# ---------------------------------------------------------------------------
SEG_ALIGN = 8   # flat-buffer segment alignment in elements (FlatGroup)


def flat_extent(numels):
    """elements a FlatGroup of segments of these sizes spans (SEG_ALIGN-aligned starts)"""
    off = 0
    for n in numels:
        off = -(-off // SEG_ALIGN) * SEG_ALIGN + n
    return off


def _filled(shape, value, dev):
    """fp32 framework array filled with ``value`` (native fill kernel on the device)"""
    t = _NA.empty(shape, dtype=torch.float32, device=dev)
    if t.is_cuda:
        from .kernels.tensor import fill_
        fill_(t, float(value))
    else:
        t.fill_(float(value))
    return t


class FlatGroup(object):
    """Flat fp32 storage for a set of dense parameters (one per device)."""

    def __init__(self, params: List[Op], values: Dict[Op, torch.Tensor], n_states: int,
                 state_init=(0.0, 0.0), shadow: bool = False, device=None, pad_to: int = 1,
                 state_numel: Optional[int] = None):
        self.params = params
        self.offsets = {}
        off = 0
        for p in params:
            # every segment starts 16-byte aligned in the bf16 shadow (8 elements): the
            # MFMA loaders stage 16-byte chunks, and one odd-sized bias ahead of a weight
            # (the MoE gate's 2) otherwise sent every later weight to the library GEMM
            off = -(-off // SEG_ALIGN) * SEG_ALIGN
            self.offsets[p] = (off, values[p].numel(), tuple(values[p].shape))
            off += values[p].numel()
        self.numel = off
        # ZeRO-1 pads the buffers so every bucket splits evenly over the ranks
        self.padded = max(-(-off // pad_to) * pad_to, 1)
        dev = device
        self.param = _NA.zeros(self.padded, dtype=torch.float32, device=dev)
        for p in params:
            self.view(p, 'param').copy_(values[p].float())
        self.grad = _NA.zeros_like(self.param)
        ns = self.padded if state_numel is None else state_numel   # ZeRO-1: this rank's shard only
        self.s1 = _filled((ns,), state_init[0], dev) if n_states >= 1 else None
        self.s2 = _filled((ns,), state_init[1], dev) if n_states >= 2 else None
        self.shadow = None
        if shadow:
            self.shadow = self.param.to(torch.bfloat16)  # same (channels-last) layout
        self.gscale = 1.0
        offs = [self.offsets[p][0] for p in params] + [off]
        self.seg_host = offs
        self.seg_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.norms_ws = _NA.zeros(2 * max(len(params), 1), dtype=torch.float32, device=dev)

    def view(self, p, which='param'):
        """View of parameter ``p`` inside a flat buffer.  4-D (conv) weights are
        laid out channels-last ([Cout, kh, kw, Cin] in memory) so the bf16 copy
        feeds the NHWC convolutions directly and their (channels-last) weight
        gradients land in the flat gradient buffer with a contiguous copy."""
        o, n, shp = self.offsets[p]
        buf = getattr(self, which)
        if len(shp) == 4:
            co, ci, kh, kw = shp
            return buf[o:o + n].view(co, kh, kw, ci).permute(0, 3, 1, 2)
        return buf[o:o + n].view(shp)


class Bucket(object):
    __slots__ = ('start', 'end', 'pending', 'total', 'work', 'own', 'zoff')

    def __init__(self, start, end, total):
        self.start, self.end, self.total = start, end, total
        self.pending = total
        self.work = None
        self.own, self.zoff = None, 0


class OptimizerOp(Op):
    def __init__(self, grads, optimizer):
        super().__init__(OptimizerOp, [g for g in grads if g is not None], None)
        self.name = 'Optimizer_%s' % optimizer.name
        self.optimizer = optimizer
        self.all_params = list(optimizer.params)
        self.param_of_input = [p for p, g in zip(optimizer.params, grads) if g is not None]
        self.step = 0
        self.flat: Optional[FlatGroup] = None
        self.sparse_state = {}
        self.comm = None
        self.dp = False
        self.buckets: List[Bucket] = []
        self.bucket_of = {}
        self.bucket_bytes = 32 << 20
        self.allreduce_mode = 'sum'
        self.ps_params = set()
        self.zero = False
        # gradient wire format of the DP all-reduce: 'fp32', or 'bf16' (half the bytes,
        # fp32 accumulation: Communicator.all_reduce_bf16)
        self.grad_wire = os.environ.get('HETU_GRAD_WIRE', 'fp32')
        # per-step bucket timeline (HETU_COMM_TRACE=1): host launch times relative to
        # the end of the backward pass, and device events on GPUs (comm_trace())
        self.trace = os.environ.get('HETU_COMM_TRACE', '0') == '1'
        self._trace = []

    # ----------------------------------------------------------------------------
    def gradient(self, output_grad):
        return None

    def infer_shape(self, input_shapes):
        return None

    def backward_hook(self, config):
        # data parallel wiring: AllReduce / Hybrid modes all-reduce dense grads
        self.config = config
        if config.comm_mode in ('AllReduce', 'Hybrid') and (config.nrank > 1 or getattr(config, 'force_dp', False)):
            self.dp = True
            self.comm = config.comm
        self.bucket_bytes = int(getattr(config, 'bucket_mb', 32) * (1 << 20))
        self.grad_wire = getattr(config, 'grad_wire', None) or self.grad_wire
        # PS placement (reference optimizer.py:145-163, Variable.py:55-81): embedding
        # tables (row-sparse grads) live on the PS in PS and Hybrid modes; in pure PS
        # mode the dense parameters are held there too (one flat key).
        self.ps_dense = None
        self.ps_dense_wanted = config.comm_mode == 'PS'
        if config.comm_mode in ('PS', 'Hybrid'):
            for p, g in zip(self.param_of_input, self.inputs):
                if getattr(p, 'is_embed', False) and g.use_indexed_slices:
                    p.ps_managed = True
                    self.ps_params.add(p)
        self.topo_input_order = self._grad_order()

    def _grad_order(self):
        """Order the executor computes the gradients in (find_topo_sort follows it).
        PS-held gradients first: their D2H copy and push overlap everything after.
        Dense gradients then follow the parameter order ('forward': the data-
        gradient chain runs first and the weight gradients after it, stem first),
        or last layer first ('reverse': each weight gradient right after the data
        gradient that feeds it, so all-reduce buckets launch throughout the
        backward pass).  Measured on ResNet-50 (1 GPU, bs 256): reverse costs
        0.5 ms/step of compute, more than the all-reduce it would expose at 8 GPUs
        with forward order (only the last 32 MB bucket), so forward is the default;
        ``HETU_GRAD_ORDER=reverse`` selects the other."""
        n = len(self.inputs)
        mode = os.environ.get('HETU_GRAD_ORDER', 'forward')
        first = [i for i in range(n) if self.param_of_input[i] in self.ps_params]
        rest = [i for i in range(n) if self.param_of_input[i] not in self.ps_params]
        if mode == 'reverse':
            rest = rest[::-1]
        return first + rest

    def forward_hook(self, config):
        self.ctx = config.context
        self.on_gpu = ndarray.is_gpu_ctx(self.ctx)
        self.on_cpu = not self.on_gpu

    def excluded_from_dp(self, p) -> bool:
        return p.name.startswith('expert') or getattr(p, 'no_dp', False)

    # ---- build flat storage in arrival order (called by the SubExecutor) ---------
    def setup(self, config, arrival_order: List[int]):
        if self.flat is not None:
            return
        opt = self.optimizer
        values = config.placeholder_to_arr_map
        dense, sparse = [], []
        for i in arrival_order:
            p = self.param_of_input[i]
            g = self.inputs[i]
            if p in self.ps_params:
                continue
            if g.use_indexed_slices and not getattr(p, 'force_dense_grad', False):
                sparse.append(p)
            else:
                dense.append(p)
        amp = config.mixed_precision
        self.zero = bool(getattr(config, 'zero', 0)) and self.dp and opt.mode != 'lamb' \
            and not any(self.excluded_from_dp(p) for p in dense)
        pad_to, state_numel = 1, None
        if self.zero:
            P = self.comm.nrank
            self.zero_unit = P * 64                       # every bucket splits into 64-aligned shards
            pad_to = self.zero_unit
            total = -(-flat_extent([values[p].numel() for p in dense]) // pad_to) * pad_to
            state_numel = max(total // P, 1)
        self.flat = FlatGroup(dense, values, opt.n_states, getattr(opt, 'state_init', (0.0, 0.0)),
                              shadow=amp, device=self.ctx.torch_device if self.ctx else None,
                              pad_to=pad_to, state_numel=state_numel)
        # ops that can write their gradient straight into the flat buffer get its view
        grad_of = {pp: g for pp, g in zip(self.param_of_input, self.inputs)}
        for p in dense:
            g = grad_of.get(p)
            if g is not None and hasattr(g, 'set_grad_dest') and not config.cpu_only:
                g.set_grad_dest(self.flat.view(p, 'grad'))
        for p in dense:
            values[p] = self.flat.view(p, 'param')
            # 1-D parameters (biases, BN/LN affine) are consumed by fp32 epilogues and
            # normalisation kernels: they read the fp32 master directly (no bf16 copy,
            # no per-step cast kernels)
            if amp and len(self.flat.offsets[p][2]) >= 2:
                config.compute_values[p] = self.flat.view(p, 'shadow')
            elif amp:   # library GEMM bias epilogues take bf16: hand them the shadow (no cast)
                values[p].hetu_bf16 = self.flat.view(p, 'shadow')
        for p in sparse:
            st = {}
            t = values[p]
            if opt.n_states >= 1:
                st['s1'] = torch.full_like(t, getattr(opt, 'state_init', (0.0,))[0])
            if opt.n_states >= 2:
                st['s2'] = _NA.zeros_like(t)
            self.sparse_state[p] = st
        # buckets over the flat gradient (contiguous, arrival order)
        self.slot = {}
        for i, p in enumerate(self.param_of_input):
            self.slot[i] = p
        if self.zero:
            self._make_zero_buckets(dense)
        elif self.dp:
            self._make_buckets(dense)
        if self.ps_dense_wanted and self.flat.numel > 0:
            from .ps.table import PSDense
            from .ps import PS_KEY_OPT_FLAT
            # key space: node ids are < 2^20; the flat dense key sits above them
            self.ps_dense = PSDense(self.flat, PS_KEY_OPT_FLAT + self.id, config)

    def _make_buckets(self, dense):
        """Contiguous buckets over the flat gradient, built from the END of the
        arrival order with growing caps (bucket_bytes/8, /4, /2, then full): the
        all-reduce that can only start once the last gradient has arrived -- the
        one the backward pass cannot hide -- is the smallest, while the early
        buckets stay large (few, big RCCL calls over the xGMI ring)."""
        full = max(self.bucket_bytes // 4, 1)
        cap = max(full // 8, 1)
        groups, cur, cur_n, nxt = [], [], 0, None
        for p in reversed([p for p in dense if not self.excluded_from_dp(p)]):
            o, n, _ = self.flat.offsets[p]
            # members must stay contiguous in the flat buffer (the next member starts at
            # the aligned end of this one; the alignment gap rides along, all zeros)
            if cur and (-(-(o + n) // SEG_ALIGN) * SEG_ALIGN != nxt or cur_n + n > cap):
                groups.append(cur)
                cur, cur_n = [], 0
                cap = min(cap * 2, full)
            cur.append(p)
            cur_n += n
            nxt = o
        if cur:
            groups.append(cur)
        self.buckets = []
        for members in reversed(groups):
            members = members[::-1]
            start = self.flat.offsets[members[0]][0]
            o_last, n_last, _ = self.flat.offsets[members[-1]]
            self._close_bucket(start, o_last + n_last - start, members)

    def _make_zero_buckets(self, dense):
        """ZeRO-1 (absent in the reference): fixed-size buckets
        over the padded flat buffer.  Each bucket is reduce-scattered as soon as
        every parameter overlapping it has its gradient (same overlap with the
        backward pass as the all-reduce buckets); rank r owns the r-th 1/P of
        every bucket, keeps optimizer state for that shard only, updates it, and
        all-gathers the fp32 weights.  Same bytes on the wire as an all-reduce,
        optimizer state memory / P."""
        P, r = self.comm.nrank, self.comm.rank
        unit = self.zero_unit
        cap = max(self.bucket_bytes // 4 // unit, 1) * unit
        total = self.flat.padded
        self.buckets, self.bucket_of = [], {}
        zoff = 0
        for s in range(0, total, cap):
            e = min(s + cap, total)
            b = Bucket(s, e, 0)
            n = (e - s) // P
            b.own, b.zoff = (s + r * n, s + (r + 1) * n), zoff
            zoff += n
            self.buckets.append(b)
        assert zoff == self.flat.s1.numel() if self.flat.s1 is not None else True
        self.flat.zgrad = _NA.zeros(max(zoff, 1), dtype=torch.float32, device=self.flat.param.device)
        for p in dense:
            o, n, _ = self.flat.offsets[p]
            bs = self.buckets[o // cap:(o + n - 1) // cap + 1]
            self.bucket_of[p] = bs
            for b in bs:
                b.total += 1
        for b in self.buckets:
            b.pending = b.total

    def _reduce_bucket(self, b, async_op=True):
        from .parallel.watchdog import labelled
        with labelled('grad bucket [%d:%d] of %d' % (b.start, b.end, self.flat.padded)):
            return self._reduce_bucket_inner(b, async_op)

    def _reduce_bucket_inner(self, b, async_op):
        if self.trace:
            self._trace_launch(b)
        if not self.zero:
            g = self.flat.grad[b.start:b.end]
            if self.grad_wire == 'bf16' and self.allreduce_mode == 'sum':
                w = self.comm.all_reduce_bf16(g, async_op=async_op)
            else:
                w = self.comm.all_reduce(g, self.allreduce_mode, async_op=async_op)
            if self.trace and w is not None:
                self._trace[-1]['work'] = w
            return w
        lo, hi = b.own
        return self.comm.reduce_scatter(self.flat.zgrad[b.zoff:b.zoff + hi - lo], self.flat.grad[b.start:b.end],
                                        self.allreduce_mode, async_op=async_op)

    def _zero_step(self):
        f, opt = self.flat, self.optimizer
        h = opt.hyper(self.step)
        dyn = getattr(self, 'dyn', None)
        gathers = []
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
            else:
                self._reduce_bucket(b, async_op=False)
            lo, hi = b.own
            sl = slice(b.zoff, b.zoff + hi - lo)
            KO.optimizer_flat(opt.mode, f.param[lo:hi], f.zgrad[sl], f.s1[sl] if f.s1 is not None else None,
                              f.s2[sl] if f.s2 is not None else None, None, gscale=f.gscale, dyn=dyn, **h)
            # the gather of this bucket overlaps the update of the next one
            gathers.append(self.comm.all_gather(f.param[b.start:b.end], f.param[lo:hi].clone(), async_op=True))
        for w in gathers:
            if w is not None:
                w.wait()
        if f.shadow is not None:
            f.shadow.copy_(f.param)

    def _close_bucket(self, start, n, members):
        b = Bucket(start, start + n, len(members))
        self.buckets.append(b)
        for p in members:
            self.bucket_of[p] = b

    # ---- called by the executor as each gradient is produced ---------------------
    def on_grad_ready(self, i, value):
        p = self.param_of_input[i]
        if p in self.ps_params:
            table = self.config.placeholder_to_arr_map[p]
            table.stage_grad(value, self.optimizer.get_learning_rate())
            self._pending_ps.append(table)
            return
        if isinstance(value, ndarray.IndexedSlices) or p in self.sparse_state:
            if self.dp and isinstance(value, ndarray.IndexedSlices) and not self.excluded_from_dp(p):
                value = _allgather_slices(self.comm, value)
            self._pending_sparse.append((p, value))
            return
        dst = self.flat.view(p, 'grad')
        if isinstance(value, ndarray.IndexedSlices):      # dense-updated sparse gradient
            value = value.to_dense()
        if not (value.data_ptr() == dst.data_ptr() and value.dtype == dst.dtype and
                value.stride() == dst.stride()):
            if value.shape != dst.shape:
                value = value.reshape(dst.shape)
            from .kernels.tensor import copy_into
            copy_into(dst, value)
        if self.dp:
            bs = self.bucket_of.get(p)
            if bs is not None:
                for b in (bs if self.zero else (bs,)):
                    b.pending -= 1
                    if b.pending == 0:
                        b.work = self._reduce_bucket(b)

    # ---- communication timeline (bench.py --comm-trace / HETU_COMM_TRACE=1) ------------
    def _trace_launch(self, b):
        import time
        rec = {'bytes': (b.end - b.start) * 4, 't_host': time.perf_counter(), 'ev': None}
        if self.flat is not None and self.flat.grad.is_cuda:
            from .runtime import DeviceEvent
            rec['ev'] = DeviceEvent(timing=True).record()
        self._trace.append(rec)

    def comm_trace(self):
        """Bucket timeline of the last step: per bucket its size, the host-side launch
        time relative to the end of the backward pass (negative = launched while the
        backward was still running), and on GPUs the device-side launch / completion
        times relative to the same point (ms)."""
        out = []
        end = getattr(self, '_bwd_end', None)
        if end is None:
            return out
        for r in self._trace:
            e = {'bytes': r['bytes'], 'launch_host_ms': round((r['t_host'] - end[0]) * 1e3, 3)}
            if r['ev'] is not None and end[1] is not None:
                end[1].synchronize()
                e['launch_dev_ms'] = round(-r['ev'].elapsed_time(end[1]), 3)
                ev = getattr(r.get('work'), 'event', None)
                if ev is not None:
                    try:
                        ev.synchronize()
                        e['done_dev_ms'] = round(-ev.elapsed_time(end[1]), 3)
                    except RuntimeError:   # event without timing
                        pass
            out.append(e)
        return out

    def begin_step(self):
        self._trace = []
        self._pending_sparse = []
        self._pending_ps = []
        for b in self.buckets:
            b.pending = b.total
            b.work = None

    def compute(self, input_vals, output_val=None, stream_handle=None):
        self.step += 1
        if self.trace:
            import time
            ev = None
            if self.flat is not None and self.flat.grad.is_cuda:
                from .runtime import DeviceEvent
                ev = DeviceEvent(timing=True).record()
            self._bwd_end = (time.perf_counter(), ev)
        if self.zero:
            self._zero_step()
        for b in self.buckets if not self.zero else ():
            if b.work is not None:
                b.work.wait()
            elif self.dp:
                # a bucket whose grads never arrived this step (should not happen)
                self.comm.all_reduce(self.flat.grad[b.start:b.end], self.allreduce_mode)
        if self.zero:
            pass
        elif self.ps_dense is not None:
            self.ps_dense.step(self.optimizer.get_learning_rate())
        elif self.flat is not None and self.flat.numel > 0:
            self.optimizer.dense_update(self.flat, self.step, getattr(self, 'dyn', None))
        for table in self._pending_ps:
            table.flush_grad(force=False)     # ASP + prefetch: behind the next step's staging
        self._pending_ps = []
        for p, sl in self._pending_sparse:
            table = self.config.placeholder_to_arr_map[p]
            nrows = table.shape[0] if isinstance(table, torch.Tensor) else 0
            if nrows and table.is_cuda and nrows <= 65536 and nrows * 4 <= sl._t(sl.indices).numel() * 64:
                # small table: all-rows dedup with -1 for untouched rows (no host sync
                # on the number of distinct ids; the sparse kernel skips -1 rows)
                from .kernels import sparse as ksparse
                w = sl.dense_shape[-1]
                uniq, merged = ksparse.dedup_rows_dense(sl._t(sl.indices), sl._t(sl.values).reshape(-1, w), nrows)
            else:
                uniq, merged = sl.deduplicate().indices, sl.values
            if self.optimizer.mode == 'lamb':
                pass
            self.optimizer.sparse_update(table, self.sparse_state.get(p, {}), uniq, merged, self.step)
        self._pending_sparse = []
        lr = self.optimizer.learning_rate
        return None


def _allgather_slices(comm, sl):
    idx = sl._t(sl.indices).reshape(-1).contiguous()
    val = sl._t(sl.values).reshape(idx.numel(), -1).contiguous()
    oi = _NA.empty((idx.numel() * comm.nrank,), dtype=idx.dtype, device=idx.device)
    ov = _NA.empty((val.shape[0] * comm.nrank, val.shape[1]), dtype=val.dtype, device=val.device)
    comm.all_gather(oi, idx)
    comm.all_gather(ov, val)
    return ndarray.IndexedSlices(oi, ov, sl.dense_shape)
