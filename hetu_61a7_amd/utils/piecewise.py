"""Piecewise hipGraph replay for steps that talk to the host in the middle.

A parameter-server step (Wide&Deep, BASELINE config 3) cannot be one graph: the embedding
lookups read the HET cache / PS on the host, the embedding gradient is staged to the host
as soon as it exists, and the optimizer pushes and pulls on the host.  Everything between
those points is plain device work -- the dense MLP forward and backward -- which the
eager executor pays for at Python speed, op by op (the step is launch-bound: ~40 small
kernels at batch 128).  Here the executor's op list is cut at the host ops into segments;
each device segment is captured once into its own HIP graph (its allocations carved from
a private BFC capture pool) and replayed every step, and the host ops run eagerly between
the replays, on the same stream.

Values a captured segment reads from outside it are either stable (parameters, outputs of
earlier captured segments -- the same buffers every step) or volatile (feeds, dataloader
batches, host-op outputs): a volatile input is copied into a static buffer before each
replay.  Gradient hooks (optimizer ``on_grad_ready``) end a segment and run after its
replay, in executor order.  A step whose inputs change shape, or a capture that fails,
falls back to eager execution.  The reference runs every op eagerly
(``python/hetu/gpu_ops/executor.py:1000-1056``); SURVEY §7.4.4 (graph capture instead of
a tracing compiler).
"""
from __future__ import annotations

import sys

import torch

from .. import native_array as _NA


def host_bound(sub, n):
    """ops that must run eagerly between the captured segments"""
    from ..optimizer import OptimizerOp
    from ..ops.embedding import EmbeddingLookUp, EmbeddingLookUp_Gradient
    if getattr(n, 'host_bound', False) or isinstance(n, (OptimizerOp, EmbeddingLookUp_Gradient)):
        return True
    if isinstance(n, EmbeddingLookUp):
        t = sub.config.placeholder_to_arr_map.get(n.inputs[0])
        return not isinstance(t, torch.Tensor)      # a PS / HET-cache table
    return False


class _Segment(object):
    __slots__ = ('lo', 'hi', 'host', 'graph', 'pool', 'stream', 'ext', 'static', 'outputs', 'aux_out',
                 'shapes', 'hooked', 'sig')

    def __init__(self, lo, hi, host):
        self.lo, self.hi, self.host = lo, hi, host
        self.graph = self.pool = self.stream = None
        self.ext = []            # (node, kind) read from outside the segment
        self.static = {}         # (node, kind) -> static buffer of a volatile input
        self.outputs, self.aux_out, self.shapes = {}, {}, {}
        self.hooked = []
        self.sig = None


class PiecewiseRunner(object):
    def __init__(self, sub, warmup=3):
        self.sub = sub
        self.warmup = warmup
        self.calls = 0
        self.failed = False
        self.segments = None
        self.replays = 0

    # -- plan ------------------------------------------------------------------------------
    def _plan(self):
        sub = self.sub
        nodes = sub.computing_nodes
        segs, lo = [], 0
        for i, n in enumerate(nodes):
            if host_bound(sub, n):
                if lo < i:
                    segs.append(_Segment(lo, i, False))
                segs.append(_Segment(i, i + 1, True))
                lo = i + 1
            elif sub.grad_hooks.get(n):
                segs.append(_Segment(lo, i + 1, False))   # hooks run after the replay
                lo = i + 1
        if lo < len(nodes):
            segs.append(_Segment(lo, len(nodes), False))
        produced_by = {n: k for k, s in enumerate(segs) for n in nodes[s.lo:s.hi]}
        for k, s in enumerate(segs):
            if s.host:
                continue
            own = set(nodes[s.lo:s.hi])
            seen = set()
            for i in range(s.lo, s.hi):
                for inp, kind in sub.input_specs[i]:
                    if inp in own or (inp, kind) in seen:
                        continue
                    seen.add((inp, kind))
                    if kind == 'shape':
                        continue                           # host metadata (signature-checked)
                    src = produced_by.get(inp)
                    stable = inp in sub.param_nodes or (src is not None and not segs[src].host)
                    if not stable:
                        for k2 in (('value', 'aux') if kind == 'va' else (kind,)):
                            if (inp, k2) not in s.ext:
                                s.ext.append((inp, k2))
            s.hooked = [n for n in nodes[s.lo:s.hi] if sub.grad_hooks.get(n)]
        self.segments = segs

    # -- step ------------------------------------------------------------------------------
    def run(self, feed_dict, convert):
        sub = self.sub
        self.calls += 1
        if self.calls <= self.warmup or self.failed:
            vals = sub._run_eager(feed_dict)
            return sub._collect(vals, convert)
        if self.segments is None:
            self._plan()
        try:
            vals = self._step(feed_dict)
        except _Fallback as e:
            print('piecewise hipgraph: %s; running this executor eagerly' % e, file=sys.stderr)
            self.failed = True
            self._drop()
            return sub._collect(e.vals, convert)
        return self._collect(vals, convert)

    def _drop(self):
        for s in self.segments or ():
            s.graph = None
            if s.pool is not None:
                s.pool.release()
                s.pool = None

    def close(self):
        self._drop()

    def _collect(self, vals, convert):
        """captured outputs are overwritten by the next replay: unconverted device outputs
        are handed out as copies"""
        if convert:
            return self.sub._collect(vals, True)
        from ..kernels.tensor import copy_into
        out = dict(vals)
        for n in self.sub.eval_node_list:
            v = vals.get(n)
            if isinstance(v, torch.Tensor) and v.is_cuda:
                out[n] = copy_into(_NA.empty(tuple(v.shape), dtype=v.dtype, device=v.device), v)
        return self.sub._collect(out, False)

    def _step(self, feed_dict):
        from ..kernels import rng as _RNG
        sub = self.sub
        vals = sub._prepare_inputs(feed_dict)
        _RNG.new_step()
        aux, shapes = {}, {}
        for op in sub.opt_ops:
            op.begin_step()
        for s in self.segments:
            if s.host:
                self._run_ops(s.lo, s.hi, vals, aux, shapes, hooks=True)
                continue
            sig = tuple((id(n), kind, _sig(vals, aux, n, kind)) for n, kind in s.ext)
            if any(x[2] is None for x in sig):
                raise _Fallback('a volatile segment input is not a device tensor', self._finish_eager(s, vals, aux, shapes))
            if s.graph is None:
                s.sig = sig
                self._capture(s, vals, aux, shapes)
            elif sig != s.sig:
                raise _Fallback('a segment input changed shape', self._finish_eager(s, vals, aux, shapes))
            from ..kernels.tensor import copy_into
            for key, st in s.static.items():
                n, kind = key
                copy_into(st, aux[n] if kind == 'aux' else vals[n])
            from .._base import cur_stream
            s.graph.replay(cur_stream())
            self.replays += 1
            vals.update(s.outputs)
            aux.update(s.aux_out)
            shapes.update(s.shapes)
            for n in s.hooked:
                for op, j in sub.grad_hooks[n]:
                    op.on_grad_ready(j, vals[n])
            for i in range(s.lo, s.hi):
                for dead in sub.release_after[i]:
                    vals.pop(dead, None)
                    aux.pop(dead, None)
        sub.step_count += 1
        return vals

    def _finish_eager(self, s, vals, aux, shapes):
        """run the rest of this step eagerly from segment ``s`` on (fallback)"""
        self._run_ops(s.lo, len(self.sub.computing_nodes), vals, aux, shapes, hooks=True)
        self.sub.step_count += 1
        return vals

    def _run_ops(self, lo, hi, vals, aux, shapes, hooks, keep=()):
        from ..ops.executor import _shape_of
        from ..ops.nn import AuxResult
        sub = self.sub
        for i in range(lo, hi):
            n = sub.computing_nodes[i]
            args = []
            for inp, kind in sub.input_specs[i]:
                if kind == 'value':
                    args.append(vals[inp])
                elif kind == 'shape':
                    sh = shapes.get(inp)
                    args.append(sh if sh is not None else _shape_of(vals[inp]))
                elif kind == 'aux':
                    args.append(aux[inp])
                elif kind == 'va':
                    args.append((vals[inp], aux[inp]))
            r = n.compute(args)
            if isinstance(r, AuxResult):
                aux[n] = r.aux
                r = r.value
            vals[n] = r
            if r is not None:
                shapes[n] = _shape_of(r)
            if hooks:
                for op, j in sub.grad_hooks.get(n, ()):
                    op.on_grad_ready(j, r)
            for dead in sub.release_after[i]:
                if dead in keep:        # a captured gradient whose hook runs after the replay
                    continue
                v = vals.pop(dead, None)
                if v is not None and dead not in shapes:
                    shapes[dead] = _shape_of(v)
                aux.pop(dead, None)

    def _capture(self, s, vals, aux, shapes):
        from .. import memory_pool as MP
        from .. import runtime as RT
        from . import hipgraph
        sub = self.sub
        dev = sub.config.device.index or 0
        from ..kernels.tensor import copy_into
        # static buffers of the volatile inputs (this step's values copied in)
        for n, kind in s.ext:
            v = aux[n] if kind == 'aux' else vals[n]
            st = copy_into(_NA.empty(tuple(v.shape), dtype=v.dtype, device=v.device), v)
            s.static[(n, kind)] = st
        local_vals, local_aux = dict(vals), dict(aux)
        for (n, kind), st in s.static.items():
            if kind == 'aux':
                local_aux[n] = st
            else:
                local_vals[n] = st
        cap = RT.DeviceStream(dev, persistent=True)
        cap.wait_stream(None)
        g = RT.Graph()
        s.pool = MP.capture_pool(dev, cap)
        try:
            with hipgraph.no_gc(), s.pool, RT.use_stream(cap):
                g.begin(cap)
                hipgraph._CAPTURING[0] += 1
                try:
                    self._run_ops(s.lo, s.hi, local_vals, local_aux, shapes, hooks=False, keep=set(s.hooked))
                finally:
                    hipgraph._CAPTURING[0] -= 1
                    g.end(cap)
        except Exception as e:   # noqa: BLE001 -- an op that cannot be captured
            raise _Fallback('capture of ops %d..%d failed (%s: %s)' % (s.lo, s.hi, type(e).__name__, e),
                            self._finish_eager(s, vals, aux, shapes))
        s.graph, s.stream = g, cap
        own = sub.computing_nodes[s.lo:s.hi]
        s.outputs = {n: local_vals[n] for n in own if n in local_vals}
        s.aux_out = {n: local_aux[n] for n in own if n in local_aux}
        s.shapes = {n: shapes[n] for n in own if n in shapes}


def _sig(vals, aux, n, kind):
    v = aux.get(n) if kind == 'aux' else vals.get(n)
    if not (isinstance(v, torch.Tensor) and v.is_cuda):
        return None
    return (tuple(v.shape), v.dtype)


class _Fallback(Exception):
    def __init__(self, why, vals):
        super().__init__(why)
        self.vals = vals
