"""Capture a SubExecutor step into a HIP graph and replay it.

Launch-bound steps (small MLPs, Wide&Deep at batch 128) spend most of their
time in host-side launch overhead; replaying a captured hipGraph removes the
per-op Python + launch cost.  Feeds and dataloader batches are copied into
static device buffers before each replay; per-step optimizer scalars (lr,
Adam bias corrections) live in a device tensor read by the fused update kernel
(``dyn``), so LR schedules keep working without re-capture.
"""
from __future__ import annotations

import atexit
import contextlib
import gc
import weakref

import torch
from .. import native_array as _NA

_CAPTURING = [0]
# host seed draws (kernels/rng.next_seed counts them): whether a captured step has random
# ops (reported; replay-safe through the device step counter)
_HOST_RANDOM = [0]
# >0: GraphRunner runs the next steps eagerly (a profiler census of the kernels a replayed
# step launches: a graph launch hides them from the activity trace)
FORCE_EAGER = [0]


def note_host_random():
    """called by every host seed draw (kernels/rng.py)"""
    _HOST_RANDOM[0] += 1


@contextlib.contextmanager
def no_gc():
    """Python's cycle collector stays off while a step is captured: a finaliser running
    inside the capture (a runner or pool of an earlier executor freeing device memory,
    destroying its graph, stream or events) invalidates it -- seen as hipError 901 at the
    next launch, depending on when the collector happened to run.  One collection first,
    outside the capture (torch.cuda.graph does the same)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def capturing():
    """True while a step is being captured into a graph (every capture of a framework step
    goes through GraphRunner, which counts it): ops that keep per-call host state (e.g.
    double-buffered BatchNorm totals flipped by a Python counter) must use a replay-safe
    form then -- a replay repeats the captured call, not the host logic around it"""
    return _CAPTURING[0] > 0


# live runners: their graphs are dropped at interpreter exit while the HIP runtime and
# torch's allocator are still up (a torch CUDAGraph collected during module teardown fails
# its destructor's HIP call and aborts the process after a clean run)
_RUNNERS = weakref.WeakSet()


def _close_all():
    runners = list(_RUNNERS)
    if not runners:
        return
    try:
        torch.cuda.synchronize()
    except Exception:       # noqa: BLE001
        pass
    for r in runners:
        try:
            r.close()
        except Exception:   # noqa: BLE001
            pass


atexit.register(_close_all)


class GraphRunner(object):
    def __init__(self, sub, warmup=3):
        _RUNNERS.add(self)
        self.sub = sub
        self.warmup = warmup
        self.calls = 0
        self.graph = None
        self.static_in = {}
        self.static_vals = None

    def close(self):
        """drop the graph, then its outputs, then the capture pool (the pool
        was never released; a pool still holding chunks the caller kept retires and goes
        back to the driver with its last free)"""
        self.graph = None
        self.static_vals = None
        pool, self.pool = getattr(self, 'pool', None), None
        if pool is not None:
            pool.release()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _inputs(self, feed_dict):
        sub = self.sub
        vals = {}
        for n, v in feed_dict.items():
            vals[n] = sub._feed_value(n, v)
        for d in sub.dataloader_nodes:
            vals[d] = d.get_arr(sub.name, sub.config)
        return vals

    def _update_dyn(self):
        for op in self.sub.opt_ops:
            opt = op.optimizer
            if getattr(op, 'dyn', None) is None:
                op.dyn = _NA.zeros(4, dtype=torch.float32, device=self.sub.config.device)
                op.dyn_host = _NA.zeros(4, dtype=torch.float32).pin_memory()
            step = op.step + 1
            h = opt.hyper(step)
            op.dyn_host[0] = h.get('lr', 0.0)
            op.dyn_host[1] = h.get('beta1t', 1.0)
            op.dyn_host[2] = h.get('beta2t', 1.0)
            op.dyn_host[3] = op.flat.gscale if op.flat is not None else 1.0
            op.dyn.copy_(op.dyn_host, non_blocking=True)

    def run(self, feed_dict, convert):
        sub = self.sub
        self.calls += 1
        self._update_dyn()
        if self.calls <= self.warmup or getattr(self, 'eager_only', False) or FORCE_EAGER[0]:
            vals = sub._run_eager(feed_dict)
            return sub._collect(vals, convert)
        new_in = self._inputs(feed_dict)
        sig = tuple(sorted((id(n), tuple(v.shape), str(v.dtype)) for n, v in new_in.items()))
        if self.graph is not None and sig != self.sig:
            # a feed changed shape or dtype: the captured graph's buffers no longer fit --
            # run this step eagerly and capture again once the new shapes have warmed up
            self.close()
            self.calls = 0
            self.static_in = {}
            base = {p: sub.config.compute_value(p) for p in sub.param_nodes}
            base.update(new_in)                 # this step's (already fetched) inputs
            vals = sub._run_eager(None, vals=base)
            return sub._collect(vals, convert)
        if self.graph is None:
            self.sig = sig
            r0 = _HOST_RANDOM[0]
            # static input buffers
            for n, v in new_in.items():
                self.static_in[n] = v.clone()
            base = {p: sub.config.compute_value(p) for p in sub.param_nodes}
            base.update(self.static_in)
            torch.cuda.synchronize()
            from .. import memory_pool as MP
            steps0 = [op.step for op in sub.opt_ops]
            try:
                if MP.torch_bfc_enabled():
                    self._capture_native(sub, base)
                else:
                    self._capture_torch(sub, base)
            except Exception as e:          # noqa: BLE001 -- an op that cannot be captured
                import sys
                print('hipgraph: capture failed (%s: %s); running this executor eagerly'
                      % (type(e).__name__, e), file=sys.stderr)
                self.close()
                self.eager_only = True
                torch.cuda.synchronize()
                for op, st in zip(sub.opt_ops, steps0):
                    op.step = st            # the failed capture executed nothing
                base = {p: sub.config.compute_value(p) for p in sub.param_nodes}
                base.update(new_in)
                vals = sub._run_eager(None, vals=base)
                return sub._collect(vals, convert)
            for op in sub.opt_ops:
                op.step -= 1  # the capture itself executes nothing
            # (random ops are replay-safe: their host seeds are fixed per op and call, and
            # the captured rng_advance kernel moves the device step counter every replay --
            # kernels/rng.py)
            self.random_ops = _HOST_RANDOM[0] != r0
        for n, v in new_in.items():
            self.static_in[n].copy_(v, non_blocking=True)
        self.graph.replay()
        for op in sub.opt_ops:
            op.step += 1
        return self._collect_outputs(convert)

    def _collect_outputs(self, convert):
        """outputs of the replayed step: the graph's static buffers are overwritten by the
        next replay, so unconverted device outputs are handed out as copies (native copy
        kernel), never as aliases"""
        if convert:
            return self.sub._collect(self.static_vals, True)
        from ..kernels.tensor import copy_into
        vals = {}
        for n in self.sub.eval_node_list:
            v = self.static_vals.get(n)
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v = copy_into(_NA.empty(tuple(v.shape), dtype=v.dtype, device=v.device), v)
            vals[n] = v
        return self.sub._collect(vals, False)

    def _capture_torch(self, sub, base):
        """capture through torch's graph API (torch's caching allocator owns device memory)"""
        from .. import runtime as RT
        self.graph = torch.cuda.CUDAGraph()
        cap = self.capture_stream = RT.DeviceStream(persistent=True)
        _CAPTURING[0] += 1
        try:
            # torch captures on `cap`; the framework's launches follow it there.  use_stream
            # is the OUTER context: on exit it restores torch's stream to the framework's
            # previous one, which must happen after the graph's capture_end ran on `cap`
            with no_gc(), RT.use_stream(cap), torch.cuda.graph(self.graph, stream=cap.torch):
                self.static_vals = sub._run_eager(None, vals=dict(base))
        finally:
            _CAPTURING[0] -= 1

    def _capture_native(self, sub, base):
        """Capture on a framework stream into a native HIP graph, every allocation of
        the captured step carved from a private BFC pool (torch's graph pools need its
        caching allocator, which the BFC pool replaces)."""
        from .. import memory_pool as MP
        from .. import runtime as RT
        dev = sub.config.device.index or 0
        cap = RT.DeviceStream(dev, persistent=True)
        cap.wait_stream(None)                 # after the work queued on the current stream
        g = RT.Graph()
        self.pool = MP.capture_pool(dev, cap)
        with no_gc(), self.pool, RT.use_stream(cap):
            g.begin(cap)
            _CAPTURING[0] += 1
            try:
                self.static_vals = sub._run_eager(None, vals=dict(base))
            finally:
                _CAPTURING[0] -= 1
                g.end(cap)
        self.capture_stream = cap
        self.graph = _NativeReplay(g)


class _NativeReplay(object):
    """replay() on torch's current stream, like torch.cuda.CUDAGraph"""

    def __init__(self, g):
        self.g = g

    def replay(self):
        from .._base import cur_stream
        self.g.replay(cur_stream())
