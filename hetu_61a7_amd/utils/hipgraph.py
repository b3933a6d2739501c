"""Capture a SubExecutor step into a HIP graph and replay it.

Launch-bound steps (small MLPs, Wide&Deep at batch 128) spend most of their
time in host-side launch overhead; replaying a captured hipGraph removes the
per-op Python + launch cost.  Feeds and dataloader batches are copied into
static device buffers before each replay; per-step optimizer scalars (lr,
Adam bias corrections) live in a device tensor read by the fused update kernel
(``dyn``), so LR schedules keep working without re-capture.
"""
from __future__ import annotations

import torch
from .. import native_array as _NA

_CAPTURING = [0]
# per-call host random draws (dropout seeds, attention dropout counters): a captured graph
# would replay the draws of the capture step forever -- the same dropout masks every step
_HOST_RANDOM = [0]


def note_host_random():
    """called by every op that draws a host-side seed for its kernel launch"""
    _HOST_RANDOM[0] += 1


def capturing():
    """True while a step is being captured into a graph (framework capture or torch's):
    ops that keep per-call host state (e.g. double-buffered BatchNorm totals flipped by
    a Python counter) must use a replay-safe form then -- a replay repeats the captured
    call, not the host logic around it"""
    if _CAPTURING[0]:
        return True
    try:
        return bool(torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
    except RuntimeError:
        return False


class GraphRunner(object):
    def __init__(self, sub, warmup=3):
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
        if self.calls <= self.warmup or getattr(self, 'eager_only', False):
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
            if MP.torch_bfc_enabled():
                self._capture_native(sub, base)
            else:
                self.graph = torch.cuda.CUDAGraph()
                _CAPTURING[0] += 1
                try:
                    with torch.cuda.graph(self.graph):
                        self.static_vals = sub._run_eager(None, vals=dict(base))
                finally:
                    _CAPTURING[0] -= 1
            for op in sub.opt_ops:
                op.step -= 1  # the capture itself executes nothing
            if _HOST_RANDOM[0] != r0:
                # the step draws host seeds (dropout): a replay would repeat this step's masks
                # forever -- keep running eagerly (correct randomness beats the launch savings)
                import sys
                print('hipgraph: step draws host-side random seeds (dropout); running eagerly instead',
                      file=sys.stderr)
                self.close()
                self.eager_only = True
                base = {p: sub.config.compute_value(p) for p in sub.param_nodes}
                base.update(new_in)
                vals = sub._run_eager(None, vals=base)
                return sub._collect(vals, convert)
        for n, v in new_in.items():
            self.static_in[n].copy_(v, non_blocking=True)
        self.graph.replay()
        for op in sub.opt_ops:
            op.step += 1
        return sub._collect(self.static_vals, convert)

    def _capture_native(self, sub, base):
        """Capture on a framework stream into a native HIP graph, every allocation of
        the captured step carved from a private BFC pool (torch's graph pools need its
        caching allocator, which the BFC pool replaces)."""
        from .. import memory_pool as MP
        from .. import runtime as RT
        dev = sub.config.device.index or 0
        cap = RT.DeviceStream(dev, persistent=True)
        cap.wait_stream(torch.cuda.current_stream())
        g = RT.Graph()
        self.pool = MP.capture_pool(dev, cap)
        with self.pool, torch.cuda.stream(cap.torch):
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
        self.g.replay(torch.cuda.current_stream())
