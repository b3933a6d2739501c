"""Op and collective microbenchmarks (reference ``profiler.py:26-606``).

``HetuProfiler`` times each node of a SubExecutor on synthetic inputs (warm-up
5, timed 100, GPU events or CPU timer).  ``NCCLProfiler`` times RCCL collectives
(all-reduce / all-gather / reduce-scatter / broadcast / send-recv) over message
sizes and sub-groups; both feed the auto-parallel planner's cost model.
"""
from __future__ import annotations

import itertools
import json
import time

import numpy as np
import torch


def _timeit(fn, warmup=5, iters=100, gpu=True):
    for _ in range(warmup):
        fn()
    if gpu and torch.cuda.is_available():
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t) * 1000.0 / iters


class HetuProfiler(object):
    def __init__(self, subexecutor, feed_shapes, log_file=None, profiler='gpu', warmup=5, iters=100):
        self.sub = subexecutor
        self.feed_shapes = feed_shapes or {}
        self.log_file = log_file
        self.gpu = profiler == 'gpu'
        self.warmup, self.iters = warmup, iters

    def _synthetic(self, node, shape):
        dev = self.sub.config.device
        if getattr(node, 'is_embed_index', False) or 'id' in node.name.lower():
            # Zipf-distributed ids, like the reference's embedding sampler
            z = np.random.zipf(1.2, size=shape) % 1000
            return torch.from_numpy(z.astype(np.int64)).to(dev)
        return torch.randn(shape, device=dev)

    def run(self):
        sub = self.sub
        feed = {n: self._synthetic(n, s) for n, s in self.feed_shapes.items()}
        vals = sub._prepare_inputs(feed)
        results = {}
        aux = {}
        for i, n in enumerate(sub.computing_nodes):
            args = []
            ok = True
            for inp, kind in sub.input_specs[i]:
                if inp not in vals:
                    ok = False
                    break
                v = vals[inp]
                if kind == 'shape':
                    args.append(v.shape if hasattr(v, 'shape') else None)
                elif kind == 'aux':
                    args.append(aux.get(inp))
                elif kind == 'va':
                    args.append((v, aux.get(inp)))
                elif kind == 'value':
                    args.append(v)
            if not ok or type(n).__name__ == 'OptimizerOp':
                continue
            r = n.compute(args)
            from ..ops.nn import AuxResult
            if isinstance(r, AuxResult):
                aux[n] = r.aux
                r = r.value
            vals[n] = r
            results[n.name] = _timeit(lambda: n.compute(args), self.warmup, self.iters, self.gpu)
        if self.log_file:
            with open(self.log_file, 'w') as f:
                json.dump(results, f, indent=1)
        return results


class NCCLProfiler(object):
    """Collective timings over sub-groups of local GPUs (one process per GPU)."""

    def __init__(self, comm=None):
        from ..parallel import comm as C
        self.comm = comm or C.init_process_group()

    def profile_allreduce(self, size, groups=None, iters=20):
        from ..parallel import comm as C
        out = {}
        world = self.comm.nrank
        groups = groups or [tuple(range(world))]
        dev = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else 'cpu'
        for g in groups:
            c = C.new_group_comm(g)
            if self.comm.global_rank not in g:
                continue
            t = torch.ones(int(size), dtype=torch.float32, device=dev)
            out[g] = _timeit(lambda: c.all_reduce(t), 3, iters, torch.cuda.is_available())
        return out

    def profile_sendrecv(self, size, pairs=None, iters=20):
        dev = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else 'cpu'
        world = self.comm.nrank
        pairs = pairs or [(i, (i + 1) % world) for i in range(world)]
        t = torch.ones(int(size), dtype=torch.float32, device=dev)
        out = {}
        r = self.comm.rank
        for a, b in pairs:
            def f():
                if r == a:
                    self.comm.send(t, b).wait()
                elif r == b:
                    self.comm.recv(t, a).wait()
            out[(a, b)] = _timeit(f, 2, iters, torch.cuda.is_available())
        return out

    def bandwidth_sweep(self, sizes=(1 << 16, 1 << 20, 1 << 24, 1 << 26)):
        res = {}
        for s in sizes:
            ms = list(self.profile_allreduce(s).values())
            if ms:
                n = self.comm.nrank
                algbw = s * 4 / (ms[0] / 1000.0) / 1e9
                res[s] = dict(ms=ms[0], algbw_GBps=algbw, busbw_GBps=algbw * 2 * (n - 1) / n)
        return res
