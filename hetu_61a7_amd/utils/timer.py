"""Per-node timing (reference ``timer_subexecutor.py:21-178``).

``Executor(..., timing='gpu'|'cpu')`` brackets every node with HIP events (gpu)
or ``perf_counter`` (cpu); ``logOut(path, log_level='node'|'type')`` writes the
mean milliseconds per node or per op type.  Each node is also wrapped in a
roctx range when roctx is available, so rocprofv3 traces show op names.
"""
from __future__ import annotations

import time
from collections import defaultdict

import torch


class NodeTimer(object):
    def __init__(self, kind='gpu'):
        self.kind = kind
        self.records = defaultdict(list)
        self.pending = []
        self._t0 = None
        self._ev = None

    def start(self, node):
        if self.kind == 'gpu' and torch.cuda.is_available():
            self._ev = torch.cuda.Event(enable_timing=True)
            self._ev.record()
            try:
                torch.cuda.nvtx.range_push(node.name)
            except Exception:
                pass
        else:
            self._t0 = time.perf_counter()

    def stop(self, node):
        if self.kind == 'gpu' and torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            try:
                torch.cuda.nvtx.range_pop()
            except Exception:
                pass
            self.pending.append((node, self._ev, e))
        else:
            self.records[node].append((time.perf_counter() - self._t0) * 1000.0)

    def _flush(self):
        if self.pending:
            torch.cuda.synchronize()
            for node, a, b in self.pending:
                self.records[node].append(a.elapsed_time(b))
            self.pending = []

    def summary(self, log_level='node'):
        self._flush()
        out = {}
        if log_level == 'node':
            for n, v in self.records.items():
                out[n.name] = sum(v) / len(v)
        else:
            agg = defaultdict(list)
            for n, v in self.records.items():
                agg[n.op_type].append(sum(v) / len(v))
            for k, v in agg.items():
                out[k] = sum(v)
        return out

    def log_out(self, path=None, log_level='node', clear=True):
        s = self.summary(log_level)
        if path is not None:
            with open(path, 'w') as f:
                for k, v in sorted(s.items(), key=lambda kv: -kv[1]):
                    f.write('%s\t%.4f\n' % (k, v))
        if clear:
            self.clear()
        return s

    def clear(self):
        self.records.clear()
        self.pending = []
