"""Per-node timing (reference ``timer_subexecutor.py:21-178``).

``Executor(..., timing='gpu'|'cpu')`` brackets every node with HIP events (gpu)
or ``perf_counter`` (cpu); ``logOut(path, log_level='node'|'type')`` writes the
mean milliseconds per node or per op type.  Each node is also wrapped in a
roctx range when roctx is available, so rocprofv3 traces show op names, and
``export_chrome_trace(path)`` writes every timed node as a Chrome / Perfetto
trace event (chrome://tracing, ui.perfetto.dev).
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
        self._base = None          # first event / time: trace origin
        self.trace = []            # (name, op_type, start_ms, dur_ms)

    def start(self, node):
        if self.kind == 'gpu' and torch.cuda.is_available():
            self._ev = torch.cuda.Event(enable_timing=True)
            self._ev.record()
            if self._base is None:
                self._base = self._ev
            try:
                torch.cuda.nvtx.range_push(node.name)
            except Exception:
                pass
        else:
            self._t0 = time.perf_counter()
            if self._base is None:
                self._base = self._t0

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
            t1 = time.perf_counter()
            self.records[node].append((t1 - self._t0) * 1000.0)
            self.trace.append((node.name, type(node).__name__, (self._t0 - self._base) * 1e3, (t1 - self._t0) * 1e3))

    def _flush(self):
        if self.pending:
            torch.cuda.synchronize()
            for node, a, b in self.pending:
                d = a.elapsed_time(b)
                self.records[node].append(d)
                self.trace.append((node.name, type(node).__name__, self._base.elapsed_time(a), d))
            self.pending = []

    def export_chrome_trace(self, path, pid=0):
        """Chrome trace-event JSON of every timed node (microseconds)."""
        import json
        self._flush()
        ev = [{'name': n, 'cat': t, 'ph': 'X', 'ts': round(s * 1e3, 3), 'dur': round(d * 1e3, 3), 'pid': pid,
               'tid': 0, 'args': {'op_type': t}} for n, t, s, d in self.trace]
        with open(path, 'w') as f:
            json.dump({'traceEvents': ev, 'displayTimeUnit': 'ms'}, f)
        return len(ev)

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
        self.trace = []
        self._base = None
