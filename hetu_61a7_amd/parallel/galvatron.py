"""Galvatron-style automatic parallelism planner (SURVEY §2.3 S15, §7.1
"Auto-parallel"; the reference ships only ``tools/Galvatron/README.md:1-2``).

Given a layer-wise cost description of a model and a single MI355X node, the
planner searches hybrid strategies and returns the fastest one that fits the
HBM budget:

* pipeline degree ``pp`` (a divisor of the GPU count) with a contiguous layer
  partition into stages (balanced by a min-max dynamic program over layer
  times),
* inside every stage, per layer, a (tensor-parallel ``tp``, data-parallel
  ``dp``) split with ``tp * dp = gpus / pp``, chosen by a dynamic program over
  the layer sequence whose state is the previous layer's ``tp`` (re-sharding
  between different ``tp`` costs an all-gather) under the per-GPU memory cap,
* the number of micro-batches.

Cost model (per training step, seconds), all terms for ONE GPU:
  compute     3 * fwd_flops * batch_per_replica / (tp * flops)          (fwd + 2x bwd)
  tp comm     4 all-reduces of the layer output per micro-batch (Megatron
              column/row pairs: 2 fwd, 2 bwd), ring over ``tp`` GPUs
  dp comm     gradient all-reduce of the layer's params / tp over ``dp``
              replicas, partially hidden behind backward (``overlap``)
  pp          GPipe bubble: (m + pp - 1) * slowest stage micro-batch time,
              plus the stage-boundary activation send/recv per micro-batch
  memory      params+grads+optimizer state (16 B/param for Adam mixed
              precision: bf16 param/grad + fp32 master/m/v) / tp, plus stored
              activations (act_bytes per sample / tp) x in-flight micro-batches
Link model: xGMI full mesh, 7 links x ~153 GB/s per GPU.  A collective over
``p`` GPUs of one node can drive ``min(p - 1, 7)`` links (RCCL rings/channels
over distinct peers), so its bus bandwidth is ``min(p-1, 7) * link_bw * eff``.

The plan is emitted as RCCL-only schedules: ``Plan.stage_devices()`` gives the
``ht.context`` device group of every pipeline stage (DP inside a stage is the
bucketed RCCL all-reduce of the pipeline executor), ``Plan.tp_groups`` the
tensor-parallel rank groups for the dispatch lowering.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class LayerSpec:
    """Per-layer costs for ONE sample (forward only; the model multiplies)."""
    name: str
    fwd_flops: float           # forward FLOPs per sample
    params: float              # parameter count
    act_bytes: float           # activation bytes kept for backward, per sample
    out_bytes: float           # bytes of the layer output per sample (PP / TP traffic)
    tp_able: bool = True       # can be Megatron-split


@dataclass
class Hardware:
    """One MI355X node.  ``flops`` is the achieved (not peak) bf16 matmul rate."""
    gpus: int = 8
    flops: float = 9.0e14
    hbm_bytes: float = 288e9
    link_bw: float = 153e9
    links: int = 7
    eff: float = 0.8
    latency: float = 8e-6

    def bus_bw(self, p):
        return max(1, min(p - 1, self.links)) * self.link_bw * self.eff

    def allreduce(self, nbytes, p):
        if p <= 1 or nbytes <= 0:
            return 0.0
        return 2.0 * (p - 1) / p * nbytes / self.bus_bw(p) + 2 * (p - 1) * self.latency

    def allgather(self, nbytes, p):
        if p <= 1 or nbytes <= 0:
            return 0.0
        return (p - 1) / p * nbytes / self.bus_bw(p) + (p - 1) * self.latency

    def p2p(self, nbytes):
        return nbytes / (self.link_bw * self.eff) + self.latency

    @classmethod
    def calibrate(cls, gpus=None, gemm=(8192, 3072, 768), comm=None, sizes=(1 << 22, 1 << 24), **kw):
        """Profile-driven hardware model: the achieved bf16 GEMM rate of this
        device (a transformer-sized matmul, the HetuProfiler role) and, when a
        multi-rank communicator is given, the measured all-reduce bus bandwidth
        (NCCLProfiler.bandwidth_sweep) replacing the xGMI link defaults."""
        import time
        import torch
        hw = cls(gpus=gpus or (comm.nrank if comm is not None else 1), **kw)
        M, N, K = gemm
        dev = 'cuda' if torch.cuda.is_available() else 'cpu'
        dt = torch.bfloat16 if dev == 'cuda' else torch.float32
        a = torch.randn(M, K, device=dev).to(dt)
        b = torch.randn(K, N, device=dev).to(dt)
        for _ in range(3):
            a @ b
        if dev == 'cuda':
            torch.cuda.synchronize()
        it = 20 if dev == 'cuda' else 2
        t0 = time.perf_counter()
        for _ in range(it):
            a @ b
        if dev == 'cuda':
            torch.cuda.synchronize()
        hw.flops = 2.0 * M * N * K * it / (time.perf_counter() - t0)
        if comm is not None and comm.nrank > 1:
            from ..utils.profiler import NCCLProfiler
            sweep = NCCLProfiler(comm).bandwidth_sweep(sizes)
            if sweep:
                busbw = max(v['busbw_GBps'] for v in sweep.values()) * 1e9
                hw.link_bw = busbw / max(1, min(comm.nrank - 1, hw.links))
                hw.eff = 1.0
        return hw


@dataclass
class Plan:
    pp: int
    stages: List[Tuple[int, int]]          # [start, end) layer index per stage
    tp: List[int]                          # per layer
    dp: List[int]                          # per layer
    micro_batches: int
    global_batch: int
    time: float                            # estimated step seconds
    memory: List[float]                    # estimated bytes per GPU per stage
    gpus: int
    detail: Dict[str, float] = field(default_factory=dict)

    @property
    def throughput(self):
        return self.global_batch / self.time if self.time > 0 else 0.0

    def stage_ranks(self, s):
        per = self.gpus // self.pp
        return list(range(s * per, (s + 1) * per))

    def stage_devices(self, s):
        """Device group for ``ht.context`` of stage ``s`` (one process per GPU)."""
        from .. import ndarray
        return [ndarray.gpu(r) for r in self.stage_ranks(s)]

    def tp_groups(self, layer):
        """Rank groups of size tp (consecutive ranks: the xGMI peers) for a layer."""
        s = next(i for i, (a, b) in enumerate(self.stages) if a <= layer < b)
        ranks = self.stage_ranks(s)
        t = self.tp[layer]
        return [ranks[i:i + t] for i in range(0, len(ranks), t)]

    def short(self):
        tps = sorted(set(self.tp))
        return 'pp%d tp%s mb%d' % (self.pp, '/'.join(map(str, tps)), self.micro_batches)

    def describe(self):
        lines = ['pp=%d micro_batches=%d est %.2f ms/step, %.1f samples/s' %
                 (self.pp, self.micro_batches, self.time * 1e3, self.throughput)]
        for s, (a, b) in enumerate(self.stages):
            tps = sorted(set(self.tp[a:b]))
            lines.append('  stage %d: layers [%d, %d) gpus %s tp %s mem %.1f GB' %
                         (s, a, b, self.stage_ranks(s), tps, self.memory[s] / 1e9))
        return '\n'.join(lines)


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def _pareto(points):
    """Non-dominated (time, memory, choice) points, sorted by memory."""
    points.sort(key=lambda p: (p[1], p[0]))
    out, best_t = [], float('inf')
    for p in points:
        if p[0] < best_t:
            out.append(p)
            best_t = p[0]
    return out


class GalvatronPlanner(object):
    def __init__(self, layers: Sequence[LayerSpec], hw: Optional[Hardware] = None,
                 bytes_per_param: float = 16.0, overlap: float = 0.7, max_tp: Optional[int] = None,
                 mem_fraction: float = 0.9):
        self.layers = list(layers)
        self.hw = hw or Hardware()
        self.bpp = bytes_per_param
        self.overlap = overlap
        self.max_tp = max_tp or self.hw.gpus
        self.mem_cap = self.hw.hbm_bytes * mem_fraction

    # ---- per-layer terms ------------------------------------------------------------
    def layer_time(self, L: LayerSpec, tp, dp, batch_per_replica, m):
        hw = self.hw
        comp = 3.0 * L.fwd_flops * batch_per_replica / (tp * hw.flops)
        mb = batch_per_replica / m
        tpc = 4 * m * hw.allreduce(L.out_bytes * mb, tp) if tp > 1 else 0.0
        dpc = hw.allreduce(2.0 * L.params / tp, dp)   # bf16 gradients
        return comp + tpc + (1.0 - self.overlap) * dpc, comp, tpc, dpc

    def layer_mem(self, L, tp, batch_per_replica, m, inflight):
        mb = batch_per_replica / m
        return self.bpp * L.params / tp + L.act_bytes * mb * inflight / tp

    # ---- within-stage (tp, dp) choice: DP over layers --------------------------------
    # State = the previous layer's tp (re-sharding between different tp layouts costs
    # an all-gather); per state the DP keeps the Pareto front of (time, memory), so the
    # memory cap is handled exactly (a min-time-only state would prune the feasible
    # low-memory prefixes Galvatron's memory-budget dimension keeps).
    def _stage_opt(self, lo, hi, n, batch, m, inflight):
        hw = self.hw
        opts = [t for t in _divisors(n) if t <= self.max_tp]
        fronts = {None: [(0.0, 0.0, ())]}
        for li in range(lo, hi):
            L = self.layers[li]
            nxt = {}
            for t in opts:
                if t > 1 and not L.tp_able:
                    continue
                dp = n // t
                bpr = batch / dp
                lt = self.layer_time(L, t, dp, bpr, m)[0]
                lm = self.layer_mem(L, t, bpr, m, inflight)
                cand = []
                for pt, front in fronts.items():
                    trans = 0.0
                    if pt is not None and pt != t:
                        trans = 2 * m * hw.allgather(L.out_bytes * bpr / m, max(pt, t))
                    for ptime, pmem, ch in front:
                        mem = pmem + lm
                        if mem <= self.mem_cap:
                            cand.append((ptime + lt + trans, mem, ch + (t,)))
                if cand:
                    nxt[t] = _pareto(cand)
            if not nxt:
                return None
            fronts = nxt
        t, mem, ch = min((p for f in fronts.values() for p in f), key=lambda v: (v[0], v[1]))
        return t, mem, list(ch)

    # ---- balanced contiguous partition for pp stages (min-max DP) ----------------------
    def _partition(self, pp, weights):
        n = len(weights)
        pre = [0.0]
        for w in weights:
            pre.append(pre[-1] + w)
        INF = float('inf')
        dp = [[INF] * (n + 1) for _ in range(pp + 1)]
        cut = [[0] * (n + 1) for _ in range(pp + 1)]
        dp[0][0] = 0.0
        for s in range(1, pp + 1):
            for j in range(s, n + 1):
                for i in range(s - 1, j):
                    v = max(dp[s - 1][i], pre[j] - pre[i])
                    if v < dp[s][j]:
                        dp[s][j], cut[s][j] = v, i
        bounds, j = [], n
        for s in range(pp, 0, -1):
            i = cut[s][j]
            bounds.append((i, j))
            j = i
        return bounds[::-1]

    # ---- search -------------------------------------------------------------------------
    def search(self, global_batch: int, micro_batches: Sequence[int] = (1, 2, 4, 8, 16, 32),
               pp_options: Optional[Sequence[int]] = None, schedule: str = 'gpipe') -> Plan:
        hw = self.hw
        N = hw.gpus
        best: Optional[Plan] = None
        for pp in (pp_options or _divisors(N)):
            if pp > len(self.layers) or N % pp:
                continue
            n = N // pp
            base_w = [3.0 * L.fwd_flops for L in self.layers]
            bounds = self._partition(pp, base_w)
            for m in micro_batches:
                if pp == 1 and m > 1:
                    continue
                if global_batch % m or (global_batch // n) % m:
                    continue       # every data-parallel replica's batch splits into m micro-batches
                stage_time, stage_mem, tps, dps = [], [], [], []
                ok = True
                for s, (a, b) in enumerate(bounds):
                    # micro-batches in flight on stage s: all m (GPipe), pp - s (1F1B)
                    inflight = m if schedule == 'gpipe' else min(m, pp - s)
                    r = self._stage_opt(a, b, n, global_batch, m, inflight)
                    if r is None:
                        ok = False
                        break
                    t, mem, ch = r
                    stage_time.append(t)
                    stage_mem.append(mem)
                    tps += ch
                    dps += [n // x for x in ch]
                if not ok:
                    continue
                # pipeline: per-micro-batch stage time, bubble, boundary p2p
                per_mb = [t / m for t in stage_time]
                p2p = 0.0
                for s in range(pp - 1):
                    L = self.layers[bounds[s][1] - 1]
                    p2p = max(p2p, 2 * hw.p2p(L.out_bytes * global_batch / (n * m)))
                step = (m + pp - 1) * (max(per_mb) + p2p) if pp > 1 else stage_time[0]
                plan = Plan(pp, bounds, tps, dps, m, global_batch, step, stage_mem, N,
                            detail={'bubble_frac': (pp - 1) / (m + pp - 1) if pp > 1 else 0.0})
                if best is None or plan.time < best.time:
                    best = plan
        if best is None:
            raise RuntimeError('no parallel strategy fits %.0f GB per GPU' % (self.mem_cap / 1e9))
        return best

    def brute_force(self, global_batch, pp, m, schedule='gpipe'):
        """Exhaustive per-layer tp search for one (pp, m) -- test oracle for the DP."""
        N = self.hw.gpus
        n = N // pp
        bounds = self._partition(pp, [3.0 * L.fwd_flops for L in self.layers])
        total_best = 0.0
        for s, (a, b) in enumerate(bounds):
            inflight = m if schedule == 'gpipe' else min(m, pp - s)
            opts = [t for t in _divisors(n) if t <= self.max_tp]
            best = None
            for combo in itertools.product(opts, repeat=b - a):
                tot = mem = 0.0
                prev = None
                valid = True
                for li, t in zip(range(a, b), combo):
                    L = self.layers[li]
                    if t > 1 and not L.tp_able:
                        valid = False
                        break
                    bpr = global_batch / (n // t)
                    tot += self.layer_time(L, t, n // t, bpr, m)[0]
                    mem += self.layer_mem(L, t, bpr, m, inflight)
                    if prev is not None and prev != t:
                        tot += 2 * m * self.hw.allgather(L.out_bytes * bpr / m, max(prev, t))
                    prev = t
                if valid and mem <= self.mem_cap and (best is None or tot < best):
                    best = tot
            if best is None:
                return None
            total_best = max(total_best, best) if pp > 1 else best
        return total_best


# ---------------------------------------------------------------------------------------
# model descriptions
def bert_layers(hidden=768, layers=12, seq_len=128, vocab=30522, intermediate=None,
                dtype_bytes=2) -> List[LayerSpec]:
    """Analytic per-sample costs of BERT (embeddings, encoder layers, MLM/NSP head)."""
    H, S = hidden, seq_len
    I = intermediate or 4 * H
    out = []
    out.append(LayerSpec('embeddings', fwd_flops=2 * S * H, params=(vocab + 512 + 2) * H + 2 * H,
                         act_bytes=S * H * dtype_bytes * 2, out_bytes=S * H * dtype_bytes, tp_able=False))
    for i in range(layers):
        flops = 2 * S * (4 * H * H + 2 * H * I) + 4 * S * S * H
        params = 4 * H * H + 2 * H * I + 9 * H + I
        act = S * (16 * H + 2 * I) * dtype_bytes + 2 * S * S * (H // 64) * dtype_bytes
        out.append(LayerSpec('encoder%d' % i, flops, params, act, S * H * dtype_bytes))
    out.append(LayerSpec('mlm_head', fwd_flops=2 * S * (H * H + H * vocab), params=H * H + 3 * H + vocab,
                         act_bytes=S * (2 * H + 2 * vocab) * dtype_bytes, out_bytes=4, tp_able=True))
    return out


def plan_bert(global_batch=64, hidden=768, layers=12, seq_len=128, hw=None, **kw) -> Plan:
    return GalvatronPlanner(bert_layers(hidden, layers, seq_len), hw=hw, **kw).search(global_batch)
