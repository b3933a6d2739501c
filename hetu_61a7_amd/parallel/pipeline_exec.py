"""Pipeline-parallel sub-executors: GPipe, PipeDream (1F1B) and HetPipe.

Reference: ``pipeline_subexecutor.py:13-130`` (stage partition),
``gpipe_subexecutor.py:8-123`` (all forwards, then all backwards, one update),
``pipedream_subexecutor.py:25-48`` (1F1B generator) and ``:51-372``,
HetPipe = PipeDream + PS-held weights (``:77-83,149-176``); SURVEY §2.3 S6-S8.

MI355X design
-------------
* One process per GPU.  A *stage* is the device set of a ``with
  ht.context(...)`` block; a stage with several devices is data-parallel
  inside (replica ``r`` of stage ``s`` talks to replica ``r`` of stage
  ``s+1``), and its parameter gradients are all-reduced over the replica
  group with the same bucketed RCCL path as plain DP.
* Partitioning is automatic: forward nodes go to their context's stage, every
  node created while differentiating forward node X goes to X's stage (the
  ``bw_of`` tag written by ``gradients``), and every cross-stage edge becomes
  one point-to-point message (RCCL send/recv over xGMI; gloo on CPU).  Sends
  are asynchronous, receives block, so any schedule in which each stage
  processes micro-batches in the same order is deadlock-free.
* Schedules: ``gpipe`` (F0..Fm-1, B0..Bm-1), ``pipedream`` (1F1B: warm-up of
  ``stages - s - 1`` forwards then alternate, cooldown), ``pipedream_flush``
  (the same order, gradients accumulated and applied once per step) and
  ``hetpipe`` (1F1B plus a PS sync of the stage's dense parameters each step).
* ``pipedream`` is asynchronous PipeDream with weight stashing: every micro-batch
  snapshots the stage's current weights at its forward, its backward runs
  against that snapshot, and its gradient is applied to the latest weights
  right after the backward (reference ``pipedream_subexecutor.py:90-147``).
  GPipe / PipeDream-flush / HetPipe accumulate over the micro-batches of a step
  and apply once (pipeline flush), the step semantics of the unpipelined model.
"""
from __future__ import annotations

import os
from typing import Dict, List

import numpy as np

import torch
import torch.distributed as dist

from .. import ndarray
from ..ps import PS_KEY_HETPIPE_STAGE
from ..ops.node import Op
from ..ops.variable import PlaceholderOp
from ..ops.executor import find_topo_sort, AuxResult, _shape_of

_DT = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16, 3: torch.int64, 4: torch.int32}
_DT_INV = {v: k for k, v in _DT.items()}
HDR = 10


def _dev_key(ctx):
    if isinstance(ctx, ndarray.DLContext):
        return (ctx.hostname, 'gpu' if ndarray.is_gpu_ctx(ctx) else 'cpu', ctx.device_id)
    return ctx


def _group_key(raw_ctx):
    if raw_ctx is None:
        return None
    return tuple(_dev_key(d) for d in raw_ctx.all_devices())


class _P2P(object):
    """Point-to-point tensor messages between pipeline stages (RCCL send/recv over xGMI
    through ``Communicator``; gloo on CPU).

    Shape protocol (reference executor.py:774-833 exchanges shapes once per
    (re)allocation): the first message of each key (a cross-stage edge) in a step
    carries a small header (ndim, dtype, shape); the receiver reads it -- the one host
    synchronisation -- and caches it, and every later micro-batch of the step sends the
    payload alone, received into a buffer of the cached shape.  All payload sends of a
    phase go out as one RCCL group (batch_isend_irecv), so do all payload receives whose
    shapes are known.  ``hdr_syncs`` counts the header reads (tests).

    The protocol is symmetric by construction: with static shapes (default) the
    sender raises if a later micro-batch of a key changes shape within a step (the
    receiver would post a payload recv of the stale shape); ``dynamic=True``
    (``HETU_PP_DYNAMIC_SHAPES=1``: short last micro-batches, variable sequence
    lengths) sends and reads a header with every message."""

    def __init__(self, device, comm=None, dynamic=None):
        self.device = device
        self.comm = comm
        self.pending = []
        self.shapes = {}        # key -> (shape, dtype) known for this step
        self.hdr_syncs = 0
        if dynamic is None:
            dynamic = os.environ.get('HETU_PP_DYNAMIC_SHAPES', '0') == '1'
        self.dynamic = dynamic

    def new_step(self):
        self.shapes = {}

    def _batch(self, ops):
        if self.comm is not None:
            return self.comm.batch_p2p(ops)
        return dist.batch_isend_irecv([dist.P2POp(dist.isend if k == 'send' else dist.irecv, t, p)
                                       for k, t, p in ops]) if ops else []

    def send_many(self, items):
        """items: [(key, tensor, dst)] -- one group (plus headers of new keys)."""
        hdrs, ops = [], []
        for key, t, dst in items:
            t = t.contiguous()
            sig = (tuple(t.shape), t.dtype)
            if not self.dynamic and key in self.shapes and self.shapes[key] != sig:
                raise ValueError('pipeline edge %r changed shape within a step (%s -> %s): the receiver '
                                 'cached the first shape; set HETU_PP_DYNAMIC_SHAPES=1 (a header per '
                                 'message) for variable micro-batch shapes' % (key, self.shapes[key], sig))
            if self.dynamic or key not in self.shapes:
                hdr = torch.zeros(HDR, dtype=torch.int64)
                hdr[0] = t.dim()
                hdr[1] = _DT_INV[t.dtype]
                hdr[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
                hdr = hdr.to(t.device)
                hdrs.append(('send', hdr, dst))
                self.shapes[key] = (tuple(t.shape), t.dtype)
            ops.append(('send', t, dst))
        for w in self._batch(hdrs):
            self.pending.append((w, hdrs))
        for w in self._batch(ops):
            self.pending.append((w, ops))

    def recv_many(self, items):
        """items: [(key, src)] -> tensors in the same order."""
        out = [None] * len(items)
        hdr_ops, need = [], []
        for j, (key, src) in enumerate(items):
            if self.dynamic or key not in self.shapes:
                hdr = torch.zeros(HDR, dtype=torch.int64, device=self.device)
                hdr_ops.append(('recv', hdr, src))
                need.append((j, key, hdr))
        if hdr_ops:
            for w in self._batch(hdr_ops):
                w.wait()
            for j, key, hdr in need:
                h = hdr.tolist()          # the host sync, once per key per step
                self.hdr_syncs += 1
                nd = int(h[0])
                self.shapes[key] = (tuple(int(x) for x in h[2:2 + nd]), _DT[int(h[1])])
        ops = []
        for j, (key, src) in enumerate(items):
            shape, dt = self.shapes[key]
            out[j] = torch.empty(shape, dtype=dt, device=self.device)
            ops.append(('recv', out[j], src))
        for w in self._batch(ops):
            w.wait()
        return out

    def flush(self):
        for w, _ in self.pending:
            w.wait()
        self.pending = []


def pipedream_schedule(stage, nstages, m):
    """1F1B order for one stage: list of ('F'|'B', micro-batch)."""
    warm = min(nstages - stage - 1, m)
    order = [('F', i) for i in range(warm)]
    f, b = warm, 0
    while b < m:
        if f < m:
            order.append(('F', f))
            f += 1
        order.append(('B', b))
        b += 1
    return order


def gpipe_schedule(stage, nstages, m):
    return [('F', i) for i in range(m)] + [('B', i) for i in range(m)]


class PipelineSubExecutor(object):
    def __init__(self, kind, name, eval_node_list, config):
        from ..optimizer import OptimizerOp
        assert kind in ('gpipe', 'pipedream', 'pipedream_flush', 'hetpipe'), kind
        self.kind, self.name, self.config = kind, name, config
        self.eval_node_list = list(eval_node_list)
        topo = find_topo_sort(self.eval_node_list)
        self.opt_nodes = [n for n in topo if isinstance(n, OptimizerOp)]
        self.inference = not self.opt_nodes

        # ---- stages ----------------------------------------------------------------------
        order = []
        for n in topo:
            if isinstance(n, OptimizerOp) or getattr(n, 'bw_of', None) is not None:
                continue
            k = _group_key(n.raw_ctx)
            if k is not None and k not in order:
                order.append(k)
        assert order, 'pipeline needs nodes placed with ht.context(...)'
        self.stage_keys = order
        self.nstages = len(order)
        stage_of: Dict[Op, int] = {}
        for n in topo:
            if isinstance(n, OptimizerOp):
                continue
            origin = getattr(n, 'bw_of', None)
            while origin is not None and getattr(origin, 'bw_of', None) is not None:
                origin = origin.bw_of
            src = origin if origin is not None else n
            k = _group_key(src.raw_ctx)
            if k is None:
                k = order[-1]
            stage_of[n] = order.index(k)
        self.stage_of = stage_of

        # ---- my stage / replica ------------------------------------------------------------
        rank = config.rank
        self.stage = self.replica = None
        for s, key in enumerate(order):
            devs = [d for d in key if d[1] == 'gpu']
            ids = [d[2] for d in devs]
            if config.local_rank in ids:
                self.stage, self.replica = s, ids.index(config.local_rank)
        assert self.stage is not None, 'rank %d has no pipeline stage' % rank
        self.nreplica = len([d for d in order[self.stage] if d[1] == 'gpu'])
        # global rank of (stage, replica): ranks are GPU ordinals on one node
        self.rank_of = lambda s, r: [d[2] for d in order[s] if d[1] == 'gpu'][r]

        # ---- phases and local node lists ----------------------------------------------------
        backward = set()
        for n in topo:
            if isinstance(n, OptimizerOp):
                continue
            if getattr(n, 'bw_of', None) is not None or any(i in backward for i in n.inputs):
                backward.add(n)
        self.backward = backward
        mine = [n for n in topo if stage_of.get(n) == self.stage]
        self.params = [n for n in mine if isinstance(n, PlaceholderOp) and n.is_param]
        self.feeds = [n for n in mine if isinstance(n, PlaceholderOp) and not n.is_param]
        from ..dataloader import DataloaderOp
        self.loaders = [n for n in mine if isinstance(n, DataloaderOp)]
        comp = [n for n in mine if not isinstance(n, (PlaceholderOp, DataloaderOp))]
        self.fwd = [n for n in comp if n not in backward]
        self.bwd = [n for n in comp if n in backward]

        # ---- messages ---------------------------------------------------------------------
        self.recv_msgs = {'F': [], 'B': []}
        self.send_msgs = {'F': [], 'B': []}
        seen = set()
        for n in topo:
            if n not in stage_of:
                continue
            for inp in n.inputs:
                if inp is None or inp not in stage_of:
                    continue
                a, b = stage_of[inp], stage_of[n]
                if a == b or (inp, b) in seen:
                    continue
                seen.add((inp, b))
                phase = 'B' if inp in backward else 'F'
                if phase == 'F':
                    assert a < b, 'forward edge %s -> %s goes to an earlier stage' % (inp.name, n.name)
                else:
                    assert a > b, 'backward edge %s -> %s goes to a later stage' % (inp.name, n.name)
                if b == self.stage:
                    self.recv_msgs[phase].append((inp.id, a, inp))
                if a == self.stage:
                    self.send_msgs[phase].append((b, inp.id, inp))
        for ph in ('F', 'B'):
            self.recv_msgs[ph].sort(key=lambda t: (t[1], t[0]))
            self.send_msgs[ph].sort(key=lambda t: (t[0], t[1]))

        # replica groups: dist.new_group is collective over the world, so every
        # rank creates every stage's group in the same order
        self.replica_comms = {}
        if any(len([d for d in k if d[1] == 'gpu']) > 1 for k in order) and dist.is_initialized():
            from . import comm as C
            for s, key in enumerate(order):
                ranks = [d[2] for d in key if d[1] == 'gpu']
                if len(ranks) > 1:
                    self.replica_comms[s] = C.new_group_comm(ranks)

        # tied parameters across stages (``p.tied_to = q``, e.g. BERT's MLM decoder on the
        # last stage and the word embeddings on the first): replica r of each of the two
        # stages sums the pair's gradients over a 2-rank group before every update, so
        # the copies (identical at init) stay identical -- Megatron's embedding tie.
        # Groups are created collectively, in topo order, by every rank.
        self.ties = {}
        pairs = []
        for n in topo:
            t = getattr(n, 'tied_to', None)
            if isinstance(n, PlaceholderOp) and t is not None and n in stage_of and t in stage_of \
                    and stage_of[n] != stage_of[t]:
                pairs.append((n, t))
        if pairs and dist.is_initialized():
            from . import comm as C
            for a, b in pairs:
                sa, sb = stage_of[a], stage_of[b]
                for r in range(min(self._nrep(sa), self._nrep(sb))):
                    g = C.new_group_comm([self.rank_of(sa, r), self.rank_of(sb, r)])
                    if self.replica == r and self.stage in (sa, sb):
                        mine = a if self.stage == sa else b
                        self.ties[mine] = g
                        # the pair's summed gradient is dense (the decoder's is), so the
                        # copy whose own gradient is row-sparse (the embedding lookup's)
                        # takes the dense update, exactly like the untied single graph
                        mine.force_dense_grad = True

        # ---- parameters, local optimizer ----------------------------------------------------
        for p in self.params:
            config.init_param(p)
        self.opt = None
        if self.opt_nodes:
            self._build_local_optimizer()
        self.p2p = _P2P(config.device, getattr(config, 'comm', None) if dist.is_initialized() else None)
        self.step_count = 0

    # ---------------------------------------------------------------------------------------
    def _build_local_optimizer(self):
        from ..optimizer import OptimizerOp
        import copy
        gop = self.opt_nodes[0]
        local = [(p, g) for p, g in zip(gop.param_of_input, gop.inputs) if self.stage_of.get(g) == self.stage]
        self.local_grads = {g: i for i, (p, g) in enumerate(local)}
        if not local:
            return
        opt = copy.copy(gop.optimizer)
        opt.params = [p for p, _ in local]
        op = OptimizerOp.__new__(OptimizerOp)
        OptimizerOp.__init__(op, [g for _, g in local], opt)
        op.forward_hook(self.config)
        op.config = self.config
        op.bucket_bytes = int(getattr(self.config, 'bucket_mb', 32) * (1 << 20))
        op.ps_dense = None
        op.ps_dense_wanted = False
        # HetPipe: the PS aggregates the replicas' gradients, so no replica all-reduce
        ps_sync = self.kind == 'hetpipe' and self.config.ps_comm is not None
        if self.nreplica > 1 and not ps_sync:
            op.comm = self.replica_comms[self.stage]
            op.dp = True
        op.setup(self.config, list(range(len(local))))
        self.opt = op
        if ps_sync:
            from ..ps.table import PSDense
            op.ps_dense = PSDense(op.flat, PS_KEY_HETPIPE_STAGE + self.stage, self.config, publish=self.replica == 0,
                                  overlap=False)

    # ---------------------------------------------------------------------------------------
    def _nrep(self, s):
        return len([d for d in self.stage_keys[s] if d[1] == 'gpu'])

    def _sum_ties(self, grads):
        """grads: {local optimizer index: tensor} -- sum the tied parameters' gradients
        with the other stage's copy (in place; dense gradients only)."""
        if not self.ties:
            return grads
        for i, g in list(grads.items()):
            c = self.ties.get(self.opt.param_of_input[i])
            if c is not None:
                if isinstance(g, ndarray.IndexedSlices):
                    g = g.to_dense()
                g = g.float().contiguous().clone()
                c.all_reduce(g, 'sum')
                grads[i] = g
        return grads

    def _compute(self, nodes, vals, aux):
        for n in nodes:
            args = []
            so = set(getattr(n, 'shape_only_inputs', ()))
            ax = set(getattr(n, 'aux_inputs', ()))
            va = set(getattr(n, 'value_and_aux_inputs', ()))
            for k, inp in enumerate(n.inputs):
                if k in so:
                    args.append(_shape_of(vals[inp]))
                elif k in va:
                    args.append((vals[inp], aux[inp]))
                elif k in ax:
                    args.append(aux[inp])
                else:
                    args.append(vals[inp])
            r = n.compute(args)
            if isinstance(r, AuxResult):
                aux[n] = r.aux
                r = r.value
            vals[n] = r

    def _peer(self, stage):
        return self.rank_of(stage, self.replica if self.nreplica > 1 else 0)

    def _phase(self, ph, mb, state):
        vals, aux = state
        msgs = self.recv_msgs[ph]
        if msgs:
            got = self.p2p.recv_many([((nid, src), self._peer(src)) for nid, src, _ in msgs])
            for (_, _, node), v in zip(msgs, got):
                vals[node] = v
        self._compute(self.fwd if ph == 'F' else self.bwd, vals, aux)
        items = []
        for dst, nid, node in self.send_msgs[ph]:
            v = vals[node]
            if isinstance(v, ndarray.IndexedSlices):
                v = v.to_dense()
            items.append(((nid, self.stage), v, self._peer(dst)))
        if items:
            self.p2p.send_many(items)

    def run(self, eval_node_list=None, feed_dict=None, convert_to_numpy_ret_vals=False, batch_num=None, **kw):
        cfg = self.config
        feed_dict = feed_dict or {}
        m = int(batch_num or 1)
        from ..kernels import rng
        rng.new_step()
        for n in find_topo_sort(self.eval_node_list):
            if hasattr(n, 'inference'):
                n.inference = self.inference
        states = []
        for mb in range(m):
            vals, aux = {}, {}
            for p in self.params:
                vals[p] = cfg.compute_value(p)
            for n in self.feeds:
                if n in feed_dict:
                    v = feed_dict[n]
                    v = v.tensor if isinstance(v, ndarray.NDArray) else v
                    v = torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v)
                    chunk = v.shape[0] // m
                    v = v[mb * chunk:(mb + 1) * chunk]
                    if v.dtype == torch.float64:
                        v = v.float()
                    vals[n] = v.to(cfg.device)
            states.append((vals, aux))
        if self.inference:
            sched = [('F', i) for i in range(m)]
        elif self.kind == 'gpipe':
            sched = gpipe_schedule(self.stage, self.nstages, m)
        else:
            sched = pipedream_schedule(self.stage, self.nstages, m)
        acc = {}
        results = [None] * m
        self.p2p.new_step()
        stash = self.kind == 'pipedream' and not self.inference and self.opt is not None
        for ph, mb in sched:
            vals, aux = states[mb]
            if ph == 'F':
                for d in self.loaders:
                    vals[d] = d.get_arr(self.name, cfg)
                if stash:
                    # weight stashing (reference pipedream_subexecutor.py:90-128): this
                    # micro-batch's forward AND backward use the weights current at its
                    # forward; updates of earlier micro-batches land in the live copy
                    for p in self.params:
                        vals[p] = cfg.compute_value(p).clone()
            self._phase(ph, mb, states[mb])
            if ph == 'B' or self.inference:
                results[mb] = self._outputs(vals, convert_to_numpy_ret_vals)
                if self.opt is not None:
                    grads = {}
                    for g, i in self.local_grads.items():
                        v = vals.get(g)
                        if v is None:
                            continue
                        if stash:
                            grads[i] = v
                        elif isinstance(v, ndarray.IndexedSlices):
                            # sparse (embedding) grads stay sparse across micro-batches
                            acc[i] = v if i not in acc else acc[i].merge(v)
                        else:
                            # clone: v may be a slot of the flat gradient buffer that the next
                            # micro-batch overwrites in place
                            acc[i] = v.float().clone() if i not in acc else acc[i] + v.float()
                    if stash and grads:
                        # PipeDream: apply this micro-batch's gradient to the LATEST weights
                        # right after its backward (reference copy_latest_weight :130-147 +
                        # OptimizerOp per backward) -- no pipeline flush
                        self._apply(grads)
                states[mb] = None
        self.p2p.flush()
        if self.opt is not None and acc:
            acc = self._sum_ties(acc)
            op = self.opt
            op.begin_step()
            for i in range(len(op.inputs)):
                if i in acc:
                    op.on_grad_ready(i, acc[i])
            op.compute([])
        self.step_count += 1
        return results

    def _apply(self, grads):
        grads = self._sum_ties(grads)
        op = self.opt
        op.begin_step()
        for i in range(len(op.inputs)):
            if i in grads:
                op.on_grad_ready(i, grads[i])
        op.compute([])

    def _outputs(self, vals, convert):
        out = []
        for n in self.eval_node_list:
            v = vals.get(n)
            if v is None or not isinstance(v, torch.Tensor):
                out.append(None)
            elif convert:
                out.append(v.detach().float().cpu().numpy())
            else:
                out.append(ndarray.NDArray(v))
        return out

    @property
    def batch_num(self):
        nums = [d.get_batch_num(self.name) for d in self.loaders]
        nums = [x for x in nums if x is not None]
        return min(nums) if nums else None
