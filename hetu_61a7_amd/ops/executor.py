"""Autodiff, HetuConfig, Executor and SubExecutor.

Parity: reference ``gpu_ops/executor.py`` (HetuConfig ``:134-358``, Executor
``:361-563``, SubExecutor ``:566-1063``, gradients ``:1066-1181``).

MI355X execution model:
* A SubExecutor compiles its eval-node set once into a static *plan*: topological
  compute order, per-step input references (value / aux / shape-only), and the
  list of values whose last use is each step (liveness-based freeing on top of the
  HIP stream-ordered caching allocator -- the reference's HetuMemoryPool plan).
* Everything is issued asynchronously on the device's current HIP stream; no
  host-side ``event.sync()`` per dependency (reference ``executor.py:1034-1036``).
  Gradient buckets are all-reduced on RCCL's stream as soon as they complete.
* hipGraph replay (default for single-GPU executors, ``use_hipgraph`` / HETU_HIPGRAPH):
  the whole steady-state step is captured after a warm-up and replayed, with feeds
  copied into static device buffers; random ops stay fresh through the device step
  counter of ``kernels/rng.py``.
* Mixed precision (``mixed_precision='bf16'``): fp32 master weights in the
  optimizer's flat buffer, bf16 compute copies refreshed by the fused update
  kernel, bf16 activations, fp32 BN/LN statistics and fp32 losses.
"""
from __future__ import annotations

import os
import sys
import pickle
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .._base import gpu_available, set_device
from ..kernels import rng as _RNG

from .node import Op
from .variable import PlaceholderOp
from .nn import AuxResult
from .. import ndarray
from ..context import DeviceGroup, get_current_context, dist_env, get_launch_config_by_traverse_nodes
from ..stream import Stream, Event


# ---------------------------------------------------------------------------
# graph utilities
def find_topo_sort(node_list) -> List[Op]:
    """Iterative post-order DFS (no recursion limit on deep nets).

    A node may set ``topo_input_order`` (a permutation of its input indices) to
    change the order its inputs are visited in; the optimizer uses it to order the
    weight-gradient computations (see ``OptimizerOp.backward_hook``)."""
    visited = set()
    order = []
    for root in node_list:
        if root is None or root in visited:
            continue
        stack = [(root, 0)]
        while stack:
            node, i = stack.pop()
            if i == 0:
                if node in visited:
                    continue
            if i < len(node.inputs):
                stack.append((node, i + 1))
                perm = getattr(node, 'topo_input_order', None)
                child = node.inputs[perm[i] if perm is not None else i]
                if child is not None and child not in visited:
                    stack.append((child, 0))
            else:
                if node not in visited:
                    visited.add(node)
                    order.append(node)
    return order


def sum_node_list(node_list, ctx=None):
    node_list = [n for n in node_list if n is not None]
    if not node_list:
        return None
    if len(node_list) == 1:
        return node_list[0]
    from .reduce import sum_op
    return sum_op(node_list, ctx=ctx)


def _mark_backward(roots, start_id, origin):
    stack = [r for r in roots if r is not None]
    while stack:
        n = stack.pop()
        if n.id < start_id or getattr(n, 'bw_of', None) is not None:
            continue
        n.bw_of = origin
        stack.extend(i for i in n.inputs if i is not None)


def gradients(output_node, node_list, insert_grad=None, return_all=False):
    """Reverse-mode autodiff (reference executor.py:1066-1181).

    Every node created while differentiating forward node X is tagged
    ``bw_of = X`` -- the pipeline partitioner places it on X's stage."""
    from .basic import oneslike_op
    from . import node as _N
    start = _N.G_NODE_ID
    if insert_grad is None:
        insert_grad = oneslike_op(output_node, ctx=output_node.raw_ctx)
    _mark_backward([insert_grad], start, output_node)
    node_to_grads = {output_node: [insert_grad]}
    node_to_output_grad = {}
    backward2forward = {}
    forward2backward = {}
    topo = find_topo_sort([output_node])
    for node in reversed(topo):
        if node not in node_to_grads:
            continue
        start = _N.G_NODE_ID
        grad = sum_node_list(node_to_grads[node], ctx=node.raw_ctx)
        node_to_output_grad[node] = grad
        if grad is None:
            continue
        input_grads = node.gradient(grad)
        _mark_backward([grad] + list(input_grads or []), start, node)
        if input_grads is None:
            continue
        forward2backward[node] = [g for g in input_grads if g is not None]
        for inp, g in zip(node.inputs, input_grads):
            if g is None:
                continue
            node_to_grads.setdefault(inp, []).append(g)
            backward2forward[g] = (node, inp)
    grads = [node_to_output_grad.get(n) for n in node_list]
    if return_all:
        return grads, backward2forward, forward2backward
    return grads


# ---------------------------------------------------------------------------
class HetuConfig(object):
    """Per-process execution configuration (reference executor.py:134-358)."""

    def __init__(self, eval_node_list, ctx=None, seed=None, comm_mode=None, use_sparse_pull=True,
                 cstable_policy=None, bsp=-1, prefetch=True, enable_lazy=False, cache_bound=100,
                 log_path=None, pipeline=None, dist_strategy=None, use_preduce=False, overlap=True,
                 use_nccl_collectives=True, mixed_precision=None, bucket_mb=32, use_hipgraph=None,
                 timing=None, zero=0, deterministic=None, **kwargs):
        self.eval_node_list = eval_node_list
        if deterministic is not None:
            # bitwise-reproducible kernels (kernels.deterministic); process-wide
            from ..kernels import set_deterministic
            set_deterministic(deterministic)
        self.seed = seed if seed is not None else int(os.environ.get('HETU_SEED', 0) or 0) or int(time.time())
        if seed is None and os.environ.get('HETU_SEED') is None:
            # identical seeds on every data-parallel rank keep parameters identical
            self.seed = 1234
        _RNG.set_base_seed(self.seed)
        self.comm_mode = comm_mode
        self.use_sparse_pull, self.cstable_policy, self.bsp = use_sparse_pull, cstable_policy, bsp
        self.prefetch, self.enable_lazy, self.cache_bound = prefetch, enable_lazy, cache_bound
        self.log_path, self.pipeline, self.dist_strategy = log_path, pipeline, dist_strategy
        self.use_preduce, self.overlap, self.use_nccl_collectives = use_preduce, overlap, use_nccl_collectives
        self.mixed_precision = mixed_precision in ('bf16', 'bfloat16', True)
        self.bucket_mb = bucket_mb
        self.zero = int(zero)   # 1: ZeRO-1 sharded optimizer state (optimizer.py _make_zero_buckets)
        self.timing = timing
        self.h2d_ops, self.d2h_ops = {}, {}
        self.placeholder_to_arr_map: Dict[Op, torch.Tensor] = {}
        self.compute_values: Dict[Op, torch.Tensor] = {}
        self.ps_comm = None
        self.comm = None
        self.extra = kwargs
        self.grad_wire = kwargs.get('grad_wire')   # DP all-reduce wire format: 'fp32' | 'bf16'

        rank, world, local = dist_env()
        self.rank, self.nrank, self.local_rank = rank, world, local

        # ---- placement / mode decision (reference executor.py:243-256) ----------
        if dist_strategy is not None:
            ctx = dist_strategy.set_raw_ctxs_n_states(eval_node_list, None)
        if ctx is None:
            ctx = get_current_context()
        if ctx is None:
            ctx = ndarray.gpu(local) if (gpu_available() and world > 1) else ndarray.cpu(0)
        launch_mpi = launch_ps = False
        if isinstance(ctx, DeviceGroup) or isinstance(ctx, (list, tuple)):
            dg = ctx if isinstance(ctx, DeviceGroup) else DeviceGroup(list(ctx))
            launch_mpi, launch_ps, self.node_strategy, devices, _ = get_launch_config_by_traverse_nodes(eval_node_list, dg)
            workers = [d for d in dg.all_devices() if ndarray.is_gpu_ctx(d)]
            if dg.worker_num > 1:
                self.context = self._local_worker(workers)
            elif workers:
                self.context = workers[0]
            else:
                self.context = dg.servers[0] if dg.server_num else ndarray.cpu(0)
            self.device_group = dg
        else:
            self.context = ctx
            self.node_strategy = {}
            self.device_group = None
        from ..parallel.lowering import lower_dispatch, PENDING_MESHES
        lower_dispatch(list(eval_node_list))
        self.spmd = bool(PENDING_MESHES)
        if pipeline is not None or self.spmd:
            # one process per GPU: this rank's device is its own GPU ordinal
            self.context = ndarray.gpu(local) if gpu_available() else ndarray.cpu(0)
            launch_mpi = launch_ps = False
        if comm_mode is None:
            if launch_mpi and launch_ps:
                comm_mode = 'Hybrid'
            elif launch_mpi:
                comm_mode = 'AllReduce'
            elif launch_ps:
                comm_mode = 'PS'
            elif world > 1 and dist_strategy is None and pipeline is None:
                comm_mode = None
        self.comm_mode = comm_mode
        self.cpu_only = not gpu_available()
        if ndarray.is_gpu_ctx(self.context) and not gpu_available():
            # CPU-only process (tests / gloo rehearsal of the distributed path)
            self.context = ndarray.cpu(0)
            for n in find_topo_sort(eval_node_list):
                if ndarray.is_gpu_ctx(n.ctx):
                    n.ctx = self.context
        if self.context is not None and ndarray.is_gpu_ctx(self.context) and gpu_available():
            n_dev = torch.cuda.device_count()
            if self.context.device_id >= n_dev and os.environ.get('HETU_DIST_BACKEND') == 'gloo':
                # multi-rank rehearsal on a box with fewer GPUs than ranks (gloo only)
                self.context = ndarray.gpu(self.context.device_id % n_dev)
            set_device(self.context.device_id)

        # ---- communicators ------------------------------------------------------------
        # HETU_FORCE_DP=1: run the data-parallel gradient path (buckets, async all-reduce on
        # the communicator's stream, bf16 wire) with a single rank -- the one-GPU rehearsal of
        # the multi-GPU path on real RCCL (tests/test_rccl_gpu.py)
        self.force_dp = os.environ.get('HETU_FORCE_DP', '0') == '1' and dist_strategy is not None
        if self.force_dp and self.comm_mode is None:
            self.comm_mode = 'AllReduce'
        if self.comm_mode in ('AllReduce', 'Hybrid') or pipeline is not None or world > 1:
            if world > 1 or self.force_dp:
                from ..parallel import comm as C
                self.comm = C.init_process_group(use_gpu=ndarray.is_gpu_ctx(self.context))
                if self.spmd:
                    from ..parallel.lowering import create_groups
                    create_groups(PENDING_MESHES, world)
        if self.comm_mode in ('PS', 'Hybrid'):
            from ..ps import worker as psw
            self.ps_comm = psw.get_worker(self)

        # ---- streams (reference executor.py:319-334) -------------------------------------
        if ndarray.is_gpu_ctx(self.context) and gpu_available():
            from ..runtime import _torch_view, current_stream
            self.comp_stream = Stream(self.context, torch_stream=_torch_view(current_stream())[1])
        else:
            self.comp_stream = Stream(self.context, torch_stream=None)
        self.h2d_stream = Stream(self.context)
        self.d2h_stream = Stream(self.context)
        self.nccl_stream = None

        # ---- hipGraph replay: on by default for single-GPU executors --------
        # ``use_hipgraph`` True / False forces it; None follows HETU_HIPGRAPH (1 / 0, default
        # auto: one GPU process, no communicator, no PS, no pipeline).  Replay-unsafe steps
        # (per-step host schedules, failed captures) fall back to eager execution.
        env = os.environ.get('HETU_HIPGRAPH', 'auto')
        if use_hipgraph is None:
            use_hipgraph = env == '1' or (env == 'auto' and gpu_available() and ndarray.is_gpu_ctx(self.context)
                                          and world == 1 and self.comm is None and self.ps_comm is None
                                          and self.comm_mode is None and pipeline is None and not self.spmd)
        self.use_hipgraph = bool(use_hipgraph)
        # piecewise replay (utils/piecewise.py) for single-GPU PS steps: the device segments
        # between the host-bound ops (PS lookups, gradient staging, the PS optimizer) are
        # captured and replayed; HETU_PIECEWISE_GRAPH=0 / 1 forces it off / on
        pw = os.environ.get('HETU_PIECEWISE_GRAPH', 'auto')
        self.use_piecewise = not self.use_hipgraph and (pw == '1' or (
            pw == 'auto' and gpu_available() and ndarray.is_gpu_ctx(self.context) and world == 1
            and self.comm is None and self.ps_comm is not None and pipeline is None and not self.spmd))

        # ---- hooks (pre-order backward_hook, post-order forward_hook) ------------------------
        self.topo_sort_with_hook(eval_node_list)

    def _local_worker(self, workers):
        local_rank = self.local_rank
        locals_ = [w for w in workers if (w.local if isinstance(w, ndarray.DLContext) else True)]
        if not locals_:
            return ndarray.gpu(local_rank)
        return locals_[local_rank % len(locals_)] if isinstance(locals_[0], ndarray.DLContext) else ndarray.gpu(local_rank)

    def resolve_ctx(self, dg):
        """Pick this process's device from a DeviceGroup raw context."""
        devs = dg.all_devices()
        if self.context in devs:
            return self.context
        gpus = [d for d in devs if ndarray.is_gpu_ctx(d)]
        if len(devs) == 1:
            return devs[0]
        if gpus:
            return self.context
        return devs[0]

    def topo_sort_with_hook(self, node_list):
        visited = set()
        # pre-order backward hooks
        order = find_topo_sort(node_list)
        for n in reversed(order):
            if n not in visited:
                n.backward_hook(self)
                visited.add(n)
        for n in order:
            n.forward_hook(self)

    # ---- parameter storage ------------------------------------------------------------
    @property
    def device(self):
        return self.context.torch_device if isinstance(self.context, ndarray.DLContext) else torch.device('cpu')

    def init_param(self, node: PlaceholderOp):
        if node in self.placeholder_to_arr_map:
            return self.placeholder_to_arr_map[node]
        if getattr(node, 'ps_managed', False):
            from ..ps.table import PSTable
            t = PSTable(node, self)
            self.placeholder_to_arr_map[node] = t
            return t
        dev = node.ctx.torch_device if isinstance(node.ctx, ndarray.DLContext) else self.device
        t = node.initial_value(self.seed, dev)
        if t.dtype == torch.float64:
            t = t.float()
        self.placeholder_to_arr_map[node] = t
        return t

    def compute_value(self, node: PlaceholderOp):
        v = self.compute_values.get(node)
        if v is not None:
            return v
        t = self.placeholder_to_arr_map[node]
        if not isinstance(t, torch.Tensor):
            return t
        if self.mixed_precision and t.dtype == torch.float32 and t.is_cuda and not node.trainable \
                and t.dim() >= 2 and not getattr(node, 'keep_fp32', False):
            v = t.to(torch.bfloat16)
            self.compute_values[node] = v
            return v
        return t


# ---------------------------------------------------------------------------
class Executor(object):
    """``ht.Executor({'train': [...], 'validate': [...]}, ctx=..., ...)``."""

    def __init__(self, eval_node_dict, config=None, timing=None, **kwargs):
        if not isinstance(eval_node_dict, dict):
            eval_node_dict = {'default': eval_node_dict}
        self.eval_node_dict = {k: list(v) for k, v in eval_node_dict.items()}
        all_nodes = []
        for v in self.eval_node_dict.values():
            for n in v:
                if n not in all_nodes:
                    all_nodes.append(n)
        if config is None:
            config = HetuConfig(eval_node_list=all_nodes, timing=timing, **kwargs)
        self.config = config
        self.timing = timing
        self.subexecutor = {}
        for k, v in self.eval_node_dict.items():
            if config.pipeline:
                from ..parallel.pipeline import make_pipeline_subexecutor
                self.subexecutor[k] = make_pipeline_subexecutor(config.pipeline, k, v, config)
            else:
                self.subexecutor[k] = SubExecutor(k, v, config)
        if timing:
            for sub in self.subexecutor.values():
                if hasattr(sub, 'enable_timer'):
                    sub.enable_timer(timing)

    # reference API ------------------------------------------------------------------------
    @property
    def rank(self):
        return self.config.rank if self.config.nrank > 1 else None

    @property
    def config_rank(self):
        return self.config.rank

    @property
    def batch_num(self):
        return list(self.subexecutor.values())[0].batch_num

    def get_batch_num(self, name='default'):
        return self.subexecutor[name].batch_num

    def run(self, name='default', eval_node_list=None, feed_dict=None, convert_to_numpy_ret_vals=False, **kwargs):
        if isinstance(name, dict) and feed_dict is None:
            feed_dict, name = name, 'default'
        return self.subexecutor[name].run(eval_node_list or [], feed_dict or {}, convert_to_numpy_ret_vals, **kwargs)

    def profile(self, feed_shapes, log_file=None, profiler='gpu', name='default'):
        from ..utils.profiler import HetuProfiler
        return HetuProfiler(self.subexecutor[name], feed_shapes, log_file, profiler).run()

    def logOut(self, *args, name='default', **kwargs):
        return self.subexecutor[name].logOut(*args, **kwargs)

    def clearTimer(self, name='default'):
        return self.subexecutor[name].clearTimer()

    def export_chrome_trace(self, path, name='default'):
        return self.subexecutor[name].export_chrome_trace(path)

    def optimizer_ops(self, name='default'):
        """The OptimizerOps of one named sub-graph (DP buckets, comm_trace())."""
        return list(getattr(self.subexecutor[name], 'opt_ops', []))

    def recordLoads(self):
        if self.config.ps_comm is not None:
            self.config.ps_comm.record_loads()

    # checkpoint (reference executor.py:457-537): {name: float32 ndarray} pickle ----------
    def _params(self):
        return [n for n in self.config.placeholder_to_arr_map if isinstance(n, PlaceholderOp) and n.trainable]

    def save(self, file_path, file_name='checkpoint.pkl', save_optimizer=False):
        from ..utils import checkpoint
        return checkpoint.save(self, file_path, file_name, save_optimizer)

    def load(self, file_path, file_name='checkpoint.pkl', consider_splits=False):
        from ..utils import checkpoint
        return checkpoint.load(self, file_path, file_name, consider_splits)

    def load_dict(self, state, consider_splits=False):
        from ..utils import checkpoint
        return checkpoint.load_dict(self, state, consider_splits)

    def return_tensor_values(self):
        return {n.name: v for n, v in self.config.placeholder_to_arr_map.items()}

    def __del__(self):
        pass


# ---------------------------------------------------------------------------
class SubExecutor(object):
    """Compiled plan for one named eval-node set."""

    def __init__(self, name, eval_node_list, config: HetuConfig):
        from ..optimizer import OptimizerOp
        from ..dataloader import DataloaderOp, GNNDataLoaderOp
        self.name = name
        self.eval_node_list = list(eval_node_list)
        self.config = config
        self.topo_order = find_topo_sort(self.eval_node_list)
        # training mode when the set updates weights or evaluates any gradient node
        self.inference = not any(isinstance(n, OptimizerOp) or getattr(n, 'bw_of', None) is not None
                                 for n in self.topo_order)
        self.param_nodes, self.feed_nodes, self.dataloader_nodes, self.computing_nodes = [], [], [], []
        for n in self.topo_order:
            if isinstance(n, PlaceholderOp):
                if n.is_param:
                    self.param_nodes.append(n)
                else:
                    self.feed_nodes.append(n)
            elif isinstance(n, (DataloaderOp, GNNDataLoaderOp)):
                self.dataloader_nodes.append(n)
            else:
                self.computing_nodes.append(n)
        for p in self.param_nodes:
            config.init_param(p)
        self.opt_ops = [n for n in self.computing_nodes if isinstance(n, OptimizerOp)]
        # PS tables looked up with dataloader-fed ids: prefetch the next batch's rows
        self.ps_prefetch = []
        if getattr(config, 'prefetch', False):
            from .embedding import EmbeddingLookUp
            for n in self.computing_nodes:
                if isinstance(n, EmbeddingLookUp) and isinstance(n.inputs[1], DataloaderOp):
                    t = config.placeholder_to_arr_map.get(n.inputs[0])
                    if t is not None and hasattr(t, 'next_ids_fn'):
                        self.ps_prefetch.append((t, n.inputs[1]))
        self.mode_nodes = [n for n in self.topo_order if hasattr(n, 'inference')]
        # per-training-step schedules owned by ops (the dense-to-sparse MoE gate's
        # temperature): stepped once after every training step of this sub-graph
        self.step_end_nodes = [n for n in self.topo_order if hasattr(n, 'on_step_end')]
        self._build_plan()
        self.timer = None
        self.graph = None
        self.piecewise = None
        self.graph_state = None
        self.step_count = 0

    # ---- plan ------------------------------------------------------------------------
    def _build_plan(self):
        from ..optimizer import OptimizerOp
        persistent = set(self.eval_node_list) | set(self.param_nodes)
        pos = {n: i for i, n in enumerate(self.computing_nodes)}
        last_use = {}
        self.grad_hooks = {}
        for i, n in enumerate(self.computing_nodes):
            if isinstance(n, OptimizerOp):
                for j, g in enumerate(n.inputs):
                    self.grad_hooks.setdefault(g, []).append((n, j))
                continue
            so = set(getattr(n, 'shape_only_inputs', ()))
            for k, inp in enumerate(n.inputs):
                if k in so:
                    continue
                last_use[inp] = i
        # a grad consumed only by the optimizer dies right after the hook fires
        for g in self.grad_hooks:
            last_use[g] = max(last_use.get(g, -1), pos.get(g, -1))
        self.release_after = [[] for _ in self.computing_nodes]
        for node, i in last_use.items():
            if node in persistent or i < 0:
                continue
            if isinstance(node, PlaceholderOp) and node.is_param:
                continue
            self.release_after[i].append(node)
        # nodes never consumed (and not eval outputs) are released right away
        for i, n in enumerate(self.computing_nodes):
            if n not in last_use and n not in persistent:
                self.release_after[i].append(n)
        # optimizer flat layout in gradient-arrival order
        for op in self.opt_ops:
            order = sorted(range(len(op.inputs)), key=lambda j: pos.get(op.inputs[j], -1))
            op.setup(self.config, order)
        self.input_specs = []
        for n in self.computing_nodes:
            so = set(getattr(n, 'shape_only_inputs', ()))
            aux = set(getattr(n, 'aux_inputs', ()))
            va = set(getattr(n, 'value_and_aux_inputs', ()))
            spec = []
            for k, inp in enumerate(n.inputs):
                if isinstance(n, OptimizerOp):
                    spec.append((inp, 'skip'))
                elif k in so:
                    spec.append((inp, 'shape'))
                elif k in va:
                    spec.append((inp, 'va'))
                elif k in aux:
                    spec.append((inp, 'aux'))
                else:
                    spec.append((inp, 'value'))
            self.input_specs.append(spec)

    @property
    def batch_num(self):
        nums = [d.get_batch_num(self.name) for d in self.dataloader_nodes]
        nums = [x for x in nums if x is not None]
        return min(nums) if nums else None

    # ---- feeds -------------------------------------------------------------------------
    def _feed_value(self, node, value):
        if isinstance(value, ndarray.NDArray):
            t = value.tensor
        elif isinstance(value, torch.Tensor):
            t = value
        elif isinstance(value, ndarray.ND_Sparse_Array):
            return value
        else:
            arr = np.asarray(value)
            if arr.dtype == np.float64:
                arr = arr.astype(np.float32)
            t = torch.from_numpy(np.ascontiguousarray(arr))
        dev = node.ctx.torch_device if isinstance(node.ctx, ndarray.DLContext) else self.config.device
        if getattr(node, 'host_feed', False):
            dev = torch.device('cpu')
        if t.device != dev:
            src = t
            t = t.to(dev, non_blocking=True)
            if not src.is_cuda and not src.is_floating_point():
                t.hetu_host = src      # host copy of fed ids: PS lookups need no device sync
        if self.config.mixed_precision and t.is_cuda and t.dtype == torch.float32 and \
                not getattr(node, 'keep_fp32', False):
            from ..kernels.elementwise import cast
            t = cast(t.contiguous(), torch.bfloat16)    # native cast kernel
        return t

    # ---- run ---------------------------------------------------------------------------
    def run(self, eval_node_list=None, feed_dict=None, convert_to_numpy_ret_vals=False, **kwargs):
        feed_dict = feed_dict or {}
        cfg = self.config
        for n in self.mode_nodes:
            n.inference = self.inference
        if not self.opt_ops:
            _ps_drain_dense()
        if cfg.use_hipgraph and cfg.device.type == 'cuda' and not self.step_end_nodes:
            # (ops with per-step host schedules -- the DTS gate's temperature and budget --
            # change launch arguments and shapes between steps: not replayable, run eager)
            return self._run_graph(feed_dict, convert_to_numpy_ret_vals)
        if getattr(cfg, 'use_piecewise', False) and cfg.device.type == 'cuda' and not self.step_end_nodes \
                and self.opt_ops and self.timer is None:
            from .. import memory_pool as _MP
            if _MP.torch_bfc_enabled():
                if self.piecewise is None:
                    from ..utils.piecewise import PiecewiseRunner
                    self.piecewise = PiecewiseRunner(self)
                return self.piecewise.run(feed_dict, convert_to_numpy_ret_vals)
        vals = self._run_eager(feed_dict)
        if self.opt_ops and not self.inference:
            for n in self.step_end_nodes:
                n.on_step_end()
        return self._collect(vals, convert_to_numpy_ret_vals)

    def _prepare_inputs(self, feed_dict):
        cfg = self.config
        vals = {}
        for p in self.param_nodes:
            vals[p] = cfg.compute_value(p)
        for n, v in feed_dict.items():
            node = n
            vals[node] = self._feed_value(node, v)
        self.last_feed_shapes = {n: tuple(vals[n].shape) for n in feed_dict if hasattr(vals[n], 'shape')}
        for n in self.feed_nodes:
            if n not in vals:
                raise KeyError('placeholder %s not fed' % n.name)
        for d in self.dataloader_nodes:
            v = d.get_arr(self.name, cfg)
            # GNN sampling handlers return host arrays: place them like a feed
            vals[d] = v if isinstance(v, torch.Tensor) else self._feed_value(d, v)
        for t, d in self.ps_prefetch:
            t.next_ids_fn = (lambda d=d, nm=self.name: d.peek_next_arr(nm))
        return vals

    def _run_eager(self, feed_dict, vals=None):
        cfg = self.config
        if vals is None:
            vals = self._prepare_inputs(feed_dict)
        _RNG.new_step()            # per-step random state (kernels/rng.py: replay-safe seeds)
        aux = {}
        shapes = {}
        for op in self.opt_ops:
            op.begin_step()
        timer = self.timer
        for i, n in enumerate(self.computing_nodes):
            args = []
            for inp, kind in self.input_specs[i]:
                if kind == 'value':
                    args.append(vals[inp])
                elif kind == 'shape':
                    s = shapes.get(inp)
                    if s is None:
                        v = vals[inp]
                        s = _shape_of(v)
                    args.append(s)
                elif kind == 'aux':
                    args.append(aux[inp])
                elif kind == 'va':
                    args.append((vals[inp], aux[inp]))
            if timer is not None:
                timer.start(n)
            if _PROFILE_OPS:
                with torch.profiler.record_function('hetu_op:%s:%s' % (n.op_type, n.name)):
                    r = n.compute(args)
            else:
                r = n.compute(args)
            if timer is not None:
                timer.stop(n)
            if isinstance(r, AuxResult):
                aux[n] = r.aux
                r = r.value
            vals[n] = r
            if r is not None:
                shapes[n] = _shape_of(r)
                if _CHECK_LAYOUT and isinstance(r, torch.Tensor) and r.dim() == 4 and r.is_cuda \
                        and not r.is_contiguous(memory_format=torch.channels_last):
                    _LAYOUT_MISSES[n.op_type] = _LAYOUT_MISSES.get(n.op_type, 0) + 1
            hooks = self.grad_hooks.get(n)
            if hooks:
                for op, j in hooks:
                    op.on_grad_ready(j, r)
            for dead in self.release_after[i]:
                v = vals.pop(dead, None)
                if v is not None and dead not in shapes:   # later shape-only consumers
                    shapes[dead] = _shape_of(v)
                aux.pop(dead, None)
        self.step_count += 1
        return vals

    def _collect(self, vals, convert):
        out = []
        for n in self.eval_node_list:
            v = vals.get(n)
            if v is None:
                out.append(None)
            elif convert:
                if isinstance(v, torch.Tensor):
                    out.append(v.detach().float().cpu().numpy() if v.dtype == torch.bfloat16 else v.detach().cpu().numpy())
                else:
                    out.append(v.asnumpy())
            else:
                out.append(ndarray.NDArray(v) if isinstance(v, torch.Tensor) else v)
        return out

    # ---- hipGraph capture ----------------------------------------------------------------
    def _run_graph(self, feed_dict, convert):
        from ..utils.hipgraph import GraphRunner
        if self.graph is None:
            self.graph = GraphRunner(self)
        return self.graph.run(feed_dict, convert)

    # ---- timing (reference timer_subexecutor.py) -------------------------------------------
    def enable_timer(self, kind='gpu'):
        from ..utils.timer import NodeTimer
        self.timer = NodeTimer(kind)

    def logOut(self, path=None, log_level='node', clear=True):
        if self.timer is None:
            return None
        return self.timer.log_out(path, log_level, clear)

    def export_chrome_trace(self, path):
        """Chrome/Perfetto trace of the timed steps (needs ``timing=``)."""
        if self.timer is None:
            raise RuntimeError('enable timing (Executor(..., timing="gpu"|"cpu")) to record a trace')
        return self.timer.export_chrome_trace(path)

    def clearTimer(self):
        if self.timer is not None:
            self.timer.clear()


_CHECK_LAYOUT = os.environ.get('HETU_CHECK_LAYOUT', '0') == '1'
# HETU_PROFILE_OPS=1: every op's compute inside a torch.profiler record_function range
# (scripts/find_torch_kernels.py attributes device kernels to graph ops through it)
_PROFILE_OPS = os.environ.get('HETU_PROFILE_OPS', '0') == '1'
_LAYOUT_MISSES = {}


def _ps_drain_dense():
    t = sys.modules.get('hetu_61a7_amd.ps.table')
    if t is not None and t._LIVE:
        t.drain_dense()


def layout_report():
    return dict(_LAYOUT_MISSES)


def _shape_of(v):
    if isinstance(v, torch.Tensor):
        return v.shape
    if isinstance(v, ndarray.IndexedSlices):
        return torch.Size(v.dense_shape)
    if isinstance(v, (tuple, list)):
        return None
    if hasattr(v, 'shape'):
        return v.shape
    return None
