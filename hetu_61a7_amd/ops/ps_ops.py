"""Parameter-server graph ops (reference
``gpu_ops/ParameterServerCommunicate.py:13-338``).

The optimizer normally drives PS traffic itself (``OptimizerOp`` stages every
PS-held gradient as soon as it is produced and pushes it after the step; see
``ps/table.py``).  These two ops expose the same machinery as explicit graph
nodes for graphs that wire PS communication by hand, as the reference's
``parameterServerCommunicate_op`` / ``parameterServerSparsePull_op`` do:

* ``parameterServerCommunicate_op(grad, parameter, optimizer)`` pushes
  ``-lr * grad`` for ``parameter`` and (ASP prefetch / BSP / SSP, as configured by
  the executor's ``bsp``) pulls the updated value back.  Embedding tables
  (row-sparse ``IndexedSlices`` gradients) go through their ``PSTable`` (HET cache
  when ``cstable_policy`` is set); dense parameters are one PS key each, seeded
  by worker 0's initial value, and the pull lands in the parameter's device
  tensor in place.
* ``parameterServerSparsePull_op(lookup, deps)`` queues the pull of the NEXT
  batch's rows of the embedding behind ``lookup`` (reference: "only the forward
  graph gets a sparse pull op"), after ``deps`` ran.

``optimizer`` may be an ``ht.optim`` optimizer or the reference wire format
``optimizer.get_config()`` (``config[1][0]`` is the learning rate).
"""
from __future__ import annotations

import torch

from .node import Op
from .. import ndarray
from ..ps import PS_KEY_DENSE_COMM


def _lr_of(optimizer):
    if hasattr(optimizer, 'get_learning_rate'):
        return float(optimizer.get_learning_rate())
    return float(optimizer[1][0])


class ParameterServerCommunicateOp(Op):
    # dense-key namespace above node ids (< 2^20) and the optimizers' flat keys
    DENSE_KEY_BASE = PS_KEY_DENSE_COMM

    def __init__(self, node, parameter, optimizer):
        super().__init__(ParameterServerCommunicateOp, [node], node.raw_ctx)
        self.parameter = parameter
        self.optimizer = optimizer
        self.config = None
        self.dense = None

    def backward_hook(self, config):
        super().backward_hook(config)
        # row-sparse embedding grads: the table lives on the PS (reference
        # Variable.py:55-81 places PS-managed params on the server)
        if config.comm_mode in ('PS', 'Hybrid') and getattr(self.parameter, 'is_embed', False) \
                and self.inputs[0].use_indexed_slices:
            self.parameter.ps_managed = True

    def forward_hook(self, config):
        super().forward_hook(config)
        self.config = config

    def _dense_state(self, value):
        if self.dense is None:
            from ..ps import worker as psw
            from ..ps.table import _pinned
            agent = psw.get_agent()
            key = self.DENSE_KEY_BASE + self.parameter.id
            n = value.numel()
            agent.InitTensor(key, psw.PARAM_DENSE, n, 1, 0, 0.0, 0.0, 0)
            if agent.rank() == 0:
                t = agent.Push(key, value.detach().float().cpu().contiguous().reshape(-1))
                agent.WaitTicket(t)
            agent.BarrierWorker()
            self.dense = (agent, key, _pinned(n), _pinned(n), 0)
        return self.dense

    def compute(self, input_vals, output_val=None, stream_handle=None):
        cfg = self.config
        grad = input_vals[0]
        lr = _lr_of(self.optimizer)
        value = cfg.placeholder_to_arr_map[self.parameter]
        if not isinstance(value, torch.Tensor):      # PSTable (embedding on the PS)
            if not isinstance(grad, ndarray.IndexedSlices):
                rows = value.rows
                grad = ndarray.IndexedSlices(torch.arange(rows), grad.reshape(rows, -1), value.shape)
            value.stage_grad(grad, lr)
            value.flush_grad()
            return None
        if isinstance(grad, ndarray.IndexedSlices):
            grad = grad.to_dense()
        agent, key, push, pull, version = self._dense_state(value)
        n = value.numel()
        push[:n].copy_((grad.reshape(-1).float() * (-lr)), non_blocking=False)
        bsp = cfg.bsp
        if bsp == 0:
            agent.WaitTicket(agent.Push(key, push))
            agent.BarrierWorker()
            agent.WaitTicket(agent.Pull(key, pull))
        elif bsp and bsp > 0:
            if version == 0:
                agent.ssp_init(key, agent.nrank(), bsp)
            agent.WaitTicket(agent.Push(key, push))
            agent.ssp_sync(key, version + 1)
            agent.WaitTicket(agent.Pull(key, pull))
        else:
            agent.WaitTicket(agent.DDPushPull(key, push, pull))
        self.dense = (agent, key, push, pull, version + 1)
        with torch.no_grad():
            value.copy_(pull[:n].view(value.shape).to(value.dtype), non_blocking=True)
        shadow = cfg.compute_values.get(self.parameter)
        if shadow is not None and shadow is not value:
            shadow.copy_(value)
        return None

    def gradient(self, output_grad):
        raise NotImplementedError('PS communication has no gradient')

    def infer_shape(self, input_shapes):
        return None


class ParameterServerSparsePullOp(Op):
    def __init__(self, node, deps_node):
        super().__init__(ParameterServerSparsePullOp, [node] + list(deps_node), node.raw_ctx)
        self.parameter = node.inputs[0]
        self.config = None

    def forward_hook(self, config):
        super().forward_hook(config)
        self.config = config

    def compute(self, input_vals, output_val=None, stream_handle=None):
        table = self.config.placeholder_to_arr_map.get(self.parameter)
        if table is None or isinstance(table, torch.Tensor):
            return None                                  # not PS-held: nothing to pull
        if table.prefetched is None:
            table._prefetch_next()
        return None

    def gradient(self, output_grad):
        raise NotImplementedError('PS pull has no gradient')

    def infer_shape(self, input_shapes):
        return None


def parameterServerCommunicate_op(node, parameter, optimizer):
    """Push ``node`` (the gradient of ``parameter``) to the PS and pull back."""
    return ParameterServerCommunicateOp(node, parameter, optimizer)


def parameterServerSparsePull_op(parameter, deps_node):
    """Queue the next batch's row pull for the embedding looked up by ``parameter``
    (an embedding-lookup node, as in the reference) after ``deps_node``."""
    return ParameterServerSparsePullOp(parameter, deps_node)
