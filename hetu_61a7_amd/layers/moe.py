"""Mixture-of-Experts layers and gates (reference layers/moe_layer.py:7-133,
TopGate.py:7-79, KTop1Gate.py, HashGate.py, SAMGate.py:7-89, BalanceGate.py,
hash_layer.py, ktop1_layer.py, sam_layer.py) plus the Dense-To-Sparse gate
(README paper #6; absent from the reference).

Expert parallelism: tokens are laid out per expert (``layout_transform_op``),
exchanged with one RCCL all-to-all over the xGMI mesh, run through the local
experts, returned with a second all-to-all and combined with the gate weights.
Expert parameters are named ``expert*`` so the optimizer keeps them out of the
data-parallel all-reduce.
"""
from __future__ import annotations

import os
import math

import numpy as np

from .. import ops as O
from .. import initializers as init
from .basic import BaseLayer


def balance_loss(gates, mask, num_experts):
    me = O.reduce_mean_op(gates, axes=0)
    ce = O.reduce_mean_op(mask, axes=0)
    return O.mul_byconst_op(O.reducesumaxiszero_op(O.mul_op(me, ce)), float(num_experts))


def _locations(masks):
    """Slot of each token inside its expert's capacity, for each choice."""
    locs = []
    acc = None
    for i, m in enumerate(masks):
        cum = O.cumsum_with_bias_op(m, bias=-1, dim=0)
        if acc is not None:
            cum = O.add_op(cum, acc)
        locs.append(O.reduce_sum_op(O.mul_op(cum, m), axes=1))
        tot = O.reduce_sum_op(m, axes=0, keepdims=True)
        acc = tot if acc is None else O.add_op(acc, tot)
    return locs


def _fused_locations(topk_indices, k, num_experts):
    """Same slots as ``_locations`` from the [T, k] index node in one native pass."""
    from ..ops.moe import topk_locations_op
    loc = topk_locations_op(topk_indices, num_experts)
    return [O.split_op(loc, axes=[1], indices=[i], splits=[k]) for i in range(k)]


def topkgating(logits, k, capacity_factor, num_tokens, num_experts, embed_dim=None, fused=True):
    capacity = k * math.ceil((num_tokens / num_experts) * capacity_factor)
    if fused and k <= 8 and num_experts <= 512:
        from ..ops.moe import topk_gating_op
        l_aux, idx, loc, gate_w = topk_gating_op(logits, k, capacity, num_experts)
        return l_aux, [idx], [loc], [gate_w], capacity
    gates = O.softmax_op(logits)
    topk_indices = O.topk_idx_op(gates, topk=k)
    indices_s = [O.split_op(topk_indices, axes=[1], indices=[i], splits=[k]) for i in range(k)]
    masks = [O.array_reshape_op(O.one_hot_op(ix, num_classes=num_experts), [-1, num_experts]) for ix in indices_s]
    l_aux = balance_loss(gates, masks[0], num_experts)
    for i in range(1, k):
        l_aux = O.add_op(l_aux, balance_loss(gates, masks[i], num_experts))
    location_s = _locations(masks)
    gates_s = [O.reduce_sum_op(O.mul_op(gates, m), axes=1) for m in masks]
    return l_aux, indices_s, location_s, gates_s, capacity


class _GateBase(BaseLayer):
    def __init__(self, embed_dim, num_tokens, num_experts, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='gate'):
        self.embed_dim, self.num_tokens, self.num_experts = embed_dim, num_tokens, num_experts
        self.top_k, self.capacity_factor, self.eval_capacity_factor = k, capacity_factor, eval_capacity_factor
        self.initializer = initializer or init.GenXavierUniform()
        self.name = name

    def _logits(self, x, n_out=None):
        n_out = n_out or self.num_experts
        w = self.initializer(shape=(self.embed_dim, n_out), name=self.name + '_linear_weight')
        b = init.zeros(shape=(n_out,), name=self.name + '_linear_bias')
        return O.linear_op(x, w, b)


class TopKGate(_GateBase):
    """``fused=True`` (default) runs the whole gate as the fused softmax/top-k/
    slot kernels (``topk_gating_op``); ``fused=False`` builds the reference's
    op-by-op graph (same values)."""

    def __init__(self, embed_dim, num_tokens, num_experts, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='TopK_Gate', fused=True):
        super().__init__(embed_dim, num_tokens, num_experts, k, capacity_factor, eval_capacity_factor,
                         initializer, name)
        self.fused = fused

    def __call__(self, x):
        return topkgating(self._logits(x), self.top_k, self.capacity_factor, self.num_tokens,
                          self.num_experts, fused=self.fused)


class KTop1Gate(_GateBase):
    """k prototypes, each a top-1 gate over num_experts/k experts."""

    def __init__(self, embed_dim, num_tokens, num_experts, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='KTop1_Gate'):
        super().__init__(embed_dim, num_tokens, num_experts, k, capacity_factor, eval_capacity_factor,
                         initializer, name)

    def __call__(self, x):
        k, E = self.top_k, self.num_experts
        per = E // k
        logits = self._logits(x)
        capacity = k * math.ceil((self.num_tokens / E) * self.capacity_factor)
        gates = [O.softmax_op(O.split_op(logits, axes=[1], indices=[i], splits=[k])) for i in range(k)]
        idx = [O.topk_idx_op(g, topk=1) for g in gates]
        masks = [O.array_reshape_op(O.one_hot_op(ix, num_classes=per), [-1, per]) for ix in idx]
        l_aux = balance_loss(gates[0], masks[0], per)
        for i in range(1, k):
            l_aux = O.add_op(l_aux, balance_loss(gates[i], masks[i], per))
        gates_s = [O.reduce_sum_op(O.mul_op(g, m), axes=1) for g, m in zip(gates, masks)]
        location_s = [O.reduce_sum_op(O.mul_op(O.cumsum_with_bias_op(m, bias=-1, dim=0), m), axes=1) for m in masks]
        indices_s = [O.addbyconst_op(ix, float(i * per)) if i else ix for i, ix in enumerate(idx)]
        return l_aux, indices_s, location_s, gates_s, capacity


class HashGate(_GateBase):
    """Routing by a precomputed hash of the token id (no learned gate)."""

    def __init__(self, embed_dim, num_tokens, num_experts, capacity_factor=1.0,
                 eval_capacity_factor=1.0, name='Hash_Gate'):
        super().__init__(embed_dim, num_tokens, num_experts, 1, capacity_factor, eval_capacity_factor,
                         None, name)

    def __call__(self, x, indice):
        capacity = math.ceil((self.num_tokens / self.num_experts) * self.capacity_factor)
        mask = O.array_reshape_op(O.one_hot_op(indice, num_classes=self.num_experts), [-1, self.num_experts])
        loc = O.reduce_sum_op(O.mul_op(O.cumsum_with_bias_op(mask, bias=-1, dim=0), mask), axes=1)
        return [indice], [loc], capacity


class SAMGate(_GateBase):
    """Switch-and-mixture gate: pick the best GPU group, then top-k inside it;
    an alignment loss pushes probability mass into the chosen group."""

    def __init__(self, embed_dim, num_tokens, num_experts, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='SAM_Gate', num_local_gpus=8):
        super().__init__(embed_dim, num_tokens, num_experts, k, capacity_factor, eval_capacity_factor,
                         initializer, name)
        self.num_local_gpus = num_local_gpus

    def __call__(self, x):
        k, E, G = self.top_k, self.num_experts, self.num_local_gpus
        gates = O.softmax_op(self._logits(x))
        capacity = k * math.ceil((self.num_tokens / E) * self.capacity_factor)
        top1_group = O.topk_idx_op(O.sam_group_sum_op(gates, G), topk=1)
        topk_indices = O.group_topk_idx_op(gates, top1_group, topk=k, num_local_gpus=E // G)
        indices_s = [O.split_op(topk_indices, axes=[1], indices=[i], splits=[k]) for i in range(k)]
        masks = [O.array_reshape_op(O.one_hot_op(ix, num_classes=E), [-1, E]) for ix in indices_s]
        l_aux = balance_loss(gates, masks[0], E)
        for i in range(1, k):
            l_aux = O.add_op(l_aux, balance_loss(gates, masks[i], E))
        tmp = O.sam_max_op(gates, top1_group, indices_s[k - 1], E // G)
        l_align = O.reduce_sum_op(O.reduce_sum_op(tmp, axes=0), axes=0)
        location_s = _fused_locations(topk_indices, k, E)
        gates_s = [O.reduce_sum_op(O.mul_op(gates, m), axes=1) for m in masks]
        return l_aux, l_align, indices_s, location_s, gates_s, capacity


def generate_orthogonal(shape, gain=0.1, seed=0):
    rows, cols = shape[0], int(np.prod(shape[1:]))
    rng = np.random.RandomState(seed)
    flat = rng.normal(0, 1, (rows, cols))
    if rows < cols:
        flat = flat.T
    q, r = np.linalg.qr(flat)
    q = q * np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return (q * gain).astype(np.float32)


class BalanceAssignmentGate(_GateBase):
    """BASE layers: balanced assignment of tokens to expert centroids."""

    def __init__(self, embed_dim, num_tokens, num_experts, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='BalanceAssignment_Gate', device_id=None):
        super().__init__(embed_dim, num_tokens, num_experts, 1, capacity_factor, eval_capacity_factor,
                         initializer, name)
        self.device_id = device_id or 0
        self.expert_centroids = O.Variable(value=generate_orthogonal((num_experts, embed_dim)),
                                           name=name + '_centroids', trainable=False)

    def __call__(self, x):
        scores = O.matmul_op(x, self.expert_centroids, trans_B=True)
        indice = O.balance_assignment_op(scores)
        centroid = O.split_op(self.expert_centroids, axes=[0], indices=[self.device_id], splits=[self.num_experts])
        return indice, O.array_reshape_op(centroid, [-1, 1])


class DTSTemperature(object):
    """Annealing schedule of the Dense-To-Sparse gate: tau_t = max(tau_min, tau0 * decay^t).
    The executor steps it once per training step (``DTSGatingOp.on_step_end``)."""

    def __init__(self, tau0=2.0, tau_min=0.3, decay=0.999):
        self.tau0, self.tau_min, self.decay = tau0, tau_min, decay
        self.t = 0

    @property
    def value(self):
        return max(self.tau_min, self.tau0 * (self.decay ** self.t))

    def step(self):
        self.t += 1
        return self.value


class DenseToSparseGate(_GateBase):
    """Dense-To-Sparse gate (Nie et al., "Dense-to-Sparse Gate for Mixture-of-
    Experts", Hetu paper #6; reference README.md:123, routing as layers/moe_layer.py:60-88).
    A Gumbel-softmax gate whose temperature anneals once per training step: routing
    starts dense -- every expert active for every token, capacity for k = E -- and
    becomes sparse as the experts whose gate weight falls below ``threshold`` drop out;
    the expert budget (and the capacity, i.e. the all-to-all and expert GEMM sizes)
    follows the measured active count down to top-1 (``k_min``).  One fused HIP kernel
    computes noise, tempered softmax, threshold and the choices (ops.moe_dts).
    ``k``: kept for API compatibility with the other gates (the dense start is k = E)."""

    def __init__(self, embed_dim, num_tokens, num_experts, k=2, capacity_factor=1.0,
                 eval_capacity_factor=1.0, initializer=None, name='DTS_Gate', threshold=1e-3,
                 temperature=None, k_start=None, k_min=1):
        super().__init__(embed_dim, num_tokens, num_experts, k, capacity_factor, eval_capacity_factor,
                         initializer, name)
        self.threshold = threshold
        self.temperature = temperature or DTSTemperature()
        self.k_start, self.k_min = k_start, k_min
        self.gating = None

    def __call__(self, x):
        from ..ops.moe_dts import dts_gating_op
        l_aux, idx, loc, gates, capacity = dts_gating_op(
            self._logits(x), self.num_tokens, self.num_experts, self.temperature, self.threshold,
            self.capacity_factor, k_start=self.k_start, k_min=self.k_min)
        self.gating = gates
        return l_aux, [idx], [loc], [gates], capacity


class Expert(BaseLayer):
    """Two-layer FFN expert; parameter names start with ``expert`` (excluded
    from data-parallel all-reduce)."""

    def __init__(self, embed_dim, ffn_dim, dropout_rate=0.0, initializer=None, bias=False,
                 activation=None, name='expert'):
        self.embed_dim, self.ffn_dim = embed_dim, ffn_dim
        self.keep_prob = 1 - dropout_rate
        self.bias = bias
        self.activation = O.relu_op if activation == 'relu' else activation
        self.initializer = initializer or init.GenXavierUniform()
        self.name = name if name.startswith('expert') else 'expert_' + name

    def __call__(self, x):
        if not self.bias:
            h, w2 = self.hidden(x)
            return O.matmul_op(h, w2)
        w1 = self.initializer(shape=(self.embed_dim, self.ffn_dim), name=self.name + '_weight_1')
        w2 = self.initializer(shape=(self.ffn_dim, self.embed_dim), name=self.name + '_weight_2')
        x = O.array_reshape_op(x, [-1, self.embed_dim])
        b1 = init.zeros(shape=(self.ffn_dim,), name=self.name + '_bias_1')
        x = O.linear_op(x, w1, b1, activation='relu' if self.activation is O.relu_op else None)
        if self.activation is not None and self.activation is not O.relu_op:
            x = self.activation(x)
        if self.keep_prob < 1.0:
            x = O.dropout_op(x, self.keep_prob)
        b2 = init.zeros(shape=(self.embed_dim,), name=self.name + '_bias_2')
        return O.linear_op(x, w2, b2)

    def hidden(self, x):
        """bias-free expert: (the FFN's hidden activations [tokens, ffn], the second weight)
        -- the caller runs the second GEMM (alone, or as a row block of the local experts'
        concatenated output)"""
        assert not self.bias
        w1 = self.initializer(shape=(self.embed_dim, self.ffn_dim), name=self.name + '_weight_1')
        w2 = self.initializer(shape=(self.ffn_dim, self.embed_dim), name=self.name + '_weight_2')
        x = O.array_reshape_op(x, [-1, self.embed_dim])
        if self.activation is O.relu_op and self.keep_prob < 1.0:
            # ReLU and dropout in the first GEMM's epilogue (ops/linalg.py MatMulActDropoutOp)
            x = O.matmul_act_dropout_op(x, w1, 'relu', self.keep_prob)
        else:
            x = O.matmul_op(x, w1)
            if self.activation is not None:
                x = self.activation(x)
            if self.keep_prob < 1.0:
                x = O.dropout_op(x, self.keep_prob)
        return x, w2


# HETU_MOE_ROW_CONCAT=0: the local experts' outputs through a concatenation (A/B switch)
_ROW_CONCAT = os.environ.get('HETU_MOE_ROW_CONCAT', '1') == '1'


def _dispatch_and_run(layer, reshaped, indices_s, location_s, gates_s, capacity):
    n_local = layer.num_local_experts
    E = n_local * layer.all2all_size
    disp = O.layout_transform_op(reshaped, indices_s, location_s, capacity, E)
    disp = O.alltoall_op(disp)
    disp = O.array_reshape_op(disp, [layer.all2all_size, n_local, -1, layer.embed_dim])
    outs = []
    if _ROW_CONCAT and n_local > 1 and layer.all2all_size == 1 and all(isinstance(e, Expert) and not e.bias for e in layer.experts):
        # one process holds every expert: their second GEMMs write row blocks of one output
        # (concatenating [1, 1, C, d] pieces along axis 1 is a row concatenation)
        hs, w2s = zip(*(layer.experts[i].hidden(O.split_op(disp, axes=[1], indices=[i], splits=[n_local]))
                        for i in range(n_local)))
        y = O.row_concat_matmul_op(list(hs), list(w2s))
    else:
        for i in range(n_local):
            tok = O.split_op(disp, axes=[1], indices=[i], splits=[n_local])
            outs.append(O.array_reshape_op(layer.experts[i](tok), [layer.all2all_size, 1, -1, layer.embed_dim]))
        y = O.concatenate_op(outs, axis=1) if n_local > 1 else outs[0]
    y = O.alltoall_op(O.array_reshape_op(y, [-1, layer.embed_dim]))
    y = O.array_reshape_op(y, [-1, layer.embed_dim])
    if gates_s is None:
        return O.reverse_layout_transform_no_gate_op(y, indices_s, location_s, capacity, E)
    return O.reverse_layout_transform_op(y, indices_s, location_s, gates_s, capacity, E)


class MoELayer(BaseLayer):
    def __init__(self, gate=None, experts=None, num_tokens=None, embed_dim=None, all2all_size=None,
                 name='MoELayer', device_id=None, top=None):
        self.name, self.gate, self.experts = name, gate, experts
        self.num_local_experts = len(experts)
        self.num_tokens, self.embed_dim = num_tokens, embed_dim
        self.all2all_size = all2all_size or 1
        self.device_id, self.top = device_id or 0, top

    def __call__(self, x):
        reshaped = O.array_reshape_op(x, [-1, self.embed_dim])
        if self.name == 'BalanceAssignmentLayer' or isinstance(self.gate, BalanceAssignmentGate):
            return self._base_layer(reshaped)
        l_aux, indices_s, location_s, gates_s, capacity = self.gate(reshaped)
        return _dispatch_and_run(self, reshaped, indices_s, location_s, gates_s, capacity), l_aux

    def _base_layer(self, reshaped):
        indice, centroid = self.gate(reshaped)
        routed = O.indexing_op(reshaped, indice)
        routed = O.alltoall_op(routed)
        r4 = O.array_reshape_op(routed, [self.all2all_size, self.num_local_experts, -1, self.embed_dim])
        outs = [O.array_reshape_op(self.experts[i](O.split_op(r4, axes=[1], indices=[i], splits=[self.num_local_experts])),
                                   [-1, self.embed_dim]) for i in range(self.num_local_experts)]
        expert_out = O.concatenate_op(outs, axis=0) if len(outs) > 1 else outs[0]
        alpha = O.sigmoid_op(O.matmul_op(routed, centroid))
        mixed = O.add_op(O.mul_op(O.broadcastto_op(alpha, expert_out), expert_out),
                         O.mul_op(O.broadcastto_op(O.minus_byconst_op(alpha, 1.0), routed), routed))
        back = O.alltoall_op(mixed)
        return O.indexing_grad_op(back, indice)


class KTop1Layer(MoELayer):
    def __init__(self, gate=None, experts=None, num_tokens=None, embed_dim=None, all2all_size=None,
                 name='KTop1Layer', k=None):
        super().__init__(gate, experts, num_tokens, embed_dim, all2all_size, name, top=k)


class HashLayer(MoELayer):
    def __init__(self, gate=None, experts=None, num_tokens=None, embed_dim=None, all2all_size=None,
                 name='HashLayer'):
        super().__init__(gate, experts, num_tokens, embed_dim, all2all_size, name, top=1)

    def __call__(self, x, indice):
        reshaped = O.array_reshape_op(x, [-1, self.embed_dim])
        indices_s, location_s, capacity = self.gate(reshaped, indice)
        return _dispatch_and_run(self, reshaped, indices_s, location_s, None, capacity)


class SAMLayer(MoELayer):
    def __init__(self, gate=None, experts=None, num_tokens=None, embed_dim=None, all2all_size=None,
                 name='SAMLayer', k=None, num_local_gpus=8):
        super().__init__(gate, experts, num_tokens, embed_dim, all2all_size, name, top=k)
        self.num_local_gpus = num_local_gpus

    def __call__(self, x):
        reshaped = O.array_reshape_op(x, [-1, self.embed_dim])
        l_aux, l_align, indices_s, location_s, gates_s, capacity = self.gate(reshaped)
        return _dispatch_and_run(self, reshaped, indices_s, location_s, gates_s, capacity), l_aux, l_align
