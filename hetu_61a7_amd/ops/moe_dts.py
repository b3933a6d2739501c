"""Ops of the Dense-To-Sparse MoE gate (Nie et al., "Dense-to-Sparse Gate for
Mixture-of-Experts", Hetu README paper #6 -- cited by the reference at README.md:123
but absent from its code; routing structure of the reference's
layers/moe_layer.py:60-88 and examples/moe/test_moe_top.py:42-53).

The fused gate (``dts_gating_op``, HIP kernel ``moe.hip dts_gate_k``):

  y = softmax((logits + gumbel) / tau)        gumbel from Philox(seed, t * E + e)
  choices: the ``budget`` largest y per token; choice j > 0 is active only while
  y >= threshold (inactive choices carry idx -1: no capacity, no compute, no gradient)

Training starts dense -- the budget is every expert (k = E, capacity for k = E: no
token is dropped) and the high temperature spreads y over all of them -- and becomes
sparse as tau anneals (``DTSTemperature``, stepped once per training step by the
executor): fewer experts stay above the threshold, and the budget (with the expert
capacity, i.e. the all-to-all and expert GEMM sizes) follows the measured number of
active experts per token down to top-1.  The histogram of active choices is read two
steps late (no host sync in the step) and, on several ranks, all-reduced first, so
every rank takes the same budget (the all-to-all needs one capacity).
"""
from __future__ import annotations

import math

import torch
from .. import native_array as _NA

from .node import Op
from .nn import AuxResult
from ..kernels import moe as KM


def _world():
    try:
        from ..parallel import comm as C
        w = C.world()
        return w if w is not None and getattr(w, 'nrank', 1) > 1 else None
    except Exception:
        return None


class DTSCapacity(object):
    """capacity of each expert for the gate's current budget: budget * ceil(T / E * cf)
    (int-like; the MoE dispatch / combine ops read ``value`` at every step)"""

    def __init__(self, gating, num_tokens, num_experts, capacity_factor):
        self.gating = gating
        self.per_choice = int(math.ceil((num_tokens / num_experts) * capacity_factor))

    @property
    def value(self):
        return int(self.gating.budget) * self.per_choice

    def __int__(self):
        return self.value

    def __index__(self):
        return self.value


class DTSGatingOp(Op):
    """value: gate weights [T, budget] (y of each active choice, 0 for inactive ones);
    aux: (probs [T, E], idx [T, budget] int64 (-1 inactive), loc [T, budget] int64,
    l_aux, balance coefficients [E], 1 / tau) -- the aux layout of the fused top-k gate,
    so its gradient op (TopKGatingGradOp, scaled by 1 / tau) and selectors are shared."""

    def __init__(self, logits, num_experts, temperature, threshold=1e-3, k_start=None, k_min=1,
                 drop_frac=1e-3, ctx=None):
        super().__init__(DTSGatingOp, [logits], ctx)
        self.num_experts = int(num_experts)
        self.temperature = temperature
        self.threshold = float(threshold)
        self.k_max = min(int(k_start or num_experts), self.num_experts, KM.MAX_K)
        self.k_min = max(1, min(int(k_min), self.k_max))
        self.budget = self.k_max
        self.drop_frac = float(drop_frac)
        self.inference = False
        self.k = self.k_max            # TopKGating-compatible attribute (static upper bound)
        self.calls = 0
        self._pending = []             # (call index, host histogram, event) of earlier steps
        self._tau_at = {}
        self.history = []              # (call, tau, budget, mean active experts per token)

    # -- budget from the measured active-expert histogram, two calls late -----------------
    LAG = 2

    def _update_budget(self):
        while self._pending and self._pending[0][0] <= self.calls - self.LAG:
            call, h, ev = self._pending.pop(0)
            if ev is not None:
                ev.synchronize()
            hist = [int(v) for v in h.tolist()]
            tot = sum(hist)
            if tot <= 0:
                continue
            mean = sum(n * c for n, c in enumerate(hist)) / float(tot)
            self.history.append((call, self._tau_at.get(call, float('nan')), len(hist) - 1, mean))
            self._tau_at.pop(call, None)
            allow = self.drop_frac * tot
            need = len(hist) - 1
            over = 0
            while need > self.k_min and over + hist[need] <= allow:
                over += hist[need]
                need -= 1
            self.budget = max(self.k_min, min(self.budget, need))

    def compute(self, input_vals, output_val=None, stream_handle=None):
        logits = input_vals[0]
        T = logits.numel() // self.num_experts
        x = logits.reshape(T, self.num_experts)
        train = not self.inference
        if train:
            self._update_budget()
        tau = float(self.temperature.value)
        from .nn import _next_seed
        seed = _next_seed(self.id, x) if train else 0
        val, idx, probs, hist = KM.dts_gate(x, self.budget, 1.0 / tau, self.threshold, seed, noise=train)
        loc, counts, psum = KM.locations(idx, self.num_experts, probs, inactive=True)
        coef, l_aux = KM.aux_terms(counts, psum, T)
        if train:
            w = _world()
            if w is not None and hist.is_cuda:
                w.all_reduce(hist, 'sum')     # one budget on every rank (one all-to-all capacity)
            if hist.is_cuda:
                from ..runtime import DeviceEvent
                h = _NA.empty(hist.shape, dtype=hist.dtype, pin_memory=True)
                h.copy_(hist, non_blocking=True)
                ev = DeviceEvent(hist.device.index).record()
            else:
                h, ev = hist.clone(), None
            self._pending.append((self.calls, h, ev))
            self._tau_at[self.calls] = tau
            self.calls += 1
        return AuxResult(val, (probs, idx, loc, l_aux, coef, 1.0 / tau))

    def on_step_end(self):
        """one training step done (executor hook): anneal the temperature"""
        if not self.inference:
            self.temperature.step()

    def gradient(self, output_grad):
        from .moe import TopKGatingGradOp
        return [TopKGatingGradOp(output_grad, self, None, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], self.budget)

    def active_experts(self):
        """mean active experts per token of the latest step whose histogram was read"""
        return self.history[-1][3] if self.history else float(self.k_max)


def dts_gating_op(logits, num_tokens, num_experts, temperature, threshold=1e-3, capacity_factor=1.0,
                  k_start=None, k_min=1, ctx=None):
    """Returns (l_aux, indices [T, k], locations [T, k], gates [T, k], capacity) nodes /
    objects of the fused dense-to-sparse gate (``capacity`` follows the budget)."""
    from .moe import AuxLossOp, GatingSelectOp
    g = DTSGatingOp(logits, num_experts, temperature, threshold, k_start, k_min, ctx=ctx)
    cap = DTSCapacity(g, num_tokens, num_experts, capacity_factor)
    return (AuxLossOp(g, logits, ctx=ctx), GatingSelectOp(g, 'indices', ctx=ctx),
            GatingSelectOp(g, 'locations', ctx=ctx), g, cap)


# ---- standalone Gumbel-softmax and threshold-mask ops (public graph API) ----------------
class GumbelSoftmaxOp(Op):
    """softmax((logits + g) / tau), g ~ Gumbel(0, 1) from Philox; tau read from the
    schedule object (``temperature.value``) at every call.  Forward on the fused DTS gate
    kernel (its probabilities), backward on the native softmax-backward kernel."""

    def __init__(self, logits, temperature, ctx=None):
        super().__init__(GumbelSoftmaxOp, [logits], ctx)
        self.temperature = temperature
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        E = x.shape[-1]
        tau = float(self.temperature.value)
        from .nn import _next_seed
        seed = _next_seed(self.id, x) if not self.inference else 0
        _, _, probs, _ = KM.dts_gate(x.reshape(-1, E), 1, 1.0 / tau, 0.0, seed, noise=not self.inference)
        return AuxResult(probs.reshape(x.shape), tau)

    def gradient(self, output_grad):
        return [GumbelSoftmaxGradOp(self, output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class GumbelSoftmaxGradOp(Op):
    value_and_aux_inputs = (0,)

    def __init__(self, fwd, grad, ctx=None):
        super().__init__(GumbelSoftmaxGradOp, [fwd, grad], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        (y, tau), g = input_vals
        from ..kernels.softmax import softmax_backward
        from ..kernels.elementwise import unary
        g = g.reshape(y.shape)
        if g.dtype != y.dtype:
            from ..kernels.elementwise import cast
            g = cast(g.contiguous(), y.dtype)
        return unary('mul_c', softmax_backward(y, g.contiguous()), 1.0 / tau)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def gumbel_softmax_op(logits, temperature, ctx=None):
    return GumbelSoftmaxOp(logits, temperature, ctx=ctx)


def _below(threshold):
    """largest float32 strictly below ``threshold``: x > it  <=>  x >= threshold"""
    import numpy as np
    return float(np.nextafter(np.float32(threshold), np.float32(-np.inf)))


class ThresholdMaskOp(Op):
    """x * (x >= threshold): drops experts whose gate weight is negligible (native
    compare + multiply kernels)."""

    def __init__(self, x, threshold, ctx=None):
        super().__init__(ThresholdMaskOp, [x], ctx)
        self.threshold = threshold

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.elementwise import unary, binary
        x = input_vals[0]
        return binary('mul', x, unary('gt_c', x, _below(self.threshold)))

    def gradient(self, output_grad):
        return [ThresholdMaskGradOp(output_grad, self.inputs[0], self.threshold, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class ThresholdMaskGradOp(Op):
    def __init__(self, g, x, threshold, ctx=None):
        super().__init__(ThresholdMaskGradOp, [g, x], ctx)
        self.threshold = threshold

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.elementwise import unary, binary
        g, x = input_vals
        g = g.reshape(x.shape)
        m = unary('gt_c', x, _below(self.threshold))
        if m.dtype != g.dtype:
            from ..kernels.elementwise import cast
            m = cast(m.contiguous(), g.dtype)
        return binary('mul', g, m)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def threshold_mask_op(x, threshold, ctx=None):
    return ThresholdMaskOp(x, threshold, ctx=ctx)
