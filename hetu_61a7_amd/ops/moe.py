"""MoE routing operators (reference LayoutTransform.py, ReverseLayoutTransform.py,
ReverseLayoutTransformNoGate.py, BalanceAssignment.py, SamGroupSum.py,
SamMax.py, GroupTopKIdx.py; SURVEY §2.4 "MoE routing", §3.6).

``indices_s``/``location_s``/``gates`` are the per-choice lists produced by the
gates (one node per top-k slot), exactly as in the reference layers.
Dispatch/combine are slot-indexed gathers (``kernels.moe``) -- deterministic,
no atomics on the forward combine.
"""
from __future__ import annotations

import os
import torch
from .. import native_array as _NA

from .node import Op
from ..kernels import moe as KM
from ..kernels import native as _native, record_fallback as _record_fallback
from ..kernels import tensor as KT


def _cap(c):
    """a capacity: an int, or an object whose ``value`` is read at every step (the
    dense-to-sparse gate's capacity follows its expert budget, ops.moe_dts.DTSCapacity)"""
    return int(c.value) if hasattr(c, 'value') else int(c)


def _keep(c):
    return c if hasattr(c, 'value') else int(c)


def _gpu(t):
    return isinstance(t, torch.Tensor) and _native(t) and t.dtype in (torch.float32, torch.bfloat16)


def _stack(vals):
    if len(vals) == 1 and vals[0].dim() == 2:
        return vals[0]          # already [T, k] (fused gate output)
    return torch.stack([v.reshape(-1) for v in vals], 1)


class LayoutTransformOp(Op):
    def __init__(self, x, indices_s, location_s, capacity, num_experts, ctx=None):
        indices_s = list(indices_s) if isinstance(indices_s, (list, tuple)) else [indices_s]
        location_s = list(location_s) if isinstance(location_s, (list, tuple)) else [location_s]
        super().__init__(LayoutTransformOp, [x] + indices_s + location_s, ctx)
        self.k = len(indices_s)
        self.capacity, self.num_experts = _keep(capacity), int(num_experts)

    def _idx(self, vals):
        k = self.k
        return _stack(vals[1:1 + k]), _stack(vals[1 + k:1 + 2 * k])

    def compute(self, input_vals, output_val=None, stream_handle=None):
        idx, loc = self._idx(input_vals)
        x = input_vals[0]
        return KM.layout_transform(x.reshape(x.shape[0], -1), idx, loc, _cap(self.capacity), self.num_experts)

    def gradient(self, output_grad):
        k = self.k
        g = LayoutTransformGradientOp(output_grad, self.inputs[1:1 + k], self.inputs[1 + k:1 + 2 * k],
                                      self.capacity, ctx=self.raw_ctx)
        return [g] + [None] * (2 * k)

    def infer_shape(self, input_shapes):
        return (self.num_experts * _cap(self.capacity), input_shapes[0][-1])


class LayoutTransformGradientOp(Op):
    def __init__(self, grad, indices_s, location_s, capacity, ctx=None):
        indices_s = list(indices_s) if isinstance(indices_s, (list, tuple)) else [indices_s]
        location_s = list(location_s) if isinstance(location_s, (list, tuple)) else [location_s]
        super().__init__(LayoutTransformGradientOp, [grad] + indices_s + location_s, ctx)
        self.k, self.capacity = len(indices_s), _keep(capacity)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        k = self.k
        idx, loc = _stack(input_vals[1:1 + k]), _stack(input_vals[1 + k:1 + 2 * k])
        return KM.layout_transform_backward(input_vals[0], idx, loc, _cap(self.capacity))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def layout_transform_op(input, indices_s, location_s, capacity, total_experts, ctx=None):
    return LayoutTransformOp(input, indices_s, location_s, capacity, total_experts, ctx=ctx)


def layout_transform_gradient_op(input, indice, location, capacity, ctx=None):
    return LayoutTransformGradientOp(input, indice, location, capacity, ctx=ctx)


class ReverseLayoutTransformOp(Op):
    """Gate-weighted combine of expert outputs back to token order."""

    def __init__(self, y, indices_s, location_s, gates, capacity, num_experts, ctx=None):
        indices_s = list(indices_s) if isinstance(indices_s, (list, tuple)) else [indices_s]
        location_s = list(location_s) if isinstance(location_s, (list, tuple)) else [location_s]
        gates = (list(gates) if isinstance(gates, (list, tuple)) else [gates]) if gates is not None else []
        super().__init__(ReverseLayoutTransformOp, [y] + indices_s + location_s + gates, ctx)
        self.k = len(indices_s)
        self.has_gate = len(gates) > 0
        self.capacity, self.num_experts = _keep(capacity), int(num_experts)

    def _parts(self, vals):
        k = self.k
        idx = _stack(vals[1:1 + k])
        loc = _stack(vals[1 + k:1 + 2 * k])
        gates = _stack(vals[1 + 2 * k:1 + 3 * k]) if self.has_gate else None
        return idx, loc, gates

    def compute(self, input_vals, output_val=None, stream_handle=None):
        idx, loc, gates = self._parts(input_vals)
        return KM.reverse_layout_transform(input_vals[0], idx, loc, gates, _cap(self.capacity))

    def gradient(self, output_grad):
        k = self.k
        ins = self.inputs
        if self.has_gate and k == 1 and _FUSED_COMBINE_BWD:
            # one [T, k] index tensor: both gradients from one kernel reading output_grad once
            gd = ReverseLayoutTransformGradientDataOp(output_grad, ins[1:2], ins[2:3], ins[3:4], self.capacity,
                                                      self.num_experts, ctx=self.raw_ctx, y=ins[0])
            return [gd, None, None, CombineGateGradOp(gd, ins[1], ctx=self.raw_ctx)]
        gd = ReverseLayoutTransformGradientDataOp(output_grad, ins[1:1 + k], ins[1 + k:1 + 2 * k],
                                                  ins[1 + 2 * k:1 + 3 * k] if self.has_gate else None,
                                                  self.capacity, self.num_experts, ctx=self.raw_ctx)
        grads = [gd] + [None] * (2 * k)
        if self.has_gate:
            for j in range(k):
                grads.append(ReverseLayoutTransformGradientGateOp(output_grad, ins[0], ins[1 + j], ins[1 + k + j],
                                                                  self.capacity, ctx=self.raw_ctx))
        return grads

    def infer_shape(self, input_shapes):
        return (input_shapes[1][0], input_shapes[0][-1])


class ReverseLayoutTransformGradientDataOp(Op):
    """Expert-slot gradient of the combine.  ``y`` (the combined expert outputs; one [T, k]
    index tensor): also the gate gradient, as the aux value read by a CombineGateGradOp --
    one kernel reads the token gradient once for both."""

    def __init__(self, grad, indices_s, location_s, gates, capacity, num_experts, ctx=None, y=None):
        indices_s = list(indices_s) if isinstance(indices_s, (list, tuple)) else [indices_s]
        location_s = list(location_s) if isinstance(location_s, (list, tuple)) else [location_s]
        gates = (list(gates) if isinstance(gates, (list, tuple)) else [gates]) if gates is not None else []
        super().__init__(ReverseLayoutTransformGradientDataOp,
                         [grad] + indices_s + location_s + gates + ([y] if y is not None else []), ctx)
        self.k, self.has_gate = len(indices_s), len(gates) > 0
        self.with_gate_grad = y is not None
        self.capacity, self.num_experts = _keep(capacity), int(num_experts)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from .nn import AuxResult
        k = self.k
        idx, loc = _stack(input_vals[1:1 + k]), _stack(input_vals[1 + k:1 + 2 * k])
        gates = _stack(input_vals[1 + 2 * k:1 + 3 * k]) if self.has_gate else None
        cap = _cap(self.capacity)
        if self.with_gate_grad:
            d, dg = KM.reverse_layout_transform_backward_fused(input_vals[0], input_vals[-1], idx, loc, gates, cap,
                                                               cap * self.num_experts)
            return AuxResult(d, dg)
        return KM.reverse_layout_transform_backward_data(input_vals[0], idx, loc, gates, cap, cap * self.num_experts)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return (_cap(self.capacity) * self.num_experts, input_shapes[0][-1])


class CombineGateGradOp(Op):
    """The gate gradient computed by a fused ReverseLayoutTransformGradientDataOp (its aux)"""
    aux_inputs = (0,)
    shape_only_inputs = (1,)

    def __init__(self, data_grad, indices, ctx=None):
        super().__init__(CombineGateGradOp, [data_grad, indices], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0].reshape(tuple(input_vals[1]))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


_FUSED_COMBINE_BWD = os.environ.get('HETU_MOE_FUSED_COMBINE_BWD', '1') != '0'


class ReverseLayoutTransformGradientGateOp(Op):
    def __init__(self, grad, y, indices, locations, capacity, ctx=None):
        super().__init__(ReverseLayoutTransformGradientGateOp, [grad, y, indices, locations], ctx)
        self.capacity = _keep(capacity)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, y, idx, loc = input_vals
        if idx.dim() != 2:
            idx, loc = idx.reshape(-1, 1), loc.reshape(-1, 1)
        return KM.reverse_layout_transform_backward_gate(g, y, idx, loc, _cap(self.capacity)).reshape(input_vals[2].shape)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def reverse_layout_transform_op(input, indices_s, location_s, gates, capacity, num_experts, ctx=None):
    return ReverseLayoutTransformOp(input, indices_s, location_s, gates, capacity, num_experts, ctx=ctx)


def reverse_layout_transform_gradient_data_op(input, indices, locations, gates, capacity, num_experts, ctx=None):
    return ReverseLayoutTransformGradientDataOp(input, indices, locations, gates, capacity, num_experts, ctx=ctx)


def reverse_layout_transform_gradient_gate_op(combined_output, expert_output, indices, locations, capacity, ctx=None):
    return ReverseLayoutTransformGradientGateOp(combined_output, expert_output, indices, locations, capacity, ctx=ctx)


def reverse_layout_transform_no_gate_op(input, indices_s, location_s, capacity, num_experts, ctx=None):
    return ReverseLayoutTransformOp(input, indices_s, location_s, None, capacity, num_experts, ctx=ctx)


def reverse_layout_transform_no_gate_gradient_op(input, indices, locations, capacity, num_experts, ctx=None):
    return ReverseLayoutTransformGradientDataOp(input, indices, locations, None, capacity, num_experts, ctx=ctx)


class BalanceAssignmentOp(Op):
    """BASE-layer balanced token->expert assignment (auction algorithm,
    reference BalanceAssignment.py:11-85) run on device: returns for each
    expert the indices of the tokens assigned to it ([E, T/E])."""

    def __init__(self, scores, max_iterations=100, ctx=None):
        super().__init__(BalanceAssignmentOp, [scores], ctx)
        self.max_iterations = max_iterations

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.moe import balanced_assignment
        return balanced_assignment(input_vals[0], self.max_iterations)

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        T, E = input_shapes[0]
        return (T,)


def balance_assignment_op(node, ctx=None):
    return BalanceAssignmentOp(node, ctx=ctx)


class SamGroupSumOp(Op):
    """Sum of gate probabilities per GPU group ([T, E] -> [T, G])."""

    def __init__(self, gate, num_local_gpus, ctx=None):
        super().__init__(SamGroupSumOp, [gate], ctx)
        self.num_local_gpus = num_local_gpus

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g = input_vals[0]
        T, E = g.shape
        G = self.num_local_gpus
        if _gpu(g):
            return KT.sam_group_sum(g, G)
        return g.float().reshape(T, G, E // G).sum(-1)

    def gradient(self, output_grad):
        return [SamGroupSumGradOp(output_grad, self.inputs[0], self.num_local_gpus, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], self.num_local_gpus)


class SamGroupSumGradOp(Op):
    shape_only_inputs = (1,)

    def __init__(self, grad, ref, num_local_gpus, ctx=None):
        super().__init__(SamGroupSumGradOp, [grad, ref], ctx)
        self.num_local_gpus = num_local_gpus

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, shape = input_vals
        T, E = tuple(shape)
        G = self.num_local_gpus
        if _gpu(g):
            return KT.sam_group_sum_grad(g, T, E, G)
        return g.float().unsqueeze(-1).expand(T, G, E // G).reshape(T, E)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def sam_group_sum_op(node, num_local_gpus, ctx=None):
    return SamGroupSumOp(node, num_local_gpus, ctx=ctx)


def _sam_mask(x, top1_group, topk_idx, n):
    T, E = x.shape
    g = top1_group.reshape(-1).long()
    cols = torch.arange(E, device=x.device).unsqueeze(0)
    outside = (cols < (g * n).unsqueeze(1)) | (cols >= ((g + 1) * n).unsqueeze(1))
    ref = torch.gather(x.float(), 1, topk_idx.reshape(-1, 1).long())
    diff = x.float() - ref
    return outside & (diff > 0), diff


class SamMaxOp(Op):
    """SAM alignment loss: max(0, g_j - g_topk) for experts outside the chosen group."""

    def __init__(self, gates, top1_group, topk_idx, num_local_gpus, ctx=None):
        super().__init__(SamMaxOp, [gates, top1_group, topk_idx], ctx)
        self.num_local_gpus = num_local_gpus

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, grp, tk = input_vals
        if _gpu(x):
            return KT.sam_max(x, grp, tk, self.num_local_gpus)
        m, diff = _sam_mask(x, grp, tk, self.num_local_gpus)
        return torch.where(m, diff, _NA.zeros_like(diff))

    def gradient(self, output_grad):
        return [sammax_grad_op(output_grad, self.inputs[0], self.inputs[1], self.inputs[2], self.num_local_gpus,
                               ctx=self.raw_ctx), None, None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class SamMaxGradOp(Op):
    def __init__(self, grad, gates, top1_group, topk_idx, num_local_gpus, ctx=None):
        super().__init__(SamMaxGradOp, [grad, gates, top1_group, topk_idx], ctx)
        self.num_local_gpus = num_local_gpus

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, x, grp, tk = input_vals
        if _gpu(x):
            return KT.sam_max_grad(g, x, grp, tk, self.num_local_gpus)
        m, _ = _sam_mask(x, grp, tk, self.num_local_gpus)
        gm = torch.where(m, g.float(), _NA.zeros_like(g, dtype=torch.float32))
        out = gm.clone()
        out.scatter_add_(1, tk.reshape(-1, 1).long(), -gm.sum(1, keepdim=True))
        return out

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def sam_max_op(node_A, node_B, node_C, num_local_gpus, ctx=None):
    return SamMaxOp(node_A, node_B, node_C, num_local_gpus, ctx=ctx)


def sammax_grad_op(node_A, node_B, node_C, node_D, num_local_gpus, ctx=None):
    return SamMaxGradOp(node_A, node_B, node_C, node_D, num_local_gpus, ctx=ctx)


class GroupTopKIdxOp(Op):
    """Top-k expert ids restricted to the group chosen per row (reference
    GroupTopKIdx.cu: group g spans experts [g*n, (g+1)*n))."""

    def __init__(self, x, top1_group, topk=1, num_local_gpus=8, ctx=None):
        super().__init__(GroupTopKIdxOp, [x, top1_group], ctx)
        self.k, self.num_local_gpus = topk, num_local_gpus

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, grp = input_vals
        n = self.num_local_gpus
        if _gpu(x):
            r = KT.group_topk_idx(x, grp, self.k, n)
            if r is not None:
                return r
            _record_fallback('group_topk_idx')
        g = grp.reshape(-1).long()
        T, E = x.shape
        cols = torch.arange(E, device=x.device).unsqueeze(0)
        inside = (cols >= (g * n).unsqueeze(1)) & (cols < ((g + 1) * n).unsqueeze(1))
        masked = torch.where(inside, x.float(), torch.full_like(x, -1e4, dtype=torch.float32))
        return torch.topk(masked, self.k, dim=1)[1]

    def gradient(self, output_grad):
        return [None, None]

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], self.k)


def group_topk_idx_op(node_A, node_B, topk, num_local_gpus, ctx=None):
    return GroupTopKIdxOp(node_A, node_B, topk, num_local_gpus, ctx=ctx)


# ---------------------------------------------------------------------------
# Fused top-k gate (MI355X path of reference TopGate.py:7-79): softmax, top-k,
# capacity slots and the balance-loss terms in two kernels instead of the
# ~6k-node softmax/topk/one_hot/cumsum/reduce chain.
class TopKGatingOp(Op):
    """value: gate weights [T, k] (softmax prob of each chosen expert);
    aux: (probs [T, E], indices [T, k] int64, locations [T, k] int64, l_aux)."""

    def __init__(self, logits, k, capacity, num_experts, ctx=None):
        super().__init__(TopKGatingOp, [logits], ctx)
        self.k, self.capacity, self.num_experts = int(k), int(capacity), int(num_experts)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from .nn import AuxResult
        logits = input_vals[0]
        T, E = logits.shape
        val, idx, probs = KM.topk(logits, self.k, softmax=True)
        loc, counts, psum = KM.locations(idx, E, probs)
        # coef_e = mean_t mask[t, e] summed over choices; l_aux = E * sum_e coef_e * mean_t probs[t, e]
        coef, l_aux = KM.aux_terms(counts, psum, T)
        return AuxResult(val, (probs, idx, loc, l_aux, coef))

    def gradient(self, output_grad):
        return [TopKGatingGradOp(output_grad, self, None, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0], self.k)


class TopKGatingGradOp(Op):
    """d logits from d gate weights (``grad`` [T, k]) or from d l_aux (scalar,
    ``aux_grad``): one fused softmax backward per token."""
    value_and_aux_inputs = (1,)

    def __init__(self, grad, gating, aux_grad, ctx=None):
        ins = [grad if grad is not None else aux_grad, gating]
        super().__init__(TopKGatingGradOp, ins, ctx)
        self.is_aux = grad is None

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, (val, aux) = input_vals
        probs, idx, loc, l_aux, coef = aux[:5]
        scale = aux[5] if len(aux) > 5 else 1.0     # 1 / tau of the dense-to-sparse gate
        T, E = probs.shape
        if self.is_aux:
            # l_aux = E * sum_e coef_e * sum_t probs[t, e] / T
            if coef.is_cuda:
                from ..kernels.elementwise import binary, unary
                gs = g.reshape(-1)[:1]          # the scalar d l_aux, read in place (scalar mode)
                c = binary('mul', unary('mul_c', coef, float(E) / float(T)), gs)
            else:
                c = coef * (float(E) / float(T)) * g.float().reshape(-1)[0]
            return KM.gate_backward(probs, idx, None, c, scale)
        return KM.gate_backward(probs, idx, g, None, scale)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


class GatingSelectOp(Op):
    """indices / locations / l_aux of a fused gate."""
    value_and_aux_inputs = (0,)
    _slot = {'indices': 1, 'locations': 2, 'l_aux': 3}

    def __init__(self, gating, what, ctx=None):
        super().__init__(GatingSelectOp, [gating], ctx)
        self.what = what
        self.gating = gating

    def compute(self, input_vals, output_val=None, stream_handle=None):
        val, aux = input_vals[0]
        r = aux[self._slot[self.what]]
        return r.reshape(1) if self.what == 'l_aux' else r

    def gradient(self, output_grad):
        if self.what != 'l_aux':
            return [None]
        return [None]   # routed to the logits by TopKGatingAuxGrad (see topk_gating_op)

    def infer_shape(self, input_shapes):
        T, k = input_shapes[0]
        return (1,) if self.what == 'l_aux' else (T, k)


class AuxLossOp(Op):
    """l_aux of a fused gate, differentiable wrt the gate logits."""
    value_and_aux_inputs = (0,)

    def __init__(self, gating, logits, ctx=None):
        super().__init__(AuxLossOp, [gating, logits], ctx)
        self.gating = gating

    def compute(self, input_vals, output_val=None, stream_handle=None):
        val, aux = input_vals[0]
        return aux[3].reshape(1)

    def gradient(self, output_grad):
        return [None, TopKGatingGradOp(None, self.gating, output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return (1,)


def topk_gating_op(logits, k, capacity, num_experts, ctx=None):
    """Returns (l_aux, indices [T,k], locations [T,k], gates [T,k]) nodes."""
    g = TopKGatingOp(logits, k, capacity, num_experts, ctx=ctx)
    return (AuxLossOp(g, logits, ctx=ctx), GatingSelectOp(g, 'indices', ctx=ctx),
            GatingSelectOp(g, 'locations', ctx=ctx), g)


class TopKLocationsOp(Op):
    """Slot of every (token, choice) inside its expert's capacity from top-k
    indices [T, k] (choice-major, as the reference's one_hot/cumsum/mul/reduce
    chain of TopGate.py): one native counting pass instead of a column scan."""

    def __init__(self, indices, num_experts, ctx=None):
        super().__init__(TopKLocationsOp, [indices], ctx)
        self.num_experts = int(num_experts)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        idx = input_vals[0]
        idx = idx.reshape(idx.shape[0], -1)
        loc, _, _ = KM.locations(idx, self.num_experts)
        return loc

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def topk_locations_op(indices, num_experts, ctx=None):
    return TopKLocationsOp(indices, num_experts, ctx=ctx)
