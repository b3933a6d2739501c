"""Forward-graph fusion pass, run by ``Optimizer.minimize`` before autodiff.

Rewrites (in place, preserving the identity of the user-visible output node):
  relu(batch_norm(x))             -> fused BN+ReLU          (one pass fwd, one bwd)
  relu(batch_norm(x) + r)         -> fused BN+add+ReLU      (ResNet block tail)
  relu(r + batch_norm(x))         -> fused BN+add+ReLU
  batch_norm(conv2d(x, w))        -> the conv epilogue also emits the per-channel
                                     sum / sum of squares of its output, so the BN
                                     skips its statistics pass (training mode;
                                     HETU_FUSE_BN_STATS=0 turns it off)
These are the memory-bound op chains that dominate ResNet time outside the
convolutions; the reference runs each as its own cuDNN/elementwise call.
Only applied when the intermediate values have no other consumer.

Backward (``fuse_backward``, run on the gradient graph):
  sum(conv_dgrad(w, g), r, ...)   -> conv_dgrad accumulating r in its epilogue
                                     (the residual-branch gradient join of ResNet)
  sum(matmul(g, w^T), r, ...)     -> matmul with r added in the GEMM epilogue
                                     (beta = 1; the transformer residual-stream join)
  reduce_sum_axis0(gelu_grad(...))  -> the GELU-gradient kernel also emits the
                                     bias gradient (column sums) of the GELU linear
  reduce_sum_axis0(d x) where x feeds a fused dropout+add+LayerNorm
                                  -> the LayerNorm backward kernel emits that bias
                                     gradient of the producing linear layer
  bn_backward(conv_dgrad(w, g), x) -> the dgrad epilogue also accumulates the BN
                                     backward's per-channel reduction (sum dy',
                                     sum dy'*x), removing its pass over dy and x
"""
from __future__ import annotations

import os

from .ops.node import Op


def _consumers(roots):
    from .ops.executor import find_topo_sort
    topo = find_topo_sort(roots)
    cons = {n: [] for n in topo}
    for n in topo:
        for i in n.inputs:
            cons.setdefault(i, []).append(n)
    return topo, cons


def fuse_forward(roots):
    if os.environ.get('HETU_FUSE', '1') == '0':
        return 0
    from .ops.basic import ReluOp, AddOp
    from .ops.nn import Batch_NormalizationOp
    topo, cons = _consumers(roots)
    root_set = set(roots)
    fused = 0
    for n in topo:
        if not isinstance(n, ReluOp) or n in root_set:
            continue
        src = n.inputs[0]
        if isinstance(src, Batch_NormalizationOp) and not src.relu and not src.has_residual \
                and len(cons.get(src, [])) == 1 and src not in root_set:
            _become_bn(n, src, relu=True, residual=None)
            fused += 1
        elif isinstance(src, AddOp) and len(cons.get(src, [])) == 1 and src not in root_set:
            a, b = src.inputs
            for bn, res in ((a, b), (b, a)):
                if isinstance(bn, Batch_NormalizationOp) and not bn.relu and not bn.has_residual \
                        and len(cons.get(bn, [])) == 1 and bn not in root_set and bn is not res:
                    _become_bn(n, bn, relu=True, residual=res)
                    fused += 1
                    break
    # conv -> BatchNorm: the conv hands the BN the statistics of its output (computed
    # in the conv epilogue), removing the BN's separate statistics pass over it
    # default since the totals are spread over replicas (conv_igemm.bn_sum_replicas): with
    # one [2C] target thousands of blocks serialised on its atomics and the fusion
    # measured neutral to -1.6% (profiles/bn_stats_fusion_r2p.md); with replicas
    # ResNet-50 bs256 10072 vs 9907 img/s without, same box
    # (profiles/bench_resnet50_r4_bn11_rep.json, bench_resnet50_r4_bn10_rep.json)
    from .kernels import deterministic
    if os.environ.get('HETU_FUSE_BN_STATS', '1') != '1' or deterministic():   # fp32 atomics
        return fused
    from .ops.nn import Conv2dOp
    topo, cons = _consumers(roots)
    for n in topo:
        if isinstance(n, Conv2dOp) and n not in root_set:
            users = cons.get(n, [])
            if len(users) == 1 and isinstance(users[0], Batch_NormalizationOp) and users[0].inputs[0] is n:
                n.emit_bn_stats = True
                fused += 1
    return fused


def _become_bn(node, bn, relu, residual):
    """Turn ``node`` (a ReluOp) into a fused BN op with bn's inputs/attributes."""
    from .ops.nn import Batch_NormalizationOp
    keep_id, keep_name = node.id, node.name
    node.__class__ = Batch_NormalizationOp
    node.__dict__.update({k: v for k, v in bn.__dict__.items() if k not in ('id', 'name', 'inputs')})
    node.inputs = list(bn.inputs[:3]) + ([residual] if residual is not None else [])
    node.relu = relu
    node.has_residual = residual is not None
    node.op_type = 'Batch_NormalizationOp'
    node.id, node.name = keep_id, keep_name
    node.running_mean = bn.running_mean
    node.running_var = bn.running_var
    node.fused_from = bn


# gradient ops whose value is always a new tensor (never a view of an input)
_FRESH_OUTPUT = ('BNGradSelectOp', 'Conv2d_Gradient_of_DataOp', 'SumOp')


def _dead_join_operand(other, rest, cons, root_set):
    """True when the join operand may be overwritten in place (the library GEMM then
    accumulates into it: beta = 1, C == D, no copy into a fresh output): this join
    is its only consumer and its op always hands out a freshly allocated tensor."""
    if other in root_set:
        return False
    return len(rest) > 1 or (len(cons.get(other, [])) == 1 and type(other).__name__ in _FRESH_OUTPUT)


def fuse_backward(roots):
    """Fold gradient fan-in sums into the data-gradient GEMM epilogue."""
    if os.environ.get('HETU_FUSE', '1') == '0':
        return 0
    from .ops.reduce import SumOp, ReduceSumAxisZeroOp
    from .ops.nn import Conv2d_Gradient_of_DataOp, DropoutAddLayerNormGradientOp, BNGradSelectOp
    from .ops.linalg import MatMulOp, LinearGeluGradOp, LinearGeluBiasGradOp
    topo, cons = _consumers(roots)
    root_set = set(roots)
    fused = 0
    # bias gradient of a GELU linear layer = row sum of its GELU gradient: summed by
    # the GELU-gradient kernel itself
    for n in topo:
        if type(n) is ReduceSumAxisZeroOp and len(n.inputs) == 1 and type(n.inputs[0]) is LinearGeluGradOp \
                and not n.inputs[0].emit_colsum:
            lg = n.inputs[0]
            lg.emit_colsum = True
            keep_id, keep_name, bw = n.id, n.name, getattr(n, 'bw_of', None)
            n.__class__ = LinearGeluBiasGradOp
            n.inputs = [lg]
            n.op_type = 'LinearGeluBiasGradOp'
            n.id, n.name = keep_id, keep_name
            if bw is not None:
                n.bw_of = bw
            fused += 1
    # linear bias gradient = row sum of the x-gradient of a fused dropout+add+LayerNorm:
    # the LayerNorm backward kernel sums it in its own row pass (no reduction over dx)
    for n in topo:
        if type(n) is not ReduceSumAxisZeroOp or len(n.inputs) != 1:
            continue
        s = n.inputs[0]
        if type(s) is BNGradSelectOp and s.index == 0 and \
                type(s.inputs[0]) is DropoutAddLayerNormGradientOp and not s.inputs[0].emit_lin_bias:
            gn = s.inputs[0]
            gn.emit_lin_bias = True
            keep_id, keep_name, bw = n.id, n.name, getattr(n, 'bw_of', None)
            n.__class__ = BNGradSelectOp
            n.inputs = [gn]
            n.index = 4
            n.op_type = 'DropoutAddLayerNorm_Gradient_of_LinearBiasOp'
            n.id, n.name = keep_id, keep_name
            if bw is not None:
                n.bw_of = bw
            fused += 1
    for n in topo:
        if not isinstance(n, SumOp) or len(n.inputs) < 2 or getattr(n, 'sparse', False):
            continue
        mm = [d for d in n.inputs if type(d) is MatMulOp and len(d.inputs) == 2 and len(cons.get(d, [])) == 1
              and d not in root_set and getattr(d, 'raw_ctx', None) == getattr(n, 'raw_ctx', None)
              and all(getattr(i, 'raw_ctx', None) == getattr(n, 'raw_ctx', None) for i in n.inputs)]
        if mm:
            d = mm[0]
            rest = [i for i in n.inputs if i is not d]
            if len(rest) > 1:
                other = SumOp(rest, ctx=n.raw_ctx)
                other.bw_of = getattr(n, 'bw_of', None)
            else:
                other = rest[0]
            keep_id, keep_name, bw = n.id, n.name, getattr(n, 'bw_of', None)
            n.__class__ = MatMulOp
            n.__dict__.update({k: v for k, v in d.__dict__.items() if k not in ('id', 'name', 'inputs', 'bw_of')})
            n.inputs = list(d.inputs) + [other]
            n.op_type = 'MatMulOp'
            n.acc_inplace = _dead_join_operand(other, rest, cons, root_set)
            n.id, n.name = keep_id, keep_name
            if bw is not None:
                n.bw_of = bw
            fused += 1
            continue
        # the ResNet downsample join: a 1x1 stride-1 and a 1x1 stride-2 data gradient of the
        # same input -- the stride-2 one stays on its subgrid (compact) and the stride-1 one
        # adds it at the even positions in its epilogue (no scattered full-size tensor)
        s2 = _s2_join(n, cons, root_set)
        if s2 is not None:
            d, other = s2
            other.compact_s2 = True
            keep_id, keep_name, bw = n.id, n.name, getattr(n, 'bw_of', None)
            n.__class__ = Conv2d_Gradient_of_DataOp
            n.__dict__.update({k: v for k, v in d.__dict__.items() if k not in ('id', 'name', 'inputs', 'bw_of')})
            n.inputs = list(d.inputs) + [other]
            n.acc_inplace = False
            n.acc_s2 = True
            n.op_type = 'Conv2d_Gradient_of_DataOp'
            n.id, n.name = keep_id, keep_name
            if bw is not None:
                n.bw_of = bw
            fused += 1
            continue
        for d in n.inputs:
            if isinstance(d, Conv2d_Gradient_of_DataOp) and len(d.inputs) == 3 and \
                    len(cons.get(d, [])) == 1 and d not in root_set:
                rest = [i for i in n.inputs if i is not d]
                if len(rest) > 1:
                    other = SumOp(rest, ctx=n.raw_ctx)
                    other.bw_of = getattr(n, 'bw_of', None)
                else:
                    other = rest[0]
                keep_id, keep_name, bw = n.id, n.name, getattr(n, 'bw_of', None)
                n.__class__ = Conv2d_Gradient_of_DataOp
                n.__dict__.update({k: v for k, v in d.__dict__.items() if k not in ('id', 'name', 'inputs', 'bw_of')})
                n.inputs = list(d.inputs) + [other]
                n.acc_inplace = _dead_join_operand(other, rest, cons, root_set)
                n.op_type = 'Conv2d_Gradient_of_DataOp'
                n.id, n.name = keep_id, keep_name
                if bw is not None:
                    n.bw_of = bw
                fused += 1
                break
    fused += _fuse_bn_backward_reduction(roots)
    return fused


def _is_1x1(d, stride):
    w = d.inputs[0]
    shp = getattr(w, 'shape', None)
    return (tuple(d.stride) == (stride, stride) and tuple(d.padding) == (0, 0) and shp is not None
            and len(shp) == 4 and shp[2] == 1 and shp[3] == 1)


def _s2_join(n, cons, root_set):
    """(stride-1 dgrad, stride-2 dgrad) when the fan-in sum ``n`` adds exactly the data
    gradients of a 1x1 stride-1 and a 1x1 stride-2 (pad 0) convolution of one input"""
    from .ops.nn import Conv2d_Gradient_of_DataOp
    if os.environ.get('HETU_S2_JOIN', '1') != '1' or len(n.inputs) != 2:
        return None
    a, b = n.inputs
    for d, o in ((a, b), (b, a)):
        if not (isinstance(d, Conv2d_Gradient_of_DataOp) and isinstance(o, Conv2d_Gradient_of_DataOp)):
            continue
        if len(d.inputs) != 3 or len(o.inputs) != 3 or d.compact_s2 or o.compact_s2:
            continue
        if any(len(cons.get(x, [])) != 1 or x in root_set for x in (d, o)):
            continue
        if d.inputs[2] is not o.inputs[2] or not _is_1x1(d, 1) or not _is_1x1(o, 2):
            continue
        ctx = getattr(n, 'raw_ctx', None)
        if getattr(d, 'raw_ctx', None) != ctx or getattr(o, 'raw_ctx', None) != ctx:
            continue
        return d, o
    return None


def _fuse_bn_backward_reduction(roots):
    """BatchNorm backward whose dy comes straight from a convolution data gradient:
    that kernel's epilogue, which holds dy, also accumulates the BN backward's
    per-channel reduction (sum(dy'), sum(dy' * x)), and the BN backward skips its own
    pass over dy and x.  The dgrad op gets the BN's input x and forward node (mean,
    invstd, ReLU keep-bits) as extra inputs; the BN forward keeps ReLU keep-bits.
    HETU_FUSE_BN_BWD=1 (default): only data gradients that join another gradient in their
    epilogue -- those already wait on a Cin load per row piece, which the x / keep-bit
    loads ride along with (ResNet-50 joins: -50..-160 us per layer); a store-only epilogue
    pays a round trip per piece and loses to the separate reduction pass (+15..+90 us per
    layer, profiles/bn_fusion_layers_r4.txt).  'all': every eligible one.  Off under
    deterministic mode (fp32 atomics) or HETU_FUSE_BN_BWD=0."""
    from .kernels import deterministic
    mode = os.environ.get('HETU_FUSE_BN_BWD', '1')
    if mode not in ('1', 'all') or deterministic():
        return 0
    from .ops.nn import Conv2d_Gradient_of_DataOp, Batch_Normalization_GradientOp
    topo, cons = _consumers(roots)
    root_set = set(roots)
    fused = 0
    for n in topo:
        if type(n) is not Batch_Normalization_GradientOp:
            continue
        d, fw = n.inputs[0], n.forward_node
        if not isinstance(d, Conv2d_Gradient_of_DataOp) or d.bn_fused is not None or d in root_set or \
                len(cons.get(d, [])) != 1 or len(d.inputs) not in ((3, 4) if mode == 'all' else (4,)):
            continue
        # same device group (a pipeline stage boundary between the BN and its consumer
        # convolution would make the forward node's aux a cross-stage input)
        ctx = getattr(n, 'raw_ctx', None)
        src = getattr(d, 'bw_of', None)
        if getattr(d, 'raw_ctx', None) != ctx or getattr(fw, 'raw_ctx', None) != ctx or \
                (src is not None and getattr(src, 'raw_ctx', None) != ctx):
            continue
        d.inputs = list(d.inputs) + [n.inputs[1], fw]
        d.bn_fused = fw
        d.value_and_aux_inputs = (len(d.inputs) - 1,)
        fw.bwd_fused = True
        fused += 1
    return fused
