"""Convolution, pooling, normalisation and dropout operators.

Parity: reference gpu_ops Conv2d.py, Conv2dAddBias.py, AvgPool.py, MaxPool.py,
BatchNorm.py, LayerNorm.py, InstanceNorm2d.py, Dropout.py, Dropout2d.py
(SURVEY §2.4 "Conv / pool / norm / dropout").

MI355X design:
* activations are logically NCHW (same API/shapes as Hetu) but physically
  channels-last (NHWC) on the GPU, which is what MFMA implicit-GEMM convs and
  the BN/pool kernels want;
* BatchNorm keeps fp32 statistics/affine while activations may be bf16, and is
  fused with the ReLU / residual-add that follow it in ResNets
  (``fused_bn_relu_op``, ``fused_bn_add_relu_op``); the backward consumes the
  saved mean/invstd through the executor's aux channel (no recompute);
* dropout masks are regenerated in the backward from a per-call Philox seed
  (reference ``Dropout.py:46-49`` recompute semantics), never stored.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F
from .. import native_array as _NA

from .node import Op
from ..kernels import norm as KN
from ..kernels import pool as KP
from ..kernels import conv as KC
from ..kernels import layernorm as KLN
from ..kernels import native
from ..kernels import dropout as KD
from ..kernels import tensor as KT


def _kn(t):
    """GPU fp32/bf16 tensor -> hand-written kernel path"""
    return isinstance(t, torch.Tensor) and native(t) and t.dtype in (torch.float32, torch.bfloat16)


class AuxResult(object):
    """Value plus auxiliary tensors saved for a gradient op."""
    __slots__ = ('value', 'aux')

    def __init__(self, value, aux):
        self.value = value
        self.aux = aux


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


# ---------------------------------------------------------------------------
# convolution
class Conv2dOp(Op):
    def __init__(self, x, w, padding=0, stride=1, ctx=None):
        super().__init__(Conv2dOp, [x, w], ctx)
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, w = input_vals
        if getattr(self, 'emit_bn_stats', False) and getattr(x, 'is_cuda', False):
            # the only consumer is a training BatchNorm: hand it the statistics of y
            # (fused into the conv epilogue where the hand-written kernel runs)
            bufs = self.__dict__.setdefault('_bn_sums', {})
            rep = KC.stats_replicas(x.shape, w.shape, self.stride, self.padding)
            if (x.device, rep) not in bufs:   # persistent: the BN zeroes the totals after reading them
                bufs[(x.device, rep)] = _NA.zeros(rep * 2 * w.shape[0], dtype=torch.float32, device=x.device)
            y, sums = KC.conv2d_with_stats(x, w, self.stride, self.padding, out_sums=bufs[(x.device, rep)])
            if sums is not None:
                y.hetu_bn_sums = sums
            return y
        return KC.conv2d(x, w, None, self.stride, self.padding)

    def gradient(self, output_grad):
        return [conv2d_gradient_of_data_op(self.inputs[1], output_grad, self.inputs[0], self.padding, self.stride, ctx=self.raw_ctx),
                conv2d_gradient_of_filter_op(self.inputs[0], output_grad, self.inputs[1], self.padding, self.stride, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        n, c, h, w = input_shapes[0]
        f, _, kh, kw = input_shapes[1]
        ho = (h + 2 * self.padding[0] - kh) // self.stride[0] + 1
        wo = (w + 2 * self.padding[1] - kw) // self.stride[1] + 1
        return (n, f, ho, wo)


def _may_overwrite(op, acc):
    """graph_opt marked the fused join operand dead after this op, and at run time it
    is not an alias of another live output"""
    return bool(getattr(op, 'acc_inplace', False)) and acc is not None and not getattr(acc, 'hetu_shared', False)


class Conv2d_Gradient_of_DataOp(Op):
    shape_only_inputs = (2,)

    def __init__(self, w, grad, x_ref, padding=0, stride=1, ctx=None):
        super().__init__(Conv2d_Gradient_of_DataOp, [w, grad, x_ref], ctx)
        self.padding, self.stride = _pair(padding), _pair(stride)

    bn_fused = None   # graph_opt: (BN forward node) whose backward reduction this epilogue computes
    compact_s2 = False   # graph_opt: 1x1 stride-2 data gradient kept on the stride-2 subgrid
    acc_s2 = False       # graph_opt: the joined gradient (input 3) is such a compact gradient

    def compute(self, input_vals, output_val=None, stream_handle=None):
        # optional 4th input: a gradient to accumulate (fused fan-in sum, graph_opt);
        # with bn_fused the last two inputs are that BN's input x and its forward node
        w, g, xshape = input_vals[:3]
        if self.compact_s2:   # dx at the even positions only = a 1x1 stride-1 gradient on the subgrid
            n, c = xshape[0], xshape[1]
            return KC.conv2d_backward_data(g, w, (n, c, g.shape[2], g.shape[3]), (1, 1), (0, 0))
        nbase = len(input_vals) - (2 if self.bn_fused is not None else 0)
        acc = input_vals[3] if nbase > 3 else None
        bn = None
        if self.bn_fused is not None:
            xb, (_, aux) = input_vals[-2], input_vals[-1]
            if len(aux) > 2 or not self.bn_fused.relu:   # ReLU keep-bits (or no ReLU)
                # persistent totals, R replicas (conv_igemm.bn_sum_replicas).  R == 1:
                # double-buffered -- call k accumulates into half k % 2 and the BN backward
                # of call k folds its coefficients in the apply kernel and zeroes the other
                # half (consumed by call k - 1); R > 1: one buffer, folded and zeroed by the
                # BN backward's finalize kernel
                # Under graph capture the flip would be frozen into the graph: every replay
                # would add into the same half and zero the other, so the captured form
                # uses one buffer, folded and zeroed by the finalize kernel.
                from ..kernels.conv_igemm import bn_sum_replicas
                from ..utils.hipgraph import capturing
                rep = bn_sum_replicas(xb.numel() // xb.shape[1])
                double = rep == 1 and not capturing()
                bufs = self.__dict__.setdefault('_bn_sums', {})
                pair = bufs.get((xb.device, rep, double))
                if pair is None:
                    pair = bufs[(xb.device, rep, double)] = [
                        _NA.zeros(rep * 2 * xb.shape[1], dtype=torch.float32, device=xb.device)
                        for _ in range(2 if double else 1)]
                    pair.append(0)
                k = pair[-1]
                if double:
                    pair[-1] = k ^ 1
                bn = (pair[k], xb, aux[2] if len(aux) > 2 else None)
        r = KC.conv2d_backward_data(g, w, tuple(xshape), self.stride, self.padding, acc=acc,
                                    acc_inplace=_may_overwrite(self, acc) and not self.acc_s2, bn=bn,
                                    acc_s2=self.acc_s2 and acc is not None)
        if bn is not None and getattr(r, 'hetu_bn_bsums', None) is not None and len(pair) == 3:
            r.hetu_bn_bsums_next = pair[pair[2]]
        return r

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        if self.compact_s2:
            x, g = input_shapes[2], input_shapes[1]
            return (x[0], x[1], g[2], g[3])
        return input_shapes[2]


class Conv2d_Gradient_of_FilterOp(Op):
    shape_only_inputs = (2,)

    def __init__(self, x, grad, w_ref, padding=0, stride=1, ctx=None):
        super().__init__(Conv2d_Gradient_of_FilterOp, [x, grad, w_ref], ctx)
        self.padding, self.stride = _pair(padding), _pair(stride)

    grad_dest = None  # set by the optimizer: this op's slot in the flat gradient buffer

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, g, wshape = input_vals
        return KC.conv2d_backward_filter(g, x, tuple(wshape), self.stride, self.padding,
                                         out=self.grad_dest)

    def set_grad_dest(self, dest):
        self.grad_dest = dest
        return True

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def conv2d_op(node_A, node_B, padding=0, stride=1, ctx=None):
    return Conv2dOp(node_A, node_B, padding, stride, ctx=ctx)


def conv2d_gradient_of_data_op(node_A, node_B, node_C, padding=0, stride=1, ctx=None):
    """(filter, grad_y, input_x_ref)"""
    return Conv2d_Gradient_of_DataOp(node_A, node_B, node_C, padding, stride, ctx=ctx)


def conv2d_gradient_of_filter_op(input_X, gradient_Y, input_filter, padding=0, stride=1, ctx=None):
    return Conv2d_Gradient_of_FilterOp(input_X, gradient_Y, input_filter, padding, stride, ctx=ctx)


class Conv2dAddBiasOp(Op):
    def __init__(self, x, w, b, padding=0, stride=1, ctx=None):
        super().__init__(Conv2dAddBiasOp, [x, w, b], ctx)
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, w, b = input_vals
        return KC.conv2d(x, w, b, self.stride, self.padding)

    def gradient(self, output_grad):
        from .shape import conv2d_reducesum_op
        return [conv2d_gradient_of_data_op(self.inputs[1], output_grad, self.inputs[0], self.padding, self.stride, ctx=self.raw_ctx),
                conv2d_gradient_of_filter_op(self.inputs[0], output_grad, self.inputs[1], self.padding, self.stride, ctx=self.raw_ctx),
                conv2d_reducesum_op(output_grad, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return Conv2dOp.infer_shape(self, input_shapes[:2])


def conv2d_add_bias_op(node_A, node_B, bias, padding=0, stride=1, ctx=None):
    return Conv2dAddBiasOp(node_A, node_B, bias, padding, stride, ctx=ctx)


# ---------------------------------------------------------------------------
# pooling
class Max_Pool2dOp(Op):
    def __init__(self, x, kh, kw, padding, stride, ctx=None):
        super().__init__(Max_Pool2dOp, [x], ctx)
        self.kh, self.kw = kh, kw
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        y, idx = KP.maxpool2d(input_vals[0], self.kh, self.kw, self.stride[0], self.stride[1],
                              self.padding[0], self.padding[1])
        return AuxResult(y, (idx, tuple(input_vals[0].shape)))

    def gradient(self, output_grad):
        return [max_pool2d_gradient_op(self, output_grad, self.inputs[0], self.kh, self.kw,
                                       self.padding, self.stride, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        n, c, h, w = input_shapes[0]
        return (n, c, (h + 2 * self.padding[0] - self.kh) // self.stride[0] + 1,
                (w + 2 * self.padding[1] - self.kw) // self.stride[1] + 1)


class Max_Pool2d_GradientOp(Op):
    aux_inputs = (0,)
    shape_only_inputs = (2,)

    def __init__(self, out, grad, x, kh, kw, padding, stride, ctx=None):
        super().__init__(Max_Pool2d_GradientOp, [out, grad, x], ctx)
        self.kh, self.kw = kh, kw
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        (idx, xshape), g, _ = input_vals
        return KP.maxpool2d_backward(g, idx, xshape, self.kh, self.kw, self.stride[0],
                                     self.stride[1], self.padding[0], self.padding[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def max_pool2d_op(node_A, kernel_H, kernel_W, padding, stride, ctx=None):
    return Max_Pool2dOp(node_A, kernel_H, kernel_W, padding, stride, ctx=ctx)


def max_pool2d_gradient_op(node_out, node_out_gradient, node_in, kernel_H, kernel_W, padding, stride, ctx=None):
    return Max_Pool2d_GradientOp(node_out, node_out_gradient, node_in, kernel_H, kernel_W, padding, stride, ctx=ctx)


class Avg_Pool2dOp(Op):
    def __init__(self, x, kh, kw, padding, stride, ctx=None):
        super().__init__(Avg_Pool2dOp, [x], ctx)
        self.kh, self.kw = kh, kw
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        n, c, h, w = x.shape
        if self.kh == h and self.kw == w and self.padding == (0, 0):
            from ..kernels import reduce as KR
            return KR.global_avg_pool(x).reshape(n, c, 1, 1)
        return KP.avgpool2d(x, self.kh, self.kw, self.stride[0], self.stride[1],
                            self.padding[0], self.padding[1])

    def gradient(self, output_grad):
        return [avg_pool2d_gradient_op(self, output_grad, self.inputs[0], self.kh, self.kw,
                                       self.padding, self.stride, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return Max_Pool2dOp.infer_shape(self, input_shapes)


class Avg_Pool2d_GradientOp(Op):
    shape_only_inputs = (0, 2)

    def __init__(self, out, grad, x, kh, kw, padding, stride, ctx=None):
        super().__init__(Avg_Pool2d_GradientOp, [out, grad, x], ctx)
        self.kh, self.kw = kh, kw
        self.padding, self.stride = _pair(padding), _pair(stride)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        _, g, xshape = input_vals
        n, c, h, w = tuple(xshape)
        if self.kh == h and self.kw == w and self.padding == (0, 0):
            from ..kernels import reduce as KR
            return KR.global_avg_pool_backward(g.reshape(n, c), tuple(xshape))
        return KP.avgpool2d_backward(g, tuple(xshape), self.kh, self.kw, self.stride[0],
                                     self.stride[1], self.padding[0], self.padding[1])

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def avg_pool2d_op(node_A, kernel_H, kernel_W, padding, stride, ctx=None):
    return Avg_Pool2dOp(node_A, kernel_H, kernel_W, padding, stride, ctx=ctx)


def avg_pool2d_gradient_op(node_out, node_out_gradient, node_in, kernel_H, kernel_W, padding, stride, ctx=None):
    return Avg_Pool2d_GradientOp(node_out, node_out_gradient, node_in, kernel_H, kernel_W, padding, stride, ctx=ctx)


# ---------------------------------------------------------------------------
# batch normalisation (+ fused ReLU / residual)
class Batch_NormalizationOp(Op):
    bwd_fused = False

    def __init__(self, x, scale, bias, momentum=0.1, eps=1e-5, relu=False, residual=None, ctx=None):
        inputs = [x, scale, bias] + ([residual] if residual is not None else [])
        super().__init__(Batch_NormalizationOp, inputs, ctx)
        self.momentum, self.eps = momentum, eps
        self.relu, self.has_residual = relu, residual is not None
        self.running_mean = None
        self.running_var = None
        self.inference = False
        self.bwd_fused = False    # graph_opt: the backward reduction runs in a dgrad epilogue

    def _init_running(self, C, device):
        if self.running_mean is None or self.running_mean.device != device:
            rm0, rv0 = getattr(self, 'running_mean_init', None), getattr(self, 'running_var_init', None)
            self.running_mean = _NA.zeros(C, dtype=torch.float32, device=device) if rm0 is None else \
                torch.as_tensor(rm0, dtype=torch.float32).to(device)
            self.running_var = torch.ones(C, dtype=torch.float32, device=device) if rv0 is None else \
                torch.as_tensor(rv0, dtype=torch.float32).to(device)

    def compute(self, input_vals, output_val=None, stream_handle=None, inference=None):
        x, scale, bias = input_vals[:3]
        res = input_vals[3] if self.has_residual else None
        self._init_running(x.shape[1], x.device)
        training = not (self.inference if inference is None else inference)
        sums = getattr(x, 'hetu_bn_sums', None) if training else None
        # fused add+ReLU: the backward needs the ReLU mask, which then depends on the
        # residual too; keep it as bits (1/16 of y's bytes) instead of re-reading y
        # (also wanted by a data-gradient epilogue that fuses this BN's backward reduction)
        mask = None
        if training and self.relu and (self.has_residual or self.bwd_fused) and x.is_cuda and native(x) and \
                x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % (8 if x.dtype == torch.bfloat16 else 4) == 0:
            mask = _NA.empty(KN.relu_mask_bytes(x), dtype=torch.uint8, device=x.device)
        if sums is None and getattr(x, 'hetu_bn_sums', None) is not None:
            x.hetu_bn_sums.zero_()    # persistent totals not consumed (inference): ready for next time
        y, mean, invstd = KN.bn_forward(x, scale.float(), bias.float(), self.running_mean,
                                        self.running_var, self.momentum, self.eps, training,
                                        relu=self.relu, residual=res, sums=sums, mask=mask)
        if not training:
            return y
        return AuxResult(y, (mean, invstd) if mask is None else (mean, invstd, mask))

    def gradient(self, output_grad):
        g = Batch_Normalization_GradientOp(output_grad, self.inputs[0], self.inputs[1], self,
                                           self.eps, ctx=self.raw_ctx, bias=self.inputs[2])
        out = [batch_normalization_gradient_of_data_op(g, self.inputs[0], ctx=self.raw_ctx),
               batch_normalization_gradient_of_scale_op(g, self.inputs[1], ctx=self.raw_ctx),
               batch_normalization_gradient_of_bias_op(g, self.inputs[2], ctx=self.raw_ctx)]
        if self.has_residual:
            out.append(BNGradSelectOp(g, 3, ctx=self.raw_ctx))
        return out

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Batch_Normalization_GradientOp(Op):
    """Computes (dx, dscale, dbias[, dresidual]) in one fused kernel pass."""
    grad_dest_slots = (1, 2)
    aux_inputs = (3,)
    value_and_aux_inputs = (3,)

    def __init__(self, out_gradient, x, scale, forward_node, eps, ctx=None, bias=None):
        super().__init__(Batch_Normalization_GradientOp,
                         [out_gradient, x, scale, forward_node] + ([bias] if bias is not None else []), ctx)
        self.forward_node = forward_node
        self.eps = eps

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, x, scale, (y, aux) = input_vals[:4]
        mean, invstd = aux[:2]
        mask = aux[2] if len(aux) > 2 else None
        bias = input_vals[4] if len(input_vals) > 4 else None
        fw = self.forward_node
        dests = getattr(self, 'grad_dests', {})
        # the reduction totals of the data-gradient epilogue that produced g (fused: ops
        # Conv2d_Gradient_of_DataOp.bn_fused); the kernel zeroes them once read
        bsums = getattr(g, 'hetu_bn_bsums', None)
        bnext = getattr(g, 'hetu_bn_bsums_next', None) if bsums is not None else None
        if bsums is not None and not (g.is_cuda and g.dtype == x.dtype == torch.bfloat16 and (mask is not None or not fw.relu)):
            bsums.zero_()         # not consumed: both halves ready for their next use
            if bnext is not None:
                bnext.zero_()
            bsums = bnext = None
        if bsums is not None and getattr(g, 'hetu_bn_masked', False):
            # g was stored already masked by the ReLU keep-bits (dy'): no mask to apply,
            # and dy' itself is the gradient of the fused residual input
            dx, dscale, dbias, _ = KN.bn_backward(g, y, x, scale.float(), mean, invstd, relu=False,
                                                  want_dres=False, bias=bias, dscale_out=dests.get(1),
                                                  dbias_out=dests.get(2), bsums=bsums, bsums_next=bnext)
            # (a fresh tensor object over the same storage: g's hetu_bn_* attributes
            # belong to this BN and must not reach the consumer of the residual gradient)
            return (dx, dscale, dbias, g.detach() if fw.has_residual else None)
        dx, dscale, dbias, dres = KN.bn_backward(g, y, x, scale.float(), mean, invstd,
                                                 relu=fw.relu, want_dres=fw.has_residual, bias=bias,
                                                 dscale_out=dests.get(1), dbias_out=dests.get(2), mask=mask,
                                                 bsums=bsums, bsums_next=bnext)
        return (dx, dscale, dbias, dres)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


class BNGradSelectOp(Op):
    def __init__(self, g, index, ctx=None):
        super().__init__(BNGradSelectOp, [g], ctx)
        self.index = index

    def set_grad_dest(self, dest):
        """dscale / dbias (BN, LayerNorm) are written by the fused backward kernel
        straight into the optimizer's flat gradient buffer."""
        src = self.inputs[0]
        if self.index in getattr(src, 'grad_dest_slots', ()) and \
                dest.dtype == torch.float32 and dest.is_contiguous():
            if not hasattr(src, 'grad_dests'):
                src.grad_dests = {}
            src.grad_dests[self.index] = dest
            return True
        return False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        tup = input_vals[0]
        v = tup[self.index]
        if isinstance(v, torch.Tensor) and v.numel() and \
                sum(1 for o in tup if isinstance(o, torch.Tensor) and o.data_ptr() == v.data_ptr()) > 1:
            v.hetu_shared = True    # aliases another output (e.g. LN dx is ds without dropout): never overwrite
        return v

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def batch_normalization_op(node_in, bn_scale, bn_bias, momentum=0.1, eps=1e-5, ctx=None):
    return Batch_NormalizationOp(node_in, bn_scale, bn_bias, momentum, eps, ctx=ctx)


def fused_bn_relu_op(node_in, bn_scale, bn_bias, momentum=0.1, eps=1e-5, ctx=None):
    """relu(batch_norm(x)) in one kernel pass (and one fused backward)."""
    return Batch_NormalizationOp(node_in, bn_scale, bn_bias, momentum, eps, relu=True, ctx=ctx)


def fused_bn_add_relu_op(node_in, bn_scale, bn_bias, residual, momentum=0.1, eps=1e-5, ctx=None):
    """relu(batch_norm(x) + residual) -- the ResNet block tail."""
    return Batch_NormalizationOp(node_in, bn_scale, bn_bias, momentum, eps, relu=True,
                                 residual=residual, ctx=ctx)


def batch_normalization_gradient_op(out_gradient, in_node, bn_scale, forward_node, eps, ctx=None):
    return Batch_Normalization_GradientOp(out_gradient, in_node, bn_scale, forward_node, eps, ctx=ctx)


def batch_normalization_gradient_of_data_op(bn_gradient, in_arr, ctx=None):
    op = BNGradSelectOp(bn_gradient, 0, ctx=ctx)
    op.op_type = 'Batch_Normalization_Gradient_of_DataOp'
    return op


def batch_normalization_gradient_of_scale_op(bn_gradient, in_scale, ctx=None):
    op = BNGradSelectOp(bn_gradient, 1, ctx=ctx)
    op.op_type = 'Batch_Normalization_Gradient_of_ScaleOp'
    return op


def batch_normalization_gradient_of_bias_op(bn_gradient, in_bias, ctx=None):
    op = BNGradSelectOp(bn_gradient, 2, ctx=ctx)
    op.op_type = 'Batch_Normalization_Gradient_of_BiasOp'
    return op


# ---------------------------------------------------------------------------
# layer normalisation
class Layer_NormalizationOp(Op):
    def __init__(self, x, scale, bias, eps=0.01, ctx=None):
        super().__init__(Layer_NormalizationOp, [x, scale, bias], ctx)
        self.eps = eps

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, g, b = input_vals
        y, mean, rstd = KLN.layer_norm(x, g, b, self.eps)
        return AuxResult(y, (mean, rstd))

    def gradient(self, output_grad):
        gn = Layer_Normalization_GradientOp(output_grad, self.inputs[0], self.inputs[1], self, self.eps, ctx=self.raw_ctx)
        return [layer_normalization_gradient_of_data_op(gn, self.inputs[0], ctx=self.raw_ctx),
                layer_normalization_gradient_of_scale_op(gn, self.inputs[1], ctx=self.raw_ctx),
                layer_normalization_gradient_of_bias_op(gn, self.inputs[2], ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Layer_Normalization_GradientOp(Op):
    aux_inputs = (3,)
    grad_dest_slots = (1, 2)

    def __init__(self, out_gradient, x, scale, forward_node, eps, ctx=None):
        super().__init__(Layer_Normalization_GradientOp, [out_gradient, x, scale, forward_node], ctx)
        self.eps = eps

    def compute(self, input_vals, output_val=None, stream_handle=None):
        dy, x, g, (mean, rstd) = input_vals
        dests = getattr(self, 'grad_dests', {})
        return KLN.layer_norm_backward(dy, x, g, mean, rstd, dg_out=dests.get(1), db_out=dests.get(2))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def layer_normalization_op(node_in, ln_scale, ln_bias, eps=0.01, ctx=None):
    return Layer_NormalizationOp(node_in, ln_scale, ln_bias, eps, ctx=ctx)


def layer_normalization_gradient_op(out_gradient, in_node, ln_scale, forward_node, eps, ctx=None):
    return Layer_Normalization_GradientOp(out_gradient, in_node, ln_scale, forward_node, eps, ctx=ctx)


def _sel(g, i, name, ctx):
    op = BNGradSelectOp(g, i, ctx=ctx)
    op.op_type = name
    return op


def layer_normalization_gradient_of_data_op(ln_gradient, in_arr, ctx=None):
    return _sel(ln_gradient, 0, 'Layer_Normalization_Gradient_of_DataOp', ctx)


def layer_normalization_gradient_of_scale_op(ln_gradient, in_scale, ctx=None):
    return _sel(ln_gradient, 1, 'Layer_Normalization_Gradient_of_ScaleOp', ctx)


def layer_normalization_gradient_of_bias_op(ln_gradient, in_bias, ctx=None):
    return _sel(ln_gradient, 2, 'Layer_Normalization_Gradient_of_BiasOp', ctx)


class DropoutAddLayerNormOp(Op):
    """y = LayerNorm(dropout(x) + residual) as ONE kernel (MI355X fusion of the
    post-LN transformer block tail, reference hetu_bert.py / hetu_transformer.py
    ``layer_norm(dropout(h) + input)`` = 3 ops, 3 kernels each way).  The
    backward regenerates the dropout mask from the seed (no mask tensor) and
    emits dx, dresidual, dscale, dbias from one row pass + one column reduce."""

    def __init__(self, x, residual, scale, bias, keep_prob=1.0, eps=1e-12, ctx=None):
        ins = [x] + ([residual] if residual is not None else []) + [scale, bias]
        super().__init__(DropoutAddLayerNormOp, ins, ctx)
        self.has_res = residual is not None
        self.keep_prob, self.eps = float(keep_prob), eps
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        res = input_vals[1] if self.has_res else None
        g, b = input_vals[-2], input_vals[-1]
        keep = 1.0 if self.inference else self.keep_prob
        seed = _next_seed(self.id, x) if keep < 1.0 else 0
        if res is not None and res.dtype != x.dtype:
            res = res.to(x.dtype)
        y, sm, mean, rstd = KLN.layer_norm_fused(x, res, g, b, self.eps, keep, seed)
        return AuxResult(y, (sm, mean, rstd, keep, seed))

    def gradient(self, output_grad):
        gn = DropoutAddLayerNormGradientOp(output_grad, self, ctx=self.raw_ctx)
        grads = [_sel(gn, 0, 'DropoutAddLayerNorm_Gradient_of_DataOp', self.raw_ctx)]
        if self.has_res:
            grads.append(_sel(gn, 1, 'DropoutAddLayerNorm_Gradient_of_ResidualOp', self.raw_ctx))
        grads += [_sel(gn, 2, 'DropoutAddLayerNorm_Gradient_of_ScaleOp', self.raw_ctx),
                  _sel(gn, 3, 'DropoutAddLayerNorm_Gradient_of_BiasOp', self.raw_ctx)]
        return grads

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class DropoutAddLayerNormGradientOp(Op):
    """Outputs (dx, dresidual, dscale, dbias[, dlinear_bias]).  ``emit_lin_bias``
    (set by graph_opt.fuse_backward when x comes from a linear layer whose bias
    gradient is the row sum of dx) adds output 4: that bias gradient, summed in the
    same kernel pass instead of a separate reduction over dx."""
    aux_inputs = (1,)
    grad_dest_slots = (2, 3, 4)
    emit_lin_bias = False

    def __init__(self, out_gradient, forward_node, ctx=None):
        super().__init__(DropoutAddLayerNormGradientOp, [out_gradient, forward_node, forward_node.inputs[-2]], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        dy, (sm, mean, rstd, keep, seed), g = input_vals
        if dy.dtype != sm.dtype:
            dy = dy.to(sm.dtype)
        dests = getattr(self, 'grad_dests', {})
        if not self.emit_lin_bias:
            ds, dx, dg, db = KLN.layer_norm_fused_backward(dy, sm, g, mean, rstd, keep, seed,
                                                           dg_out=dests.get(2), db_out=dests.get(3))
            return (dx, ds, dg, db)
        if sm.dim() == 2:
            ds, dx, dg, db, dl = KLN.layer_norm_fused_backward(dy, sm, g, mean, rstd, keep, seed,
                                                               dg_out=dests.get(2), db_out=dests.get(3),
                                                               want_dlin=True, dlin_out=dests.get(4))
        else:   # the replaced node summed over axis 0 only
            from ..kernels import reduce as KR
            ds, dx, dg, db = KLN.layer_norm_fused_backward(dy, sm, g, mean, rstd, keep, seed,
                                                           dg_out=dests.get(2), db_out=dests.get(3))
            dl = KR.reduce_mid(dx.contiguous().reshape(1, dx.shape[0], -1)).reshape(dx.shape[1:])
            d = dests.get(4)
            if d is not None and d.numel() == dl.numel():
                d.view(dl.shape).copy_(dl)
                dl = d.view(dl.shape)
        return (dx, ds, dg, db, dl)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return None


def dropout_add_layernorm_op(x, residual, ln_scale, ln_bias, keep_prob=1.0, eps=1e-12, ctx=None):
    return DropoutAddLayerNormOp(x, residual, ln_scale, ln_bias, keep_prob, eps, ctx=ctx)


class Instance_Normalization2dOp(Op):
    def __init__(self, x, eps=1e-7, ctx=None):
        super().__init__(Instance_Normalization2dOp, [x], ctx)
        self.eps = eps

    def compute(self, input_vals, output_val=None, stream_handle=None):
        if _kn(input_vals[0]):
            y, mean, rstd = KT.instance_norm2d(input_vals[0], self.eps)
            return AuxResult(y, (mean, rstd))
        x = input_vals[0].float()
        mean = x.mean((2, 3), keepdim=True)
        var = x.var((2, 3), unbiased=False, keepdim=True)
        rstd = torch.rsqrt(var + self.eps)
        return AuxResult(((x - mean) * rstd).to(input_vals[0].dtype), (mean, rstd))

    def gradient(self, output_grad):
        return [instance_normalization2d_gradient_op(output_grad, self.inputs[0], self, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Instance_Normalization2d_GradientOp(Op):
    aux_inputs = (2,)

    def __init__(self, grad, x, forward_node, ctx=None):
        super().__init__(Instance_Normalization2d_GradientOp, [grad, x, forward_node], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, x, (mean, rstd) = input_vals
        if _kn(x):
            return KT.instance_norm2d_grad(g, x, mean, rstd)
        gf, xf = g.float(), x.float()
        xhat = (xf - mean) * rstd
        m = gf.mean((2, 3), keepdim=True)
        mx = (gf * xhat).mean((2, 3), keepdim=True)
        return (rstd * (gf - m - xhat * mx)).to(x.dtype)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[1]


def instance_normalization2d_op(node_in, eps=0.01, ctx=None):
    return Instance_Normalization2dOp(node_in, eps, ctx=ctx)


def instance_normalization2d_gradient_op(out_gradient, in_node, forward_node, ctx=None):
    return Instance_Normalization2d_GradientOp(out_gradient, in_node, forward_node, ctx=ctx)


# ---------------------------------------------------------------------------
# dropout (Philox, recompute mask in backward)
def _next_seed(key, x=None):
    """host seed of op ``key``'s next draw (kernels/rng.py: fixed per op and call within a
    step; the device step counter varies it between steps, replay-safe under hipGraph)"""
    from ..kernels import rng
    return rng.next_seed(key, on_gpu=x.is_cuda if x is not None else _base_gpu())


def _base_gpu():
    from .._base import gpu_available
    return gpu_available()


class DropoutOp(Op):
    def __init__(self, x, keep_prob, recompute=True, inplace=False, ctx=None):
        super().__init__(DropoutOp, [x], ctx)
        self.keep_prob, self.recompute = keep_prob, recompute
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if self.inference or self.keep_prob >= 1.0:
            return AuxResult(x, 0)
        seed = _next_seed(self.id, x)
        return AuxResult(KD.dropout(x, self.keep_prob, seed), seed)

    def gradient(self, output_grad):
        return [dropout_gradient_recompute_op(output_grad, self.keep_prob, self, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Dropout_Gradient_recomputeOp(Op):
    aux_inputs = (1,)

    def __init__(self, grad, keep_prob, forward_node, ctx=None):
        super().__init__(Dropout_Gradient_recomputeOp, [grad, forward_node], ctx)
        self.keep_prob = keep_prob

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, seed = input_vals
        if self.keep_prob >= 1.0 or seed == 0:
            return g
        return KD.dropout(g, self.keep_prob, seed)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def dropout_op(node_in, keep_prob, recompute=True, inplace=False, ctx=None):
    return DropoutOp(node_in, keep_prob, recompute, inplace, ctx=ctx)


def dropout_gradient_recompute_op(node_in, keep_prob, forward_node, ctx=None):
    return Dropout_Gradient_recomputeOp(node_in, keep_prob, forward_node, ctx=ctx)


def dropout_gradient_op(node_in, keep_prob, forward_node, ctx=None):
    return Dropout_Gradient_recomputeOp(node_in, keep_prob, forward_node, ctx=ctx)


class Dropout2dOp(Op):
    """Channel dropout: whole (n, c) planes zeroed."""

    def __init__(self, x, keep_prob, ctx=None):
        super().__init__(Dropout2dOp, [x], ctx)
        self.keep_prob = keep_prob
        self.inference = False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        if self.inference:
            return AuxResult(x, None)
        if self.keep_prob >= 1.0:
            return AuxResult(x, None)
        seed = _next_seed(self.id, x)
        return AuxResult(_dropout2d(x, self.keep_prob, seed), seed)

    def gradient(self, output_grad):
        return [dropout2d_gradient_op(output_grad, self.keep_prob, self, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class Dropout2d_GradientOp(Op):
    aux_inputs = (1,)

    def __init__(self, grad, keep_prob, forward_node, ctx=None):
        super().__init__(Dropout2d_GradientOp, [grad, forward_node], ctx)
        self.keep_prob = keep_prob

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, seed = input_vals
        # the forward's plane mask regenerated from its seed (same planes, same 1 / keep)
        return g if seed is None else _dropout2d(g, self.keep_prob, seed)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def _dropout2d(x, keep, seed):
    """channel dropout: the HIP kernel on the GPU (random.hip, reference Dropout2d.cu:4),
    the same Philox(seed, plane) draws on the CPU"""
    if x.is_cuda:
        from ..kernels import rng
        return rng.dropout2d(x, keep, seed)
    n, c = int(x.shape[0]), int(x.shape[1])
    planes = torch.arange(n * c, dtype=torch.int64)
    u = _philox_u01_host(seed, planes)
    mask = (u < keep).to(x.dtype).reshape((n, c) + (1,) * (x.dim() - 2)) / keep
    return x * mask


def _philox_u01_host(seed, ctr):
    """Philox4x32-10 word 0 of (seed, counter) as (0,1] floats -- the kernels' draw on the host"""
    import numpy as np
    from ..kernels.moe import philox4
    x = philox4(int(seed), ctr.numpy().astype(np.uint64))[0]
    return torch.from_numpy(((x >> np.uint64(8)).astype(np.float32) + 0.5) / 16777216.0)


def dropout2d_op(node_in, keep_prob, ctx=None):
    return Dropout2dOp(node_in, keep_prob, ctx=ctx)


def dropout2d_gradient_op(node_in, keep_prob, forward_node, ctx=None):
    return Dropout2d_GradientOp(node_in, keep_prob, forward_node, ctx=ctx)
