"""Matrix products (reference MatrixMult.py, Linear.py, Addmm.py, Baddbmm.py,
BatchMatrixMult.py, CuSparse.py; SURVEY §2.4 "Linear algebra").

``matmul``/``linear`` run on the hand-written bf16 MFMA GEMM (``gemm.hip``,
fused bias/activation epilogue) where it has been selected for the shape, and
on hipBLASLt otherwise (plain library GEMM).  Mixed precision: when either
operand is bf16 both are computed in bf16 with fp32 accumulation.
"""
from __future__ import annotations

import os

import torch
from .. import native_array as _NA

from .. import ndarray
from .node import Op
from .nn import AuxResult, _may_overwrite
from ..kernels import gemm as KG


def _tr(t, flag):
    return t.transpose(-1, -2) if flag else t



_GELU_EPI = __import__('os').environ.get('HETU_GELU_EPILOGUE', '1') == '1'

class MatMulOp(Op):
    def __init__(self, a, b, trans_A=False, trans_B=False, ctx=None):
        super().__init__(MatMulOp, [a, b], ctx)
        self.matmul_attr_trans_A, self.matmul_attr_trans_B = trans_A, trans_B

    grad_dest = None  # fp32 slot in the optimizer's flat gradient buffer (weight grads)

    def set_grad_dest(self, dest):
        if dest.dtype == torch.float32 and dest.is_contiguous():
            self.grad_dest = dest
            return True
        return False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals[:2]
        if len(input_vals) == 3:   # fused gradient join (graph_opt.fuse_backward): op(a) @ op(b) + acc
            acc = input_vals[2]
            if self.grad_dest is None and not isinstance(acc, ndarray.IndexedSlices):
                return KG.matmul_acc(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, acc,
                                     inplace=_may_overwrite(self, acc))
            y = self.compute([a, b])
            if not (self.grad_dest is not None and y.data_ptr() == self.grad_dest.data_ptr()):
                if y.is_cuda:
                    from ..kernels.tensor import copy_into
                    y = copy_into(_NA.empty(y.shape, dtype=torch.float32 if self.grad_dest is not None else y.dtype,
                                              device=y.device), y)
                else:
                    y = y.float() if self.grad_dest is not None else y.clone()
            if isinstance(acc, ndarray.IndexedSlices) and y.dtype == torch.float32 and y.is_contiguous():
                # tied embedding: the lookup's row-sparse gradient lands straight in the
                # dense fp32 gradient (no densified copy of the table)
                from ..kernels import sparse as KSP
                KSP.scatter_add_rows(y.view(-1, y.shape[-1]), acc._t(acc.indices), acc._t(acc.values))
                return y
            if y.is_cuda and not isinstance(acc, ndarray.IndexedSlices) and y.is_contiguous():
                from ..kernels.elementwise import binary
                return binary('add', y, acc, out=y)
            y.add_((acc.to_dense() if isinstance(acc, ndarray.IndexedSlices) else acc).to(y.dtype))
            return y
        d = self.grad_dest
        if d is not None and a.is_cuda and a.dim() == 2 and b.dim() == 2:
            m = a.shape[1] if self.matmul_attr_trans_A else a.shape[0]
            n = b.shape[0] if self.matmul_attr_trans_B else b.shape[1]
            if d.numel() == m * n:
                return KG.matmul_into(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, d.view(m, n))
        return KG.matmul(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B)

    def gradient(self, output_grad):
        ta, tb = self.matmul_attr_trans_A, self.matmul_attr_trans_B
        A, B, G = self.inputs[0], self.inputs[1], output_grad
        c = self.raw_ctx
        if not ta and not tb:
            return [matmul_op(G, B, False, True, ctx=c), matmul_op(A, G, True, False, ctx=c)]
        if ta and not tb:
            return [matmul_op(B, G, False, True, ctx=c), matmul_op(A, G, False, False, ctx=c)]
        if not ta and tb:
            return [matmul_op(G, B, False, False, ctx=c), matmul_op(G, A, True, False, ctx=c)]
        return [matmul_op(B, G, True, True, ctx=c), matmul_op(G, A, True, True, ctx=c)]

    def infer_shape(self, input_shapes):
        a, b = input_shapes[:2]
        m = a[1] if self.matmul_attr_trans_A else a[0]
        n = b[0] if self.matmul_attr_trans_B else b[1]
        return (m, n)


def matmul_op(node_A, node_B, trans_A=False, trans_B=False, ctx=None):
    return MatMulOp(node_A, node_B, trans_A, trans_B, ctx=ctx)


class RowConcatMatMulOp(Op):
    """concat([x_0 @ w_0, ..., x_{n-1} @ w_{n-1}], axis=0) with every product written into
    its row block of one output (kernels.gemm.matmul_out) -- no per-product output and no
    concatenation copy.  The MoE layer's local experts' second GEMMs (layers/moe.py
    _dispatch_and_run; the reference concatenates the expert outputs,
    python/hetu/layers/moe_layer.py).  Gradient: row-block views of the output gradient
    into the per-expert data / weight gradient GEMMs."""

    def __init__(self, xs, ws, ctx=None):
        assert len(xs) == len(ws) and len(xs) > 0
        super().__init__(RowConcatMatMulOp, list(xs) + list(ws), ctx)
        self.n = len(xs)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        xs, ws = input_vals[:self.n], input_vals[self.n:]
        N = ws[0].shape[1]
        rows = [x.shape[0] for x in xs]
        if not xs[0].is_cuda or xs[0].dtype != torch.bfloat16:
            from ..kernels import tensor as KT
            return KT.concat([KG.matmul(x, w) for x, w in zip(xs, ws)], 0)
        out = _NA.empty((sum(rows), N), dtype=xs[0].dtype, device=xs[0].device)
        r = 0
        for x, w, m in zip(xs, ws, rows):
            KG.matmul_out(x, w, out[r:r + m])
            r += m
        return out

    def gradient(self, output_grad):
        from .shape import split_op
        xs, ws = self.inputs[:self.n], self.inputs[self.n:]
        c = self.raw_ctx
        gx, gw = [], []
        for i in range(self.n):
            g = split_op(output_grad, axes=[0], indices=[i], splits=[self.n], ctx=c)
            gx.append(matmul_op(g, ws[i], False, True, ctx=c))
            gw.append(matmul_op(xs[i], g, True, False, ctx=c))
        return gx + gw

    def infer_shape(self, input_shapes):
        xs, ws = input_shapes[:self.n], input_shapes[self.n:]
        return (sum(x[0] for x in xs), ws[0][1])


def row_concat_matmul_op(xs, ws, ctx=None):
    return RowConcatMatMulOp(xs, ws, ctx=ctx)


class LinearOp(Op):
    """A @ B + bias with the bias (and optional activation) fused in the GEMM
    epilogue."""

    def __init__(self, a, b, bias, trans_A=False, trans_B=False, activation=None, ctx=None):
        super().__init__(LinearOp, [a, b, bias], ctx)
        self.matmul_attr_trans_A, self.matmul_attr_trans_B = trans_A, trans_B
        self.activation = activation

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b, bias = input_vals
        if self.activation == 'gelu' and self.need_pre:
            # keep the pre-activation for the backward (instead of re-running the GEMM):
            # the GEMM epilogue stores both it and the activation (HETU_GELU_EPILOGUE=0: the
            # GEMM stores the pre-activation and a separate pass applies the GELU)
            if _GELU_EPI:
                y, pre = KG.matmul_pre(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, bias, 'gelu')
                return AuxResult(y, pre)
            from ..kernels.elementwise import unary
            pre = KG.matmul(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, bias=bias)
            return AuxResult(unary('gelu', pre), pre)
        return KG.matmul(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, bias=bias,
                         activation=self.activation)

    need_pre = False

    def gradient(self, output_grad):
        from .reduce import reducesumaxiszero_op
        from .basic import relu_gradient_op
        G = output_grad
        if self.activation == 'relu':
            G = relu_gradient_op(self, output_grad, ctx=self.raw_ctx)
        elif self.activation == 'gelu':
            self.need_pre = True
            G = LinearGeluGradOp(output_grad, self, ctx=self.raw_ctx)
        mm = MatMulOp(self.inputs[0], self.inputs[1], self.matmul_attr_trans_A, self.matmul_attr_trans_B)
        ga, gb = mm.gradient(G)
        return [ga, gb, reducesumaxiszero_op(G, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return MatMulOp.infer_shape(self, input_shapes[:2])


class MatMulActDropoutOp(Op):
    """dropout(relu(A @ B)) with the ReLU and the dropout in the GEMM epilogue (the MoE
    experts' first layer: reference layers/moe_layer Expert = linear, activation, dropout).
    The backward needs only this output: d(A @ B) = g / keep where out > 0, else 0 -- a
    dropped element is 0 and so is its gradient, a kept one is positive exactly where the
    ReLU passed -- so no mask is stored or regenerated."""

    def __init__(self, a, b, activation='relu', keep_prob=1.0, ctx=None):
        super().__init__(MatMulActDropoutOp, [a, b], ctx)
        assert activation == 'relu', activation
        self.activation, self.keep_prob = activation, keep_prob
        self.inference = False
        self.emit_bits = False   # set by gradient(): aux = the keep bits the backward GEMM reads

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from .nn import _next_seed, AuxResult
        a, b = input_vals
        keep = 1.0 if self.inference else self.keep_prob
        if keep >= 1.0:
            y = KG.matmul(a, b, activation=self.activation)
            return AuxResult(y, y) if self.emit_bits else y
        if self.emit_bits:
            y, mask = KG.matmul_act_dropout_bits(a, b, self.activation, keep, _next_seed(self.id, a))
            return AuxResult(y, mask)
        return KG.matmul_act_dropout(a, b, self.activation, keep, _next_seed(self.id, a))

    def gradient(self, output_grad):
        if type(output_grad) is MatMulOp and len(output_grad.inputs) == 2 and _GMASK_EPI:
            # the gradient arriving here is the next layer's data-gradient GEMM: mask it in
            # that GEMM's epilogue (one pass less over the [tokens, hidden] activation);
            # HETU_GMASK_BITS (default on, dropout layers): the forward epilogue also stores
            # its keep bits and the backward epilogue reads those, 1/16 of the output's bytes
            self.emit_bits = _GMASK_BITS and self.keep_prob < 1.0
            G = MatMulReluMaskOp(output_grad.inputs[0], output_grad.inputs[1], output_grad.matmul_attr_trans_A,
                                 output_grad.matmul_attr_trans_B, self, self.keep_prob, ctx=self.raw_ctx,
                                 bits=self.emit_bits)
        else:
            G = ReluDropoutGradOp(output_grad, self, self.keep_prob, ctx=self.raw_ctx)
        mm = MatMulOp(self.inputs[0], self.inputs[1], False, False)
        return list(mm.gradient(G))

    def infer_shape(self, input_shapes):
        return MatMulOp.infer_shape(self, input_shapes[:2])

    matmul_attr_trans_A = False
    matmul_attr_trans_B = False


class ReluDropoutGradOp(Op):
    """g / keep where the forward output is positive, else 0 (see MatMulActDropoutOp)"""

    def __init__(self, grad, fwd, keep_prob, ctx=None):
        super().__init__(ReluDropoutGradOp, [grad, fwd], ctx)
        self.keep_prob = keep_prob

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.elementwise import binary
        g, y = input_vals
        if g.dtype != y.dtype:
            from ..kernels.elementwise import cast
            g = cast(g.contiguous(), y.dtype)
        return binary('relu_grad_c', y.contiguous(), g.contiguous(), 1.0 / self.keep_prob)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class MatMulReluMaskOp(Op):
    """(op(a) @ op(b)) / keep where the forward output ``fwd`` is positive, else 0: the data
    gradient of a MatMulActDropoutOp's output, produced and masked by one GEMM
    (``HETU_GMASK_EPILOGUE=0``: the plain GEMM + ReluDropoutGradOp)."""

    def __init__(self, a, b, trans_A, trans_B, fwd, keep_prob, ctx=None, bits=False):
        super().__init__(MatMulReluMaskOp, [a, b, fwd], ctx)
        self.matmul_attr_trans_A, self.matmul_attr_trans_B = trans_A, trans_B
        self.keep_prob = keep_prob
        if bits:
            self.aux_inputs = (2,)   # the forward's mask (keep bits), not its output

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b, y = input_vals
        if getattr(self, 'aux_inputs', None):
            return KG.matmul_mask(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, y, 1.0 / self.keep_prob)
        return KG.matmul_relu_mask(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B, y.contiguous(),
                                   1.0 / self.keep_prob)

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return MatMulOp.infer_shape(self, input_shapes[:2])


_GMASK_EPI = os.environ.get('HETU_GMASK_EPILOGUE', '1') != '0'
_GMASK_BITS = os.environ.get('HETU_GMASK_BITS', '1') != '0'


def matmul_act_dropout_op(a, b, activation='relu', keep_prob=1.0, ctx=None):
    return MatMulActDropoutOp(a, b, activation, keep_prob, ctx=ctx)


class LinearGeluGradOp(Op):
    """gelu'(pre) * grad with the pre-activation saved by the forward LinearOp.
    ``emit_colsum`` (graph_opt.fuse_backward): also the row sum of the result --
    the layer's bias gradient -- from the same kernel pass, as the aux value read
    by a LinearGeluBiasGradOp."""
    value_and_aux_inputs = (1,)
    emit_colsum = False
    colsum_dest = None

    def __init__(self, grad, fwd, ctx=None):
        super().__init__(LinearGeluGradOp, [grad, fwd], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.elementwise import binary
        g, (y, pre) = input_vals
        if self.emit_colsum:
            from ..kernels.layernorm import gelu_grad_colsum
            if g.dtype != pre.dtype:
                g = g.to(pre.dtype)
            out, cs = gelu_grad_colsum(pre, g, out=self.colsum_dest)
            return AuxResult(out, cs)
        return binary('gelu_grad', pre.contiguous(), g.contiguous())

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class LinearGeluBiasGradOp(Op):
    """Bias gradient of a GELU linear layer, taken from its LinearGeluGradOp's
    fused column sums (replaces ``reducesumaxiszero_op`` of the GELU gradient)."""
    aux_inputs = (0,)

    def __init__(self, gelu_grad, ctx=None):
        super().__init__(LinearGeluBiasGradOp, [gelu_grad], ctx)

    def set_grad_dest(self, dest):
        if dest.dtype == torch.float32 and dest.is_contiguous():
            self.inputs[0].colsum_dest = dest
            return True
        return False

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0]

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[0][1:])


def linear_op(node_A, node_B, bias, trans_A=False, trans_B=False, activation=None, ctx=None):
    return LinearOp(node_A, node_B, bias, trans_A, trans_B, activation, ctx=ctx)


class AddmmOp(Op):
    """beta * input + alpha * (A @ B)."""

    def __init__(self, inp, a, b, alpha=1.0, beta=1.0, ctx=None):
        super().__init__(AddmmOp, [inp, a, b], ctx)
        self.alpha, self.beta = alpha, beta

    def compute(self, input_vals, output_val=None, stream_handle=None):
        c, a, b = input_vals
        r = KG.matmul(a, b, False, False)
        if self.alpha != 1.0:
            r = r * self.alpha
        return r + (c.to(r.dtype) * self.beta if self.beta != 1.0 else c.to(r.dtype))

    def gradient(self, output_grad):
        from .basic import mul_byconst_op
        c = self.raw_ctx
        ga = matmul_op(output_grad, self.inputs[2], False, True, ctx=c)
        gb = matmul_op(self.inputs[1], output_grad, True, False, ctx=c)
        if self.alpha != 1.0:
            ga, gb = mul_byconst_op(ga, self.alpha, ctx=c), mul_byconst_op(gb, self.alpha, ctx=c)
        return [addmm_gradient_op(self.inputs[0], output_grad, self.beta, ctx=c), ga, gb]

    def infer_shape(self, input_shapes):
        return (input_shapes[1][0], input_shapes[2][1])


class AddmmGradientOp(Op):
    shape_only_inputs = (0,)

    def __init__(self, inp, grad, beta=1.0, ctx=None):
        super().__init__(AddmmGradientOp, [inp, grad], ctx)
        self.beta = beta

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels.reduce import sum_to_shape
        shape, g = input_vals
        r = sum_to_shape(g, tuple(shape))
        return r * self.beta if self.beta != 1.0 else r

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[0]


def addmm_op(node_A, node_B, node_C, alpha=1.0, beta=1.0, ctx=None):
    return AddmmOp(node_A, node_B, node_C, alpha, beta, ctx=ctx)


def addmm_gradient_op(node_input, node_grad, beta=1.0, ctx=None):
    return AddmmGradientOp(node_input, node_grad, beta, ctx=ctx)


class BatchMatMulOp(Op):
    def __init__(self, a, b, trans_A=False, trans_B=False, ctx=None):
        super().__init__(BatchMatMulOp, [a, b], ctx)
        self.matmul_attr_trans_A, self.matmul_attr_trans_B = trans_A, trans_B

    def compute(self, input_vals, output_val=None, stream_handle=None):
        a, b = input_vals
        return KG.bmm(a, b, self.matmul_attr_trans_A, self.matmul_attr_trans_B)

    def gradient(self, output_grad):
        ta, tb = self.matmul_attr_trans_A, self.matmul_attr_trans_B
        A, B, G = self.inputs[0], self.inputs[1], output_grad
        c = self.raw_ctx
        if not ta and not tb:
            return [batch_matmul_op(G, B, False, True, ctx=c), batch_matmul_op(A, G, True, False, ctx=c)]
        if ta and not tb:
            return [batch_matmul_op(B, G, False, True, ctx=c), batch_matmul_op(A, G, False, False, ctx=c)]
        if not ta and tb:
            return [batch_matmul_op(G, B, False, False, ctx=c), batch_matmul_op(G, A, True, False, ctx=c)]
        return [batch_matmul_op(B, G, True, True, ctx=c), batch_matmul_op(G, A, True, True, ctx=c)]

    def infer_shape(self, input_shapes):
        a, b = input_shapes
        m = a[-1] if self.matmul_attr_trans_A else a[-2]
        n = b[-2] if self.matmul_attr_trans_B else b[-1]
        return tuple(a[:-2]) + (m, n)


def batch_matmul_op(node_A, node_B, trans_A=False, trans_B=False, ctx=None):
    return BatchMatMulOp(node_A, node_B, trans_A, trans_B, ctx=ctx)


class BaddbmmOp(Op):
    def __init__(self, inp, a, b, alpha=1.0, beta=1.0, ctx=None):
        super().__init__(BaddbmmOp, [inp, a, b], ctx)
        self.alpha, self.beta = alpha, beta

    def compute(self, input_vals, output_val=None, stream_handle=None):
        c, a, b = input_vals
        r = KG.bmm(a, b, False, False)
        return r * self.alpha + c.to(r.dtype) * self.beta

    def gradient(self, output_grad):
        from .basic import mul_byconst_op
        c = self.raw_ctx
        ga = mul_byconst_op(batch_matmul_op(output_grad, self.inputs[2], False, True, ctx=c), self.alpha, ctx=c)
        gb = mul_byconst_op(batch_matmul_op(self.inputs[1], output_grad, True, False, ctx=c), self.alpha, ctx=c)
        return [addmm_gradient_op(self.inputs[0], output_grad, self.beta, ctx=c), ga, gb]

    def infer_shape(self, input_shapes):
        return tuple(input_shapes[1][:-1]) + (input_shapes[2][-1],)


def baddbmm_op(node_A, node_B, node_C, alpha=1.0, beta=1.0, ctx=None):
    return BaddbmmOp(node_A, node_B, node_C, alpha, beta, ctx=ctx)


class CsrmvOp(Op):
    def __init__(self, a, b, trans=False, ctx=None):
        super().__init__(CsrmvOp, [a, b], ctx)
        self.trans = trans

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import spmm as KSP
        return KSP.csrmv(input_vals[0], input_vals[1], self.trans)

    def gradient(self, output_grad):
        return [None, csrmv_op(self.inputs[0], output_grad, not self.trans, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = input_shapes[0]
        return (s[1],) if self.trans else (s[0],)


class CsrmmOp(Op):
    def __init__(self, a, b, trans_A=False, trans_B=False, ctx=None):
        super().__init__(CsrmmOp, [a, b], ctx)
        self.trans_A, self.trans_B = trans_A, trans_B

    def compute(self, input_vals, output_val=None, stream_handle=None):
        from ..kernels import spmm as KSP
        return KSP.csrmm(input_vals[0], input_vals[1], self.trans_A, self.trans_B)

    def gradient(self, output_grad):
        return [None, csrmm_op(self.inputs[0], output_grad, not self.trans_A, False, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        a, b = input_shapes
        m = a[1] if self.trans_A else a[0]
        n = b[0] if self.trans_B else b[1]
        return (m, n)


def csrmv_op(node_A, node_B, trans=False, ctx=None):
    return CsrmvOp(node_A, node_B, trans, ctx=ctx)


def csrmm_op(node_A, node_B, trans_A=False, trans_B=False, ctx=None):
    return CsrmmOp(node_A, node_B, trans_A, trans_B, ctx=ctx)
