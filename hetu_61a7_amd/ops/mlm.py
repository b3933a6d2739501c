"""Masked-LM head over the masked positions only (kernels/mlm.py, ``mlm_gather.hip``).

BERT pretraining scores every token against the vocabulary in the reference and ignores
the unmasked ones in the loss (examples/nlp/bert/hetu_bert.py: softmaxcrossentropy_sparse_op
over [B*S, V] with ignored_index=-1); the original BERT gathers the masked positions
first (max_predictions_per_seq).  ``masked_positions_op`` compacts the labelled rows into
C slots per sequence, ``take_rows_op`` gathers rows (hidden states, labels) into the slots
and its gradient writes them back (every other row zero): the head's GEMMs and softmax-CE
then run over B*C rows, with the same loss and gradients while no sequence has more than C
labels (the kernel flags an overflow; ``MaskedPositionsOp.check()`` raises on it).
"""
from __future__ import annotations

import torch

from .. import native_array as _NA
from .node import Op
from ..kernels import mlm as KM


class MaskedPositionsOp(Op):
    def __init__(self, labels, per_seq, ctx=None):
        super().__init__(MaskedPositionsOp, [labels], ctx)
        from .loss import _label_feed
        _label_feed(labels)          # class indices: never cast to bf16 by a mixed-precision feed
        self.per_seq = int(per_seq)
        self.overflow = None

    def compute(self, input_vals, output_val=None, stream_handle=None):
        lab = input_vals[0]
        if self.overflow is None or self.overflow.device != lab.device:
            from ..kernels.tensor import zeros
            self.overflow = zeros((1,), torch.int32, lab.device) if lab.is_cuda else torch.zeros(1, dtype=torch.int32)
        return KM.masked_positions(lab.reshape(lab.shape[0], -1), self.per_seq, self.overflow)

    def check(self):
        """raise if a batch had a sequence with more labels than slots (synchronises)"""
        if self.overflow is not None and int(self.overflow.reshape(-1)[0].item()) > 0:
            raise RuntimeError('masked_positions_op: a sequence had %d labelled positions, more than '
                               'max_predictions_per_seq=%d' % (int(self.overflow.reshape(-1)[0].item()),
                                                               self.per_seq))

    def gradient(self, output_grad):
        return [None]

    def infer_shape(self, input_shapes):
        return (input_shapes[0][0] * self.per_seq,)


class TakeRowsOp(Op):
    def __init__(self, x, idx, fill_neg1=False, ctx=None):
        super().__init__(TakeRowsOp, [x, idx], ctx)
        self.fill_neg1 = bool(fill_neg1)
        if self.fill_neg1:           # a label gather: its source feed stays fp32 / integer
            from .loss import _label_feed
            _label_feed(x)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x, idx = input_vals
        if self.fill_neg1:
            x = x.reshape(-1)
        return KM.take_rows(x, idx, self.fill_neg1)

    def gradient(self, output_grad):
        if self.fill_neg1:
            return [None, None]
        return [PutRowsOp(output_grad, self.inputs[1], self.inputs[0], ctx=self.raw_ctx), None]

    def infer_shape(self, input_shapes):
        x, idx = input_shapes
        if self.fill_neg1:
            return (idx[0],)
        return (idx[0],) + tuple(x[1:])


class PutRowsOp(Op):
    shape_only_inputs = (2,)

    def __init__(self, grad, idx, ref, ctx=None):
        super().__init__(PutRowsOp, [grad, idx, ref], ctx)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        g, idx, shape = input_vals
        return KM.put_rows(g, idx, int(tuple(shape)[0]))

    def gradient(self, output_grad):
        raise NotImplementedError

    def infer_shape(self, input_shapes):
        return input_shapes[2]


def masked_positions_op(labels, per_seq, ctx=None):
    return MaskedPositionsOp(labels, per_seq, ctx=ctx)


def take_rows_op(x, idx, fill_neg1=False, ctx=None):
    return TakeRowsOp(x, idx, fill_neg1, ctx=ctx)
