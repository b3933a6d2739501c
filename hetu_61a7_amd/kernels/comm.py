"""Bindings of ``csrc/kernels/comm.hip``: the casts and the fp32-accumulated chunk sum
of the bf16-wire gradient all-reduce (``parallel/rccl.py``).  Each takes the HIP
stream to run on (the communicator's comm stream)."""
from __future__ import annotations

import torch

from . import fn, check, P, I32, I64


def cast_f32_bf16(x, y, stream):
    """y[:x.numel()] = bf16(x), y's tail zeroed."""
    check(fn('hetu_cast_f32_bf16', [P, P, I64, I64, P])(x.data_ptr(), y.data_ptr(), x.numel(), y.numel(), stream),
          'cast_f32_bf16')


def cast_bf16_f32(x, y, stream):
    """y = float(x[:y.numel()])."""
    check(fn('hetu_cast_bf16_f32', [P, P, I64, P])(x.data_ptr(), y.data_ptr(), y.numel(), stream), 'cast_bf16_f32')


def sum_chunks_bf16(inp, nchunks, c, out, stream):
    """out[j] = sum_p inp[p*c + j] (bf16 in/out, fp32 accumulation)."""
    check(fn('hetu_sum_chunks_bf16', [P, I32, I64, P, P])(inp.data_ptr(), int(nchunks), int(c), out.data_ptr(),
                                                           stream), 'sum_chunks_bf16')
