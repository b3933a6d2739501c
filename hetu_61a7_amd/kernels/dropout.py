"""Philox dropout (``dropout.hip``): y = x * (u < keep) / keep with u drawn from
Philox4x32-10 at counter = element index, so the backward regenerates the mask
from the seed (reference Dropout.cu `curand_init(seed, 0, idx)` semantics)."""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32, F32


def dropout(x, keep_prob, seed):
    if native(x) and supported_float(x):
        xc = x.contiguous()
        y = _NA.empty_like(xc)
        f = fn('hetu_dropout', [P, P, I64, F32, I64, I32, P])
        check(f(xc.data_ptr(), y.data_ptr(), xc.numel(), float(keep_prob), int(seed), is_bf16(x),
                stream_ptr()), 'dropout')
        return y
    if x.is_cuda:
        raise RuntimeError('dropout: no hand-written kernel for %s on %s (fp32 / bf16 only)' % (x.dtype, x.device))
    from . import cpu_native
    if cpu_native.active(x):
        return cpu_native.dropout(x, keep_prob, seed)
    g = torch.Generator(device=x.device)
    g.manual_seed(int(seed) & 0x7FFFFFFF)
    mask = torch.rand(x.shape, generator=g, device=x.device) < keep_prob
    return (x.float() * mask / keep_prob).to(x.dtype)
