"""Row softmax and fused softmax-cross-entropy (``softmax.hip``)."""
from __future__ import annotations

import torch
from .. import native_array as _NA

from . import fn, native, stream_ptr, is_bf16, check, supported_float, P, I64, I32


def _rows(x):
    return x.reshape(-1, x.shape[-1])


def softmax(x: torch.Tensor, log: bool = False) -> torch.Tensor:
    """Softmax over the last dim."""
    if native(x) and supported_float(x):
        x = x.contiguous()
        y = _NA.empty_like(x)
        R, N = x.numel() // x.shape[-1], x.shape[-1]
        f = fn('hetu_softmax_fwd', [P, P, I64, I32, I32, I32, P])
        check(f(x.data_ptr(), y.data_ptr(), R, N, is_bf16(x), int(log), stream_ptr()), 'softmax')
        return y
    from . import cpu_native
    if cpu_native.active(x) and x.dim() > 0:
        return cpu_native.softmax(x, log)
    cpu_native.record_fallback('softmax', x)
    xf = x.float()
    return (torch.log_softmax(xf, -1) if log else torch.softmax(xf, -1)).to(x.dtype)


def softmax_backward(y: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    if native(y) and supported_float(y) and dy.dtype == y.dtype:
        y = y.contiguous()
        dy = dy.contiguous()
        dx = _NA.empty_like(y)
        R, N = y.numel() // y.shape[-1], y.shape[-1]
        f = fn('hetu_softmax_bwd', [P, P, P, I64, I32, I32, P])
        check(f(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), R, N, is_bf16(y), stream_ptr()), 'softmax_bwd')
        return dx
    from . import cpu_native
    if cpu_native.active(y, dy) and y.dim() > 0 and dy.shape == y.shape:
        return cpu_native.softmax_backward(y, dy)
    cpu_native.record_fallback('softmax_backward', y, dy)
    yf, gf = y.float(), dy.float()
    return (yf * (gf - (gf * yf).sum(-1, keepdim=True))).to(y.dtype)


def softmax_ce(logits: torch.Tensor, labels: torch.Tensor):
    """Per-row loss -sum(y*log_softmax(x)) and the row log-sum-exp."""
    if native(logits) and supported_float(logits) and supported_float(labels):
        x = logits.contiguous()
        lab = labels.contiguous()
        R, N = x.numel() // x.shape[-1], x.shape[-1]
        loss = _NA.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
        lse = _NA.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
        f = fn('hetu_softmax_ce_fwd', [P, P, P, P, I64, I32, I32, I32, P])
        check(f(x.data_ptr(), lab.data_ptr(), loss.data_ptr(), lse.data_ptr(), R, N,
                is_bf16(x), is_bf16(lab), stream_ptr()), 'softmax_ce')
        return loss, lse
    from . import cpu_native
    if cpu_native.active(logits, labels) and logits.dim() >= 1 and labels.shape == logits.shape:
        loss, lse = cpu_native.softmax_ce(_rows(logits), _rows(labels))
        return loss.reshape(logits.shape[:-1]), lse.reshape(logits.shape[:-1])
    cpu_native.record_fallback('softmax_ce', logits, labels)
    xf = logits.float()
    lse = torch.logsumexp(xf, -1)
    loss = (labels.float() * (lse.unsqueeze(-1) - xf)).sum(-1)
    return loss, lse


def _grad_rows(grad):
    """(g, is_scalar): a per-row loss gradient, or one value broadcast to every row
    (a reduce-mean gradient arrives as an expanded view with all strides 0: its first
    element is read in place, no materialising copy)"""
    if grad.numel() == 1 or (grad.dim() > 0 and all(st == 0 for st in grad.stride())):
        return grad.as_strided((1,), (1,)), True
    return grad.contiguous(), False


def softmax_ce_backward(logits, labels, grad, lse=None):
    """d logits = grad[r] * (softmax(x)*sum(y) - y); ``grad`` per row or scalar."""
    if grad.dtype != torch.float32:
        grad = grad.float()
    if native(logits) and supported_float(logits) and supported_float(labels):
        x = logits.contiguous()
        lab = labels.contiguous()
        g, scalar = _grad_rows(grad)
        R, N = x.numel() // x.shape[-1], x.shape[-1]
        dx = _NA.empty_like(x)
        f = fn('hetu_softmax_ce_bwd', [P, P, P, I32, P, P, I64, I32, I32, I32, P])
        check(f(x.data_ptr(), lab.data_ptr(), g.data_ptr(), int(scalar),
                lse.contiguous().data_ptr() if lse is not None else None, dx.data_ptr(), R, N,
                is_bf16(x), is_bf16(lab), stream_ptr()), 'softmax_ce_bwd')
        return dx
    grad = grad.float()
    from . import cpu_native
    if cpu_native.active(logits, labels) and logits.dim() >= 1 and labels.shape == logits.shape:
        if lse is None:
            _, lse = softmax_ce(logits, labels)
        R = logits.numel() // logits.shape[-1]
        g, scalar = _grad_rows(grad)
        g = g.reshape(-1) if scalar else g.reshape(R)
        return cpu_native.softmax_ce_backward(_rows(logits), _rows(labels), g, lse.reshape(R)).reshape(logits.shape)
    cpu_native.record_fallback('softmax_ce_backward', logits, labels)
    xf = logits.float()
    yl = labels.float()
    sm = torch.softmax(xf, -1)
    g = grad if grad.numel() == 1 else grad.unsqueeze(-1)
    return (g * (sm * yl.sum(-1, keepdim=True) - yl)).to(logits.dtype)


def softmax_ce_sparse(logits, labels, ignored_index=-1):
    lab = labels.reshape(-1).long()
    if native(logits) and supported_float(logits):
        x = logits.contiguous()
        lab = lab.contiguous()
        R, N = x.numel() // x.shape[-1], x.shape[-1]
        loss = _NA.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
        lse = _NA.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
        f = fn('hetu_softmax_ce_sparse_fwd', [P, P, P, P, I64, I32, I32, I64, P])
        check(f(x.data_ptr(), lab.data_ptr(), loss.data_ptr(), lse.data_ptr(), R, N, is_bf16(x),
                int(ignored_index), stream_ptr()), 'softmax_ce_sparse')
        return loss, lse
    from . import cpu_native
    if cpu_native.active(logits):
        return cpu_native.softmax_ce_sparse(logits, lab, ignored_index)
    xf = _rows(logits.float())
    lse = torch.logsumexp(xf, -1)
    valid = (lab != ignored_index) & (lab >= 0) & (lab < xf.shape[-1])
    safe = torch.where(valid, lab, _NA.zeros_like(lab))
    picked = xf.gather(1, safe.unsqueeze(1)).squeeze(1)
    loss = torch.where(valid, lse - picked, _NA.zeros_like(lse))
    return loss.reshape(logits.shape[:-1]), lse.reshape(logits.shape[:-1])


def softmax_ce_sparse_backward(logits, labels, grad, lse=None, ignored_index=-1):
    lab = labels.reshape(-1).long()
    if grad.dtype != torch.float32:
        grad = grad.float()
    if native(logits) and supported_float(logits):
        x = logits.contiguous()
        R, N = x.numel() // x.shape[-1], x.shape[-1]
        dx = _NA.empty_like(x)
        g, scalar = _grad_rows(grad)
        f = fn('hetu_softmax_ce_sparse_bwd', [P, P, P, I32, P, P, I64, I32, I32, I64, P])
        check(f(x.data_ptr(), lab.contiguous().data_ptr(), g.data_ptr(), int(scalar),
                lse.contiguous().data_ptr() if lse is not None else None, dx.data_ptr(), R, N,
                is_bf16(x), int(ignored_index), stream_ptr()), 'softmax_ce_sparse_bwd')
        return dx
    grad = grad.float()
    from . import cpu_native
    if cpu_native.active(logits):
        if lse is None:
            _, lse = softmax_ce_sparse(logits, labels, ignored_index)
        g, scalar = _grad_rows(grad)
        return cpu_native.softmax_ce_sparse_backward(logits, lab, g.contiguous(), scalar, lse, ignored_index)
    xf = _rows(logits.float())
    sm = torch.softmax(xf, -1)
    valid = (lab != ignored_index) & (lab >= 0) & (lab < xf.shape[-1])
    safe = torch.where(valid, lab, _NA.zeros_like(lab))
    onehot = torch.nn.functional.one_hot(safe, xf.shape[-1]).float()
    g = grad.reshape(-1, 1) if grad.numel() > 1 else grad
    d = g * (sm - onehot) * valid.float().unsqueeze(1)
    return d.reshape(logits.shape).to(logits.dtype)
