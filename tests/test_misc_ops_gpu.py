"""misc_ops.hip (SAM gate helpers, instance norm 2d, bicubic interpolation) through the
graph ops that route to them, against PyTorch fp32 references of the same ops
(reference tests/test_gpu_op.py pattern).  Checks that the native kernels ran and
nothing fell back."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import hetu_61a7_amd as ht
from hetu_61a7_amd import kernels as K
from hetu_61a7_amd.kernels import tensor as KT
from hetu_61a7_amd.ops import moe as M
from hetu_61a7_amd.ops import nn as NN
from hetu_61a7_amd.ops import shape as SH

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _stats():
    K.reset_dispatch_stats()
    yield
    assert not K.FALLBACKS, K.FALLBACKS


def _close(a, b, tol=1e-5):
    np.testing.assert_allclose(np.asarray(a.cpu(), np.float64), np.asarray(b.cpu(), np.float64), rtol=tol, atol=tol)


def test_sam_ops_match_torch_formulas():
    T, G, n = 50, 4, 8
    E = G * n
    x = torch.softmax(torch.randn(T, E, device='cuda'), -1)
    op = M.SamGroupSumOp.__new__(M.SamGroupSumOp)
    op.num_local_gpus = G
    _close(op.compute([x]), x.reshape(T, G, n).sum(-1))
    g = torch.randn(T, G, device='cuda')
    gop = M.SamGroupSumGradOp.__new__(M.SamGroupSumGradOp)
    gop.num_local_gpus = G
    _close(gop.compute([g, (T, E)]), g.unsqueeze(-1).expand(T, G, n).reshape(T, E))
    grp = torch.randint(0, G, (T,), device='cuda')
    tk = grp * n + torch.randint(0, n, (T,), device='cuda')
    mask, diff = M._sam_mask(x, grp, tk, n)
    sop = M.SamMaxOp.__new__(M.SamMaxOp)
    sop.num_local_gpus = n
    _close(sop.compute([x, grp, tk]), torch.where(mask, diff, torch.zeros_like(diff)))
    gy = torch.randn(T, E, device='cuda')
    gm = torch.where(mask, gy, torch.zeros_like(gy))
    ref = gm.clone().scatter_add_(1, tk.reshape(-1, 1), -gm.sum(1, keepdim=True))
    smg = M.SamMaxGradOp.__new__(M.SamMaxGradOp)
    smg.num_local_gpus = n
    _close(smg.compute([gy, x, grp, tk]), ref)
    for k in (1, 2, 5):
        top = M.GroupTopKIdxOp.__new__(M.GroupTopKIdxOp)
        top.k, top.num_local_gpus = k, n
        got = top.compute([x, grp])
        cols = torch.arange(E, device='cuda')[None]
        inside = (cols >= (grp * n)[:, None]) & (cols < ((grp + 1) * n)[:, None])
        vals = torch.topk(torch.where(inside, x, torch.full_like(x, -1e4)), k, 1)[0]
        assert torch.equal(torch.gather(x, 1, got), vals)
        assert bool(((got >= (grp * n)[:, None]) & (got < ((grp + 1) * n)[:, None])).all())
    assert K.NATIVE_CALLS.get('group_topk_idx', 0) == 3 and K.NATIVE_CALLS.get('sam_max_grad', 0) == 1


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('channels_last', [False, True])
def test_instance_norm2d(dtype, channels_last):
    x = torch.randn(3, 5, 7, 9, device='cuda').to(dtype) * 2 + 1
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    fwd = NN.Instance_Normalization2dOp.__new__(NN.Instance_Normalization2dOp)
    fwd.eps = 1e-5
    res = fwd.compute([x])
    y, (mean, rstd) = res.value, res.aux
    xr = x.float().cpu().double().requires_grad_(True)
    yr = F.instance_norm(xr, eps=1e-5)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    _close(y.float(), yr.detach(), tol)
    g = torch.randn_like(y)
    yr.backward(g.float().cpu().double())
    bwd = NN.Instance_Normalization2d_GradientOp.__new__(NN.Instance_Normalization2d_GradientOp)
    _close(bwd.compute([g, x, (mean, rstd)]).float(), xr.grad, tol * 5)
    assert K.NATIVE_CALLS.get('instance_norm2d', 0) == 1 and K.NATIVE_CALLS.get('instance_norm2d_grad', 0) == 1


@pytest.mark.parametrize('size,scale,align', [((13, 21), None, False), ((13, 21), None, True),
                                              (None, 2.0, False), (None, 1.5, True), ((4, 3), None, False)])
def test_bicubic_matches_torch(size, scale, align):
    x = torch.randn(2, 3, 8, 10, device='cuda')
    op = SH.InterpolateOp.__new__(SH.InterpolateOp)
    op.size, op.scale_factor, op.mode, op.align_corners = size, scale, 'bicubic', align
    y = op.compute([x])
    xr = x.cpu().double().requires_grad_(True)
    yr = F.interpolate(xr, size=size, scale_factor=scale, mode='bicubic', align_corners=align)
    _close(y, yr.detach(), 1e-5)
    g = torch.randn_like(y)
    yr.backward(g.cpu().double())
    gop = SH.InterpolateGradOp.__new__(SH.InterpolateGradOp)
    gop.mode, gop.align_corners, gop.scale_factor = 'bicubic', align, None if size is not None else scale
    _close(gop.compute([g, tuple(x.shape)]), xr.grad, 1e-4)
    assert K.NATIVE_CALLS.get('bicubic', 0) == 1 and K.NATIVE_CALLS.get('bicubic_grad', 0) == 1
