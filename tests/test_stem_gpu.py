"""Direct few-channel stem convolution (csrc/kernels/stem.hip) against a plain PyTorch
fp32 convolution of the same bf16 operands, with the fused BatchNorm statistics."""
import pytest
import torch
import torch.nn.functional as F

from hetu_61a7_amd import kernels as K
from hetu_61a7_amd.kernels import conv_igemm as CI

pytestmark = pytest.mark.gpu
CL = torch.channels_last


@pytest.mark.parametrize('n,c,h,k,s,p', [(2, 3, 224, 7, 2, 3), (3, 3, 37, 7, 2, 3), (2, 2, 20, 5, 1, 2),
                                         (1, 3, 15, 3, 2, 1)])
def test_stem_forward_and_stats(n, c, h, k, s, p):
    torch.manual_seed(0)
    x = torch.randn(n, c, h, h + 3, device='cuda').bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(64, c, k, k, device='cuda') * 0.1).bfloat16().contiguous(memory_format=CL)
    K.reset_dispatch_stats()
    st = torch.zeros(128, device='cuda')
    y = CI.try_stem_forward(x, w, (s, s), (p, p), colstats=st)
    assert y is not None and K.NATIVE_CALLS.get('stem_fwd') == 1
    ref = F.conv2d(x.float().cpu(), w.float().cpu(), None, s, p)
    assert y.shape == ref.shape
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err
    yb = y.float().cpu()
    torch.testing.assert_close(st[:64].cpu(), yb.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(st[64:].cpu(), (yb * yb).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert CI.try_stem_forward(x, w, (s, s), (p, p)).float().sub(y.float()).abs().max().item() == 0.0
    st3 = torch.zeros(3 * 128, device='cuda')   # replicated totals: block b into replica b % 3
    CI.try_stem_forward(x, w, (s, s), (p, p), colstats=st3)
    torch.testing.assert_close(st3.view(3, 128).sum(0), st, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize('n,c,h,wd,k,s,p', [(2, 3, 224, 224, 7, 2, 3), (3, 3, 37, 40, 7, 2, 3), (2, 2, 20, 24, 5, 1, 2),
                                            (1, 3, 15, 16, 3, 2, 1), (5, 3, 64, 64, 7, 2, 3)])
@pytest.mark.parametrize('accumulate', [False, True])
def test_stem_weight_gradient(n, c, h, wd, k, s, p, accumulate):
    """dW of the stem against fp32 autograd of the same bf16 operands: bf16 x bf16 products
    are exact in fp32, so only the summation order differs (relative error ~1e-6)."""
    torch.manual_seed(1)
    x = torch.randn(n, c, h, wd, device='cuda').bfloat16().contiguous(memory_format=CL)
    w = torch.zeros(64, c, k, k, device='cuda')
    oh, ow = (h + 2 * p - k) // s + 1, (wd + 2 * p - k) // s + 1
    dy = torch.randn(n, 64, oh, ow, device='cuda').bfloat16().contiguous(memory_format=CL)
    xr = x.float().cpu().requires_grad_(False)
    wr = w.float().cpu().requires_grad_(True)
    F.conv2d(xr, wr, None, s, p).backward(dy.float().cpu())
    ref = wr.grad
    out = torch.randn(64, c, k, k, device='cuda').contiguous(memory_format=CL)
    base = out.clone()
    K.reset_dispatch_stats()
    r = CI.try_stem_backward_filter(dy, x, (64, c, k, k), (s, s), (p, p), out=out, accumulate=accumulate)
    assert r is not None and K.NATIVE_CALLS.get('stem_wgrad') == 1
    got = (out - base).cpu() if accumulate else out.cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 1e-4
    assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-4
