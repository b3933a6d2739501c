"""Exact-fp32 MFMA GEMM and implicit-GEMM convolution (csrc/kernels/gemm_f32.hip,
v_mfma_f32_16x16x4_f32) against fp64 references of the same ops -- the parity
(fp32) mode of the reference (src/ops/MatrixMult.cu, CudnnConv2d.cu)."""
import pytest
import torch
import torch.nn.functional as F

from hetu_61a7_amd.kernels import gemm_mfma as G, conv_igemm as CI

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.mark.parametrize('ta,tb', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('mnk', [(256, 192, 64), (131, 77, 36), (1024, 512, 1000)])
def test_gemm_f32_modes(ta, tb, mnk):
    M, N, K = mnk
    N = -(-N // 4) * 4 if tb == 0 else N
    M = -(-M // 4) * 4 if ta else M
    K = -(-K // 4) * 4
    a = torch.randn(K, M, device='cuda').t() if ta else torch.randn(M, K, device='cuda')
    b = torch.randn(N, K, device='cuda').t() if tb else torch.randn(K, N, device='cuda')
    y = G.gemm_f32(a, b)
    assert y is not None
    ref = a.double().cpu() @ b.double().cpu()
    assert _rel(y.cpu(), ref) < 2e-6


def test_gemm_f32_epilogue_and_batched():
    a = torch.randn(3, 200, 96, device='cuda')
    b = torch.randn(3, 96, 160, device='cuda')
    c = torch.randn(3, 200, 160, device='cuda')
    y = G.gemm_f32(a, b, cin=c, beta=0.5, alpha=2.0)
    ref = 2.0 * (a.double() @ b.double()) + 0.5 * c.double()
    assert _rel(y, ref) < 2e-6
    a2, b2 = a[0], b[0]
    bias = torch.randn(160, device='cuda')
    y2 = G.gemm_f32(a2, b2, bias=bias, act='relu')
    ref2 = torch.relu(a2.double() @ b2.double() + bias.double())
    assert _rel(y2, ref2) < 2e-6


@pytest.mark.parametrize('shape', [
    # N, C, H, K, k, stride, pad
    (2, 4, 17, 8, 7, 2, 3),
    (2, 16, 14, 32, 3, 1, 1),
    (2, 32, 15, 16, 3, 2, 1),
    (2, 64, 8, 64, 1, 1, 0),
    (2, 64, 9, 128, 1, 2, 0),
])
def test_conv_f32_passes(shape):
    N, C, H, K, k, s, p = shape
    x = torch.randn(N, C, H, H, device='cuda').contiguous(memory_format=CL)
    w = (torch.randn(K, C, k, k, device='cuda') * 0.1).contiguous(memory_format=CL)
    y = CI.forward_f32(x, w, (s, s), (p, p))
    xd, wd = x.double().cpu(), w.double().cpu()
    ref = F.conv2d(xd, wd, None, s, p)
    assert _rel(y.cpu(), ref) < 2e-6
    g = torch.randn_like(y).contiguous(memory_format=CL)
    dx = CI.backward_data_f32(g, w, x.shape, (s, s), (p, p))
    dw = CI.backward_filter_f32(g, x, w.shape, (s, s), (p, p))
    rdx, rdw, _ = torch.ops.aten.convolution_backward(g.double().cpu(), xd, wd, None, [s, s], [p, p], [1, 1],
                                                      False, [0, 0], 1, [True, True, False])
    assert _rel(dx.cpu(), rdx) < 2e-6
    assert _rel(dw.cpu(), rdw) < 2e-6
