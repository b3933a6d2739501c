"""Weight-gradient GEMM paths (long K, small M x N, fp32 output into the flat
gradient buffer): every MFMA split-K depth and the autotuned entry point against a
plain fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('M,N,K', [(768, 768, 8192), (768, 3072, 8192), (256, 320, 4096)])
def test_weight_grad_paths_match_fp32(M, N, K):
    from hetu_61a7_amd.kernels import gemm as KG, gemm_mfma
    torch.manual_seed(0)
    x = torch.randn(K, M, device='cuda').bfloat16()   # activations [tokens, in]
    g = torch.randn(K, N, device='cuda').bfloat16()   # output grads [tokens, out]
    ref = x.float().t() @ g.float()
    A, B = x.t(), g
    outs = {}
    for s in (1, 2, 4, 8):
        o = torch.empty(M, N, device='cuda')
        assert gemm_mfma.gemm(A, B, out=o, splitk=s) is not None
        outs['hip_sk%d' % s] = o
    o = torch.empty(M, N, device='cuda')
    outs['auto'] = KG.matmul_into(x, g, True, False, o)
    scale = ref.abs().max().item()
    for name, o in outs.items():
        err = (o - ref).abs().max().item() / scale
        assert err < 2e-2, (name, err)


@pytest.mark.gpu
@pytest.mark.parametrize('s,M,N', [(4, 768, 3072), (2, 64, 36), (8, 30522, 768), (3, 5, 4), (16, 256, 576), (11, 8, 12)])
def test_splitk_partial_sum_matches_torch(s, M, N):
    """kernels.gemm._splitk_sum (vectorised fp32 sum of split-K partials) == torch.sum."""
    from hetu_61a7_amd.kernels.gemm import _splitk_sum
    torch.manual_seed(0)
    part = torch.randn(s, M, N, device='cuda')
    out = torch.empty(M, N, device='cuda')
    _splitk_sum(part, out)
    torch.testing.assert_close(out, part.sum(0), rtol=1e-6, atol=1e-5)
