"""Fused transformer kernels on the GPU vs torch fp32 references."""
import pytest
import torch

from test_fused_ln_cpu import fused_ln_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('N', [768, 1024, 64, 2048])
@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_fp32(N, keep):
    fused_ln_check('cuda', torch.float32, R=300, N=N, keep=keep, tol=2e-5)


@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_bf16(keep):
    fused_ln_check('cuda', torch.bfloat16, R=257, N=768, keep=keep)


@pytest.mark.parametrize('S', [32, 64, 96, 128, 256])
@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_packed_attention_bf16(S, keep):
    from test_bert_cpu import packed_attention_check
    packed_attention_check('cuda', torch.bfloat16, B=3, S=S, NH=2, D=64, keep=keep, tol=2.5e-2)


def test_bert_fused_attention_gpu_bf16_trains():
    import numpy as np
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    out, init = [], None
    for fused in (False, True):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=2000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                         intermediate_size=256, batch_size=4, seq_len=64, max_position_embeddings=64,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, fused_attention=fused)
        feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-3)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=2, mixed_precision='bf16')
        from hetu_61a7_amd.utils.checkpoint import state_dict, load_dict
        if init is None:
            init = state_dict(ex)
        else:
            load_dict(ex, init)      # fp32 masters AND their bf16 compute copies
        fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
        out.append([float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
                    for _ in range(6)])
    np.testing.assert_allclose(out[0], out[1], rtol=3e-2, atol=3e-2)
    assert out[1][-1] < out[1][0]


@pytest.mark.gpu
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('keep', [1.0, 0.9])
@pytest.mark.parametrize('R,N', [(1000, 768), (37, 64)])
def test_ln_backward_emits_linear_bias_grad(dt, keep, R, N):
    """The fused LayerNorm backward's extra output (column sums of the x-gradient,
    the producing linear layer's bias gradient) equals dx summed over rows, with
    the row-slice atomics (many blocks) and with a single block."""
    from hetu_61a7_amd.kernels import layernorm as KLN
    torch.manual_seed(0)
    x = torch.randn(R, N, device='cuda').to(dt)
    res = torch.randn(R, N, device='cuda').to(dt)
    g = torch.rand(N, device='cuda') + 0.5
    b = torch.randn(N, device='cuda')
    y, s, mean, rstd = KLN.layer_norm_fused(x, res, g, b, 1e-12, keep, 1234)
    dy = torch.randn(R, N, device='cuda').to(dt)
    ds, dx, dg, db, dl = KLN.layer_norm_fused_backward(dy, s, g, mean, rstd, keep, 1234, want_dlin=True)
    ds0, dx0, dg0, db0 = KLN.layer_norm_fused_backward(dy, s, g, mean, rstd, keep, 1234)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0) and torch.equal(ds, ds0)
    ref = dx.float().sum(0)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-3
    torch.testing.assert_close(dl, ref, rtol=tol, atol=tol * (R ** 0.5))
    torch.testing.assert_close(dg, dg0, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, db0, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize('R,N', [(8192, 768), (1000, 1024), (37, 64)])
def test_ln_backward_8_wave_blocks_match_4_wave_blocks(R, N, monkeypatch):
    """The 8-waves-per-block LayerNorm backward (default) gives the 4-wave kernel's row
    gradients bit for bit and its dgamma / dbeta / bias column sums up to summation order,
    and both match the fp32 torch backward."""
    from hetu_61a7_amd.kernels import layernorm as KLN
    torch.manual_seed(1)
    dt = torch.bfloat16
    x = torch.randn(R, N, device='cuda').to(dt)
    res = torch.randn(R, N, device='cuda').to(dt)
    g = torch.rand(N, device='cuda') + 0.5
    b = torch.randn(N, device='cuda')
    y, s, mean, rstd = KLN.layer_norm_fused(x, res, g, b, 1e-12, 0.9, 77)
    dy = torch.randn(R, N, device='cuda').to(dt)
    out = {}
    for wv in (4, 8):
        monkeypatch.setattr(KLN, '_LN_BWD_WAVES', wv)
        out[wv] = KLN.layer_norm_fused_backward(dy, s, g, mean, rstd, 0.9, 77, want_dlin=True)
    for i in (0, 1):
        assert torch.equal(out[4][i], out[8][i])
    for i in (2, 3, 4):
        torch.testing.assert_close(out[8][i], out[4][i], rtol=1e-4, atol=1e-3)
    sf = s.float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(sf, (N,), g, b, 1e-12)
    ref.backward(dy.float())
    rel = (out[8][0].float() - sf.grad).norm() / sf.grad.norm()
    assert rel < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('R,N', [(8192, 3072), (100, 40), (3, 1024)])
def test_gelu_grad_colsum_matches_torch(dt, R, N):
    """hetu_gelu_grad_colsum: g = dy * gelu'(pre) and its column sums vs torch fp32."""
    from hetu_61a7_amd.kernels.layernorm import gelu_grad_colsum
    torch.manual_seed(0)
    pre = torch.randn(R, N, device='cuda').to(dt)
    dy = torch.randn(R, N, device='cuda').to(dt)
    g, cs = gelu_grad_colsum(pre, dy)
    x = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(dy.float())
    ref = x.grad
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(g.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(cs, ref.sum(0), rtol=tol, atol=tol * (R ** 0.5) * 4)


@pytest.mark.parametrize('mode', ['split', 'fused', 'w8'])
@pytest.mark.parametrize('S,keep', [(32, 1.0), (96, 0.9), (128, 1.0), (128, 0.9)])
def test_packed_attention_backward_forms(monkeypatch, mode, S, keep):
    """every form of the fixed-length backward (two-launch workspace, one 4-wave launch,
    one 8-wave launch with the dQ exchange in LDS) against the fp32 reference, and the
    forms against each other on the same operands"""
    from hetu_61a7_amd.kernels import attention as KA
    from test_bert_cpu import packed_attention_check
    monkeypatch.setattr(KA, '_BWD_MODE', mode)
    monkeypatch.setattr(KA, '_BWD_SPLIT', mode == 'split')
    packed_attention_check('cuda', torch.bfloat16, B=3, S=S, NH=2, D=64, keep=keep, tol=2.5e-2)
    B, NH, D = 4, 3, 64
    g = torch.Generator(device='cuda').manual_seed(S)
    qkv = (torch.randn((B * S, 3 * NH * D), device='cuda', generator=g) * 0.5).bfloat16()
    mask = torch.zeros(B, S, device='cuda')
    mask[1, S - 7:] = -10000.0
    out, lse = KA.attention_fwd(qkv, mask, B, S, NH, keep, 77)
    do = torch.randn(out.shape, device='cuda', generator=g).bfloat16()
    got = KA.attention_bwd(do, qkv, out, lse, mask, B, S, NH, keep, 77).float()
    monkeypatch.setattr(KA, '_BWD_MODE', 'split')
    monkeypatch.setattr(KA, '_BWD_SPLIT', True)
    ref = KA.attention_bwd(do, qkv, out, lse, mask, B, S, NH, keep, 77).float()
    assert float((got - ref).norm() / ref.norm()) < 1e-2


@pytest.mark.parametrize('waves', [4, 8])
@pytest.mark.parametrize('R,N,keep', [(257, 768, 0.9), (300, 1024, 1.0), (64, 64, 0.9), (513, 2048, 0.9)])
def test_ln_backward_waves(monkeypatch, waves, R, N, keep):
    """the LayerNorm backward at 4 and 8 rows in flight per block against the fp32
    reference, and against each other on the same operands: dsum, dx through the dropout
    mask, dgamma, dbeta and the linear-bias sums"""
    from hetu_61a7_amd.kernels import layernorm as KLN
    monkeypatch.setattr(KLN, '_LN_BWD_WAVES', waves)
    fused_ln_check('cuda', torch.bfloat16, R=R, N=N, keep=keep)
    g = torch.Generator(device='cuda').manual_seed(R)
    x, res, dy = (torch.randn(R, N, device='cuda', generator=g).bfloat16() for _ in range(3))
    gam = torch.rand(N, device='cuda', generator=g) + 0.5
    bet = torch.randn(N, device='cuda', generator=g)
    y, s, mean, rstd = KLN.layer_norm_fused(x, res, gam, bet, 1e-12, keep, 5)
    got = KLN.layer_norm_fused_backward(dy, s, gam, mean, rstd, keep, 5, want_dlin=True)
    monkeypatch.setattr(KLN, '_LN_BWD_WAVES', 4 if waves == 8 else 8)
    ref = KLN.layer_norm_fused_backward(dy, s, gam, mean, rstd, keep, 5, want_dlin=True)
    for a, b in zip(got, ref):
        a, b = a.float(), b.float()
        assert float((a - b).norm() / b.norm().clamp_min(1e-12)) < 1e-2

