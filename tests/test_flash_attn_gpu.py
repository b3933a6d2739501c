"""General fused attention (csrc/kernels/flash_attn.hip) against a plain fp32 torch
reference of the same op: softmax(q k^T * scale + mask [+ causal]) (dropout) v and its
gradients, over the shapes the reference workloads need -- the Transformer's maxlen-100
encoder, causal decoder and cross attention (examples/nlp/hetu_transformer.py:99-130,
hparams.py:48-50), BERT at 128 and phase 2 at 512 (examples/nlp/bert/hetu_bert.py:
220-271), ragged lengths and head dims 32 / 64 / 128.  Bound: relative Frobenius error
<= 3e-2 on the output and on each of dQ, dK, dV."""
import math

import numpy as np
import pytest
import torch

from hetu_61a7_amd.kernels import attention as KA
from hetu_61a7_amd.kernels.moe import philox4

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _dropmask(seed, B, NH, Sq, Sk, keep):
    sk4 = (Sk + 3) // 4
    rows = np.arange(B * NH * Sq, dtype=np.uint64)[:, None]
    keys = np.arange(Sk, dtype=np.uint64)[None, :]
    cnt = rows * np.uint64(sk4) + (keys >> np.uint64(2))
    outs = philox4(seed, cnt)
    comp = np.choose((keys & np.uint64(3)).astype(np.int64).repeat(rows.shape[0], 0), outs)
    u = (comp >> np.uint64(8)).astype(np.float64) / 16777216.0 + 0.5 / 16777216.0
    return torch.from_numpy(((u < keep) / keep).astype(np.float32)).reshape(B, NH, Sq, Sk)


def _ref(q, k, v, mask, causal, scale, dm):
    q, k, v = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    s = q @ k.transpose(-1, -2) * scale
    if mask is not None:
        s = s + mask.float()
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device), 1), float('-inf'))
    p = torch.softmax(s, -1)
    if dm is not None:
        p = p * dm.to(p.device)
    o = p @ v
    return o, (q, k, v)


def _case(B, NH, Sq, Sk, D, causal, masked, keep=1.0, layout='bhsd'):
    g = torch.Generator(device='cuda')
    g.manual_seed(Sq * 7 + Sk + D)
    mk = lambda S: torch.randn((B, S, NH, D), device='cuda', generator=g).bfloat16().permute(0, 2, 1, 3) \
        if layout == 'bshd' else torch.randn((B, NH, S, D), device='cuda', generator=g).bfloat16()
    q, k, v = mk(Sq), mk(Sk), mk(Sk)
    mask = None
    if masked:   # padding-style additive key mask [B, 1, 1, Sk] (the reference's -2^32 adder)
        lens = torch.randint(Sk // 2, Sk + 1, (B,), device='cuda', generator=g)
        mask = ((torch.arange(Sk, device='cuda')[None] >= lens[:, None]).float() * -1e9).reshape(B, 1, 1, Sk)
    scale = 1.0 / math.sqrt(D)
    seed = 1234 + Sq
    o, lse = KA.flash_fwd(q, k, v, mask, causal, keep, seed, scale)
    # the kernel's Philox key: the host seed moved by the device step counter (earlier
    # tests' dropout steps leave it non-zero)
    from hetu_61a7_amd.kernels import rng as KR
    dm = _dropmask(KR.effective_seed(seed), B, NH, Sq, Sk, keep) if keep < 1.0 else None
    ro, leaves = _ref(q, k, v, mask, causal, scale, dm)
    assert _rel(o, ro) < 3e-2, ('out', _rel(o, ro))
    do = torch.randn(ro.shape, device='cuda', generator=g)
    ro.backward(do)
    dq, dk, dv = KA.flash_bwd(do.bfloat16(), q, k, v, o, lse, mask, causal, keep, seed, scale)
    for name, a, b in (('dq', dq, leaves[0].grad), ('dk', dk, leaves[1].grad), ('dv', dv, leaves[2].grad)):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


@pytest.mark.parametrize('S', [100, 128, 384, 512])
@pytest.mark.parametrize('causal', [False, True])
def test_flash_self_attention_lengths(S, causal):
    _case(2, 4, S, S, 64, causal, masked=not causal)


@pytest.mark.parametrize('D', [32, 64, 128])
def test_flash_head_dims(D):
    _case(2, 3, 77, 77, D, False, masked=True)
    _case(1, 2, 130, 130, D, True, masked=False)


def test_flash_cross_attention_transformer_shapes():
    """decoder cross attention: 99 queries over 100 encoder keys, padding mask"""
    _case(2, 8, 99, 100, 64, False, masked=True, layout='bshd')


def test_flash_dropout_matches_reference_mask():
    _case(2, 2, 64, 96, 64, False, masked=True, keep=0.9)
    _case(1, 2, 100, 100, 64, True, masked=False, keep=0.8)


def test_flash_packed_bert_phase2_path():
    """BERT at seq 512 (phase 2): the packed-QKV op takes the flash kernels in place of
    the S <= 128 fused kernel; output and dQKV against fp32 math on the same packed rows"""
    B, S, NH, D = 2, 512, 4, 64
    H = NH * D
    g = torch.Generator(device='cuda')
    g.manual_seed(3)
    qkv = (torch.randn((B * S, 3 * H), device='cuda', generator=g) * 0.5).bfloat16()
    lens = torch.tensor([S, 300], device='cuda')
    mask = ((torch.arange(S, device='cuda')[None] >= lens[:, None]).float() * -1e4)
    out, lse = KA.attention_fwd(qkv, mask, B, S, NH)
    assert lse.dim() == 1
    q, k, v = (t.float() for t in KA.packed_heads(qkv, B, S, NH))
    ro, leaves = _ref(q, k, v, mask.reshape(B, 1, 1, S), False, 1.0 / math.sqrt(D), None)
    ro2 = ro.permute(0, 2, 1, 3).reshape(B * S, H)
    assert _rel(out, ro2) < 3e-2
    do = torch.randn(ro2.shape, device='cuda', generator=g)
    ro2.backward(do)
    dqkv = KA.attention_bwd(do.bfloat16(), qkv, out, lse, mask, B, S, NH)
    gq, gk, gv = KA.packed_heads(dqkv, B, S, NH)
    for a, b in ((gq, leaves[0].grad), (gk, leaves[1].grad), (gv, leaves[2].grad)):
        assert _rel(a, b) < 3e-2, _rel(a, b)


def test_transformer_step_launches_no_torch_kernels():
    """the Transformer example's training step (encoder, causal decoder, cross attention)
    issues no PyTorch or vendor-library kernel"""
    import collections
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models.transformer import Transformer, TransformerConfig, synthetic_batch
    from torch.profiler import profile, ProfilerActivity
    hp = TransformerConfig(vocab_size=2048, d_model=256, d_ff=512, num_blocks=2, num_heads=4, maxlen1=100,
                           maxlen2=100, dropout_rate=0.1, batch_size=8)
    xs, xm, ys, ym, lab = (ht.Variable(name=n) for n in ('xs', 'xm', 'ys', 'ym', 'lab'))
    loss, _ = Transformer(hp).train(xs, xm, ys, ym, lab)
    train = ht.optim.AdamOptimizer(1e-4).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=1)
    b = synthetic_batch(hp)
    fd = {xs: b['xs'], xm: b['src_mask'], ys: b['ys'], ym: b['tgt_mask'], lab: b['labels']}
    for _ in range(3):
        ex.run('train', feed_dict=fd)
    torch.cuda.synchronize()
    from hetu_61a7_amd import kernels as K
    K.reset_dispatch_stats()
    from hetu_61a7_amd.utils import hipgraph
    hipgraph.FORCE_EAGER[0] += 1        # an eager step: a graph replay would hide its kernels
    try:
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            ex.run('train', feed_dict=fd)
            torch.cuda.synchronize()
    finally:
        hipgraph.FORCE_EAGER[0] -= 1
    bad = collections.Counter(e.name[:100] for e in prof.events() if 'CUDA' in str(e.device_type) and
                              ('at::native' in e.name or 'Cijk' in e.name or 'MIOpen' in e.name))
    assert not bad, dict(bad)
    assert not K.VENDOR_CALLS and not K.FALLBACKS, (K.VENDOR_CALLS, K.FALLBACKS)


@pytest.mark.parametrize('S,keep,masked', [(128, 1.0, True), (128, 0.9, False), (64, 0.9, True), (96, 1.0, False)])
def test_seqblock_fast_path_matches_flash(S, keep, masked):
    """attention_op's BERT-length fast path (one workgroup per head, attention.hip) on head
    views of token-major rows equals the flash kernels on the same views -- outputs,
    gradients, and the dropout mask (same Philox layout) -- and is the path taken"""
    B, NH, D = 3, 4, 64
    g = torch.Generator(device='cuda').manual_seed(S)
    rows = [torch.randn(B, S, NH * D, generator=g, device='cuda').bfloat16() for _ in range(4)]
    q, k, v, do = (r.view(B, S, NH, D).permute(0, 2, 1, 3) for r in rows)
    mask = None
    if masked:
        mask = torch.zeros(B, 1, 1, S, device='cuda')
        mask[:, :, :, S - 17:] = -10000.0
    assert KA.seqblock_ok(q, k, v, mask, False) and not KA.seqblock_ok(q, k, v, mask, True)
    scale, seed = 1.0 / math.sqrt(D), 987654321
    o1, l1 = KA.seqblock_fwd(q, k, v, mask, keep, seed, scale)
    g1 = KA.seqblock_bwd(do, q, k, v, o1, l1, mask, keep, seed, scale)
    o2, l2 = KA.flash_fwd(q, k, v, mask, False, keep, seed, scale)
    g2 = KA.flash_bwd(do, q, k, v, o2, l2, mask, False, keep, seed, scale)
    torch.cuda.synchronize()
    assert _rel(o1, o2) < 1e-2
    assert _rel(l1.reshape(-1), l2.reshape(-1)) < 1e-4
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 2e-2


def test_attention_op_takes_seqblock_path(monkeypatch):
    import hetu_61a7_amd as ht
    calls = {'fwd': 0, 'bwd': 0}
    f0, b0 = KA.seqblock_fwd, KA.seqblock_bwd

    def fwd(*a, **k):
        calls['fwd'] += 1
        return f0(*a, **k)

    def bwd(*a, **k):
        calls['bwd'] += 1
        return b0(*a, **k)
    monkeypatch.setattr(KA, 'seqblock_fwd', fwd)
    monkeypatch.setattr(KA, 'seqblock_bwd', bwd)
    B, NH, S, D = 2, 4, 128, 64
    rng = np.random.RandomState(0)
    X = rng.randn(B, S, NH * D).astype(np.float32)
    x = ht.Variable(name='x')
    wq, wk, wv = (ht.init.xavier_normal((NH * D, NH * D), name=n) for n in ('wq', 'wk', 'wv'))

    def heads(t):
        return ht.transpose_op(ht.array_reshape_op(t, (B, S, NH, D)), (0, 2, 1, 3))
    x2 = ht.array_reshape_op(x, (B * S, NH * D))
    q, k, v = (heads(ht.matmul_op(x2, w)) for w in (wq, wk, wv))
    att = ht.attention_op(q, k, v, dropout=0.1)
    loss = ht.reduce_mean_op(ht.mul_op(att, att), [0, 1, 2, 3])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=1, mixed_precision='bf16', use_hipgraph=False)
    ls = [float(np.asarray(ex.run('train', feed_dict={x: X}, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
          for _ in range(3)]
    assert np.isfinite(ls).all()
    assert calls == {'fwd': 3, 'bwd': 3}, calls
