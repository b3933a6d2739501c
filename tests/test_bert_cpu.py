"""Fused attention op vs torch autograd, and a tiny BERT pretraining run on CPU."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht


@pytest.mark.parametrize('causal', [False, True])
def test_attention_op_matches_torch(causal):
    rng = np.random.RandomState(0)
    B, H, S, D = 2, 3, 8, 4
    qv, kv, vv = [rng.randn(B, H, S, D).astype(np.float32) for _ in range(3)]
    mv = np.zeros((B, 1, 1, S), np.float32)
    mv[1, ..., -2:] = -10000.0
    q, k, v, m = [ht.Variable(name=n) for n in 'qkvm']
    o = ht.attention_op(q, k, v, m, dropout=0.0, causal=causal)
    loss = ht.reduce_sum_op(ht.mul_op(o, o), [0, 1, 2, 3])
    gq, gk, gv = ht.gradients(loss, [q, k, v])
    ex = ht.Executor([loss, gq, gk, gv], ctx=ht.cpu(0))
    res = ex.run(feed_dict={q: qv, k: kv, v: vv, m: mv}, convert_to_numpy_ret_vals=True)
    tq, tk, tv = [torch.tensor(a, requires_grad=True) for a in (qv, kv, vv)]
    s = tq @ tk.transpose(-1, -2) / np.sqrt(D) + torch.tensor(mv)
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float('-inf'))
    to = torch.softmax(s, -1) @ tv
    tl = (to * to).sum()
    tl.backward()
    np.testing.assert_allclose(res[0], tl.item(), rtol=1e-4)
    for got, ref in zip(res[1:], (tq.grad, tk.grad, tv.grad)):
        np.testing.assert_allclose(got, ref.numpy(), rtol=1e-3, atol=1e-4)


def test_tiny_bert_pretraining_learns():
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    cfg = BertConfig(vocab_size=1200, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=64, batch_size=4, seq_len=16, max_position_embeddings=16,
                     hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    feeds, loss, train = bert_pretrain_graph(cfg, lr=3e-3)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    batch = synthetic_bert_batch(cfg, seed=1)
    fd = {feeds[k]: v for k, v in batch.items()}
    losses = [float(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]) for _ in range(15)]
    assert np.isfinite(losses).all()
    assert losses[-1] < losses[0] * 0.8, losses


def packed_attention_check(device, dtype, B=2, S=32, NH=2, D=64, keep=1.0, tol=1e-4, seed=9):
    """Packed-QKV attention fwd/bwd vs torch autograd (fp32 reference)."""
    from hetu_61a7_amd.kernels import attention as KA
    rng = np.random.RandomState(B * S + NH)
    H = NH * D
    qkv = torch.tensor(rng.randn(B * S, 3 * H).astype(np.float32) * 0.5)
    mask = torch.zeros(B, S)
    mask[-1, -5:] = -10000.0
    dout = torch.tensor(rng.randn(B * S, H).astype(np.float32))
    out, saved = KA.attention_fwd(qkv.to(device, dtype), mask.to(device), B, S, NH, keep, seed)
    # reference with the kernel's own dropout mask (flat P index -> Philox/generator bits)
    t = qkv.clone().requires_grad_(True)
    x = t.reshape(B, S, 3, NH, D)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    p = torch.softmax(q @ k.transpose(-1, -2) / np.sqrt(D) + mask.reshape(B, 1, 1, S), -1)
    if keep < 1.0:
        from hetu_61a7_amd.kernels import dropout as KD
        if device == 'cpu':
            dm = KA._ref_dropmask(p.shape, keep, seed, 'cpu')
        else:   # kernel uses the standalone Philox dropout's counters over the flat P tensor
            dm = KD.dropout(torch.ones(p.shape, device=device), keep, seed).float().cpu()
        p = p * dm
    o = (p @ v).transpose(1, 2).reshape(B * S, H)
    o.backward(dout)
    np.testing.assert_allclose(out.float().cpu().numpy(), o.detach().numpy(), rtol=tol, atol=tol)
    dqkv = KA.attention_bwd(dout.to(device, dtype), qkv.to(device, dtype), out, saved, mask.to(device), B, S, NH,
                            keep, seed)
    np.testing.assert_allclose(dqkv.float().cpu().numpy(), t.grad.numpy(), rtol=10 * tol, atol=10 * tol)
    # and per operand in relative norm (a wrong-scale dQ / dK / dV would still fit the
    # elementwise band above): <= 3e-2 in bf16, the fp32 tolerance otherwise
    rel_tol = 3e-2 if dtype == torch.bfloat16 else 10 * tol
    g = dqkv.float().cpu().reshape(B * S, 3, H)
    ref = t.grad.reshape(B * S, 3, H)
    for i, name in enumerate('qkv'):
        rel = float((g[:, i] - ref[:, i]).norm() / ref[:, i].norm().clamp_min(1e-12))
        assert rel <= rel_tol, ('d' + name, rel)
    rel = float((out.float().cpu() - o.detach()).norm() / o.detach().norm())
    assert rel <= rel_tol, ('out', rel)


def test_packed_attention_reference_cpu():
    packed_attention_check('cpu', torch.float32)
    packed_attention_check('cpu', torch.float32, B=1, S=8, NH=3, D=4, keep=0.7)


def test_bert_fused_vs_unfused_attention_graph():
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    out, init = [], None
    for fused in (False, True):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=1200, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                         intermediate_size=64, batch_size=4, seq_len=16, max_position_embeddings=16,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, fused_attention=fused)
        feeds, loss, train = bert_pretrain_graph(cfg, lr=3e-3)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=2)
        pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
        if init is None:
            init = {k: v.detach().clone() for k, v in pm.items()}
        else:
            for k, v in pm.items():
                v.copy_(init[k])
        fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
        out.append([float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
                    for _ in range(4)])
    np.testing.assert_allclose(out[0], out[1], rtol=1e-4, atol=1e-5)


def test_padded_vocab_matches_unpadded():
    """vocab 1200 padded to 1216 rows (vocab_multiple 64): the -1e4 decoder bias on the pad
    columns gives them softmax weight 0, so losses and the real rows' updates equal the
    unpadded model's (counter-based init: the first 1200 rows start identical)."""
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    from hetu_61a7_amd import optim
    out = []
    for mult in (1, 64):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=1200, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                         intermediate_size=64, batch_size=4, seq_len=16, max_position_embeddings=16,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, vocab_multiple=mult)
        assert cfg.padded_vocab_size == (1200 if mult == 1 else 1216)
        feeds, loss, train = bert_pretrain_graph(cfg, lr=0.1, optimizer=optim.SGDOptimizer(learning_rate=0.1))
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=5)
        batch = synthetic_bert_batch(cfg, seed=3)
        fd = {feeds[k]: v for k, v in batch.items()}
        losses = [float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
                  for _ in range(3)]
        emb = [v for n, v in ex.config.placeholder_to_arr_map.items() if n.name == 'word_embeddings'][0]
        out.append((losses, emb.detach().numpy().copy()))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-5)
    np.testing.assert_allclose(out[1][1][:1200], out[0][1], rtol=1e-5, atol=1e-7)
