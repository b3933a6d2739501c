"""MoE HIP kernels (moe.hip) vs the CPU/torch reference; fused-gate MoE layer
on the GPU vs the op-by-op gate."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht
from hetu_61a7_amd.kernels import moe as KM
from test_moe_cpu import dispatch_combine_check, moe_fused_vs_graph

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('dt,tol', [(torch.float32, 1e-5), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize('shape', [(10, 6, 3, 2, 5), (64, 256, 8, 2, 12), (33, 130, 4, 1, 9)])
def test_dispatch_combine(dt, tol, shape):
    T, d, E, k, cap = shape
    dispatch_combine_check('cuda', dt, T=T, d=d, E=E, k=k, cap=cap, seed=T, tol=tol)


@pytest.mark.parametrize('E,k', [(4, 1), (16, 2), (100, 3), (512, 8)])
def test_gate_topk_and_locations(E, k):
    rng = np.random.RandomState(E)
    T = 300
    x = torch.tensor(rng.randn(T, E).astype(np.float32))
    v, i, p = KM.topk(x.cuda(), k, softmax=True)
    rv, ri, rp = KM.topk(x, k, softmax=True)
    np.testing.assert_allclose(p.cpu().numpy(), rp.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v.cpu().numpy(), rv.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(i.cpu().numpy(), ri.numpy())
    loc, cnt, ps = KM.locations(i, E, p)
    rloc, rcnt, rps = KM.locations(ri, E, rp)
    np.testing.assert_array_equal(loc.cpu().numpy(), rloc.numpy())
    np.testing.assert_array_equal(cnt.cpu().numpy(), rcnt.numpy())
    np.testing.assert_allclose(ps.cpu().numpy(), rps.numpy(), rtol=1e-4, atol=1e-5)
    dg = torch.tensor(rng.randn(T, k).astype(np.float32))
    coef = torch.tensor(rng.rand(E).astype(np.float32))
    got = KM.gate_backward(p, i, dg.cuda(), coef.cuda())
    ref = KM.gate_backward(rp, ri, dg, coef)
    np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('T,E,k,inactive', [(65536, 2, 2, 0.0), (10000, 16, 2, 0.0), (5000, 8, 4, 0.3),
                                             (700, 3, 3, 0.0)])
@pytest.mark.parametrize('segmented', ['1', '0'])
def test_locations_many_segments_match_cpu(T, E, k, inactive, segmented, monkeypatch):
    """The segmented two-pass locations scan (E x S blocks) against the CPU reference:
    slot positions in choice-major order, per-expert counts and gate-probability sums;
    choices with expert -1 (the dense-to-sparse gate's inactive ones) get no slot."""
    monkeypatch.setenv('HETU_MOE_LOC_SEGMENTED', segmented)
    rng = np.random.RandomState(T + E)
    idx = rng.randint(0, E, size=(T, k)).astype(np.int64)
    if inactive:
        idx[rng.rand(T, k) < inactive] = -1
    probs = rng.rand(T, E).astype(np.float32)
    i, p = torch.tensor(idx), torch.tensor(probs)
    loc, cnt, ps = KM.locations(i.cuda(), E, p.cuda())
    rloc, rcnt, rps = KM.locations(i, E, p)
    keep = idx >= 0
    np.testing.assert_array_equal(loc.cpu().numpy()[keep], rloc.numpy()[keep])
    np.testing.assert_array_equal(cnt.cpu().numpy(), rcnt.numpy())
    np.testing.assert_allclose(ps.cpu().numpy(), rps.numpy(), rtol=1e-4, atol=1e-3)


def test_fused_gate_layer_gpu_matches_graph_gate():
    a, b = moe_fused_vs_graph(ht.gpu(0))
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    c, _ = moe_fused_vs_graph(ht.cpu(0))
    np.testing.assert_allclose(a, c, rtol=1e-3, atol=1e-4)


def test_cumsum_long_column_scan_matches_cpu():
    import hetu_61a7_amd as ht
    x = ht.Variable(name='x')
    y = ht.cumsum_with_bias_op(x, bias=-1, dim=0)
    X = (np.random.RandomState(0).rand(16384, 2) > 0.5).astype(np.float32)
    got = ht.Executor([y], ctx=ht.gpu(0)).run(feed_dict={x: X}, convert_to_numpy_ret_vals=True)[0]
    np.testing.assert_array_equal(got, np.cumsum(X, 0) - 1)


def test_matmul_out_row_blocks_match_fp32():
    """kernels.gemm.matmul_out writes each product into its row block of one bf16 buffer
    (the MoE experts' concatenated output) -- against fp32 math, blocks untouched outside"""
    from hetu_61a7_amd.kernels import gemm as KG
    g = torch.Generator(device='cuda').manual_seed(0)
    xs = [torch.randn(m, 256, device='cuda', generator=g).bfloat16() for m in (512, 384, 640)]
    ws = [(torch.randn(256, 384, device='cuda', generator=g) * 0.05).bfloat16() for _ in xs]
    out = torch.full((sum(x.shape[0] for x in xs), 384), 7.0, device='cuda').bfloat16()
    r = 0
    for x, w in zip(xs, ws):
        KG.matmul_out(x, w, out[r:r + x.shape[0]])
        r += x.shape[0]
    ref = torch.cat([x.float() @ w.float() for x, w in zip(xs, ws)], 0)
    assert float((out.float() - ref).norm() / ref.norm()) < 1e-2


def test_moe_row_concat_experts_match_concat_path(monkeypatch):
    """the MoE bench layer with the local experts' second GEMMs as row blocks of one output
    trains like the concatenation path (same losses, bf16 noise)"""
    import hetu_61a7_amd.layers.moe as LM
    from hetu_61a7_amd.ops import node as _node
    losses, init = {}, None
    for rc in (True, False):
        monkeypatch.setattr(LM, '_ROW_CONCAT', rc)
        _node.G_NODE_ID = 0
        rng = np.random.RandomState(0)
        T, d, E = 512, 128, 4
        x = ht.Variable(name='x')
        gate = LM.TopKGate(embed_dim=d, num_tokens=T, num_experts=E, k=2)
        experts = [LM.Expert(d, 256, activation='relu', name='expert_%d' % i) for i in range(E)]
        y, l_aux = LM.MoELayer(gate=gate, experts=experts, num_tokens=T, embed_dim=d)(x)
        loss = ht.add_op(ht.reduce_mean_op(ht.mul_op(y, y), [0, 1]), l_aux)
        train = ht.optim.SGDOptimizer(0.1).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, mixed_precision='bf16')
        pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
        if init is None:
            init = {k: v.detach().clone() for k, v in pm.items()}
        else:
            for k, v in pm.items():
                v.copy_(init[k])
        X = rng.randn(T, d).astype(np.float32)
        losses[rc] = [float(np.asarray(ex.run('train', feed_dict={x: X}, convert_to_numpy_ret_vals=True)[0])
                            .reshape(-1)[0]) for _ in range(4)]
    np.testing.assert_allclose(losses[True], losses[False], rtol=2e-2)


@pytest.mark.parametrize('dt,tol', [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize('T,d,E,k,cap', [(64, 256, 8, 2, 12), (300, 2048, 4, 2, 100), (33, 130, 4, 1, 9)])
def test_fused_combine_backward_matches_separate_kernels(dt, tol, T, d, E, k, cap):
    """Both gradients of the gate-weighted combine from one kernel (the token gradient read
    once) equal the slot-gather and gate-gradient kernels and the CPU reference, with
    pairs dropped at capacity (gate gradient 0) and empty slots (zero rows)"""
    rng = np.random.RandomState(T + d)
    idx = torch.tensor(rng.randint(0, E, size=(T, k)).astype(np.int64))
    probs = torch.tensor(rng.rand(T, E).astype(np.float32))
    loc, _, _ = KM.locations(idx, E, probs)
    gates = torch.tensor(rng.rand(T, k).astype(np.float32))
    g = torch.tensor(rng.randn(T, d).astype(np.float32)).to(dt)
    y = torch.tensor(rng.randn(E * cap, d).astype(np.float32)).to(dt)
    assert bool((loc >= cap).any()), 'the case should drop some pairs'
    dc, gc = KM.reverse_layout_transform_backward_fused(g, y, idx, loc, gates, cap, E * cap)   # CPU reference
    i, l, w = idx.cuda(), loc.cuda(), gates.cuda()
    d1, g1 = KM.reverse_layout_transform_backward_fused(g.cuda(), y.cuda(), i, l, w, cap, E * cap)
    d0 = KM.reverse_layout_transform_backward_data(g.cuda(), i, l, w, cap, E * cap)
    g0 = KM.reverse_layout_transform_backward_gate(g.cuda(), y.cuda(), i, l, cap)
    assert d1.dtype == dt and g1.dtype == torch.float32 and tuple(g1.shape) == (T, k)
    assert bool((d1 == d0).all())
    np.testing.assert_allclose(g1.cpu().numpy(), g0.cpu().numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(d1.float().cpu().numpy(), dc.float().numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(g1.cpu().numpy(), gc.float().numpy(), rtol=tol, atol=tol * d ** 0.5)
    assert bool((g1.cpu()[loc >= cap] == 0).all())


def test_moe_keep_bit_mask_trains_like_bf16_mask(monkeypatch):
    """experts with dropout: the backward mask GEMM reading the forward's 1-bit keep masks
    (HETU_GMASK_BITS) trains exactly like reading the bf16 forward output"""
    import hetu_61a7_amd.layers.moe as LM
    import hetu_61a7_amd.ops.linalg as OL
    from hetu_61a7_amd.ops import node as _node
    losses, init = {}, None
    for bits in (True, False):
        monkeypatch.setattr(OL, '_GMASK_BITS', bits)
        _node.G_NODE_ID = 0
        rng = np.random.RandomState(0)
        T, d, E = 512, 128, 4
        x = ht.Variable(name='x')
        gate = LM.TopKGate(embed_dim=d, num_tokens=T, num_experts=E, k=2)
        experts = [LM.Expert(d, 256, activation='relu', dropout_rate=0.1, name='expert_%d' % i) for i in range(E)]
        y, l_aux = LM.MoELayer(gate=gate, experts=experts, num_tokens=T, embed_dim=d)(x)
        loss = ht.add_op(ht.reduce_mean_op(ht.mul_op(y, y), [0, 1]), l_aux)
        train = ht.optim.SGDOptimizer(0.1).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=3, mixed_precision='bf16')
        pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
        if init is None:
            init = {k: v.detach().clone() for k, v in pm.items()}
        else:
            for k, v in pm.items():
                v.copy_(init[k])
        X = rng.randn(T, d).astype(np.float32)
        losses[bits] = [float(np.asarray(ex.run('train', feed_dict={x: X}, convert_to_numpy_ret_vals=True)[0])
                              .reshape(-1)[0]) for _ in range(4)]
    assert len(set(losses[True])) > 1
    np.testing.assert_allclose(losses[True], losses[False], rtol=1e-5)
