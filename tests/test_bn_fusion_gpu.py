"""BatchNorm reductions fused into convolution epilogues (graph_opt.fuse_forward /
_fuse_bn_backward_reduction; gemm_core.h Epi::colstats / Epi::bnx, conv3x3.hip BnB).

Forward: the conv epilogue accumulates the per-channel sum / sum of squares of its
output.  Backward: the data-gradient epilogue that produces a BN output's gradient dy
accumulates sum(dy') and sum(dy' * x) (dy' = dy masked by the forward's ReLU
keep-bits, x the BN input), and the BN backward skips its own pass over dy and x.
Reference semantics: src/ops/CudnnBn.cu:22-194 (cudnnBatchNormalizationBackward).
Each kernel is checked against a plain fp32 torch reduction of the same stored values.
"""
import os

import numpy as np
import pytest
import torch

from hetu_61a7_amd.kernels import conv as KC, conv_igemm as CI, norm as KN

pytestmark = pytest.mark.gpu
DEV = 'cuda'
CL = torch.channels_last


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _bits(mask, shape_nhwc):
    """per-element keep bits (0/1 float) of a byte-per-8-channels mask"""
    sh = torch.arange(8, device=mask.device, dtype=torch.int32)
    return ((mask.to(torch.int32).view(-1, 1) >> sh) & 1).float().view(shape_nhwc)


def _ref_sums(dx, x, mask):
    d = dx.permute(0, 2, 3, 1).float()
    if mask is not None:
        d = d * _bits(mask, d.shape)
    xv = x.permute(0, 2, 3, 1).float()
    return d.sum((0, 1, 2)), (d * xv).sum((0, 1, 2))


# (g shape [N, K, OH, OW], w shape [K, C, kh, kw], x shape, stride, pad, kernel)
CASES = [
    ((4, 256, 14, 14), (256, 64, 1, 1), (4, 64, 14, 14), 1, 0, ('gemm', 0)),
    ((4, 256, 14, 14), (256, 64, 1, 1), (4, 64, 14, 14), 1, 0, ('gemm', 2)),
    ((4, 256, 14, 14), (256, 64, 1, 1), (4, 64, 14, 14), 1, 0, ('gemm', 3)),
    ((4, 64, 14, 14), (64, 256, 1, 1), (4, 256, 14, 14), 1, 0, ('gemm', 1)),
    ((4, 128, 14, 14), (128, 64, 3, 3), (4, 64, 28, 28), 2, 1, ('gemm', 0)),      # stride classes
    ((2, 64, 56, 56), (64, 64, 3, 3), (2, 64, 56, 56), 1, 1, ('c3', None)),       # c64 halo kernel
    ((2, 128, 28, 28), (128, 128, 3, 3), (2, 128, 28, 28), 1, 1, ('c3', None)),   # wide halo kernel
    ((2, 256, 7, 7), (256, 256, 3, 3), (2, 256, 7, 7), 1, 1, ('c3', None)),
]


@pytest.mark.parametrize('case', CASES, ids=lambda c: '%s-%s-%s' % (c[1], c[5][0], c[5][1]))
@pytest.mark.parametrize('masked', [True, False])
@pytest.mark.parametrize('join', [False, True])
@pytest.mark.parametrize('reps', [1, 3])
def test_dgrad_epilogue_bn_sums(case, masked, join, reps):
    """the BN-backward reduction in the data-gradient epilogue against the fp32 reference
    sums of the stored gradient; reps > 1: the totals spread over that many replicas
    (Epi::cs_rep), whose sum is the total"""
    gs, ws, xs, s, p, (kind, tile) = case
    torch.manual_seed(0)
    g = torch.randn(gs, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(ws, device=DEV) * 0.05).bfloat16().contiguous(memory_format=CL)
    xb = (torch.randn(xs, device=DEV) + 0.5).bfloat16().contiguous(memory_format=CL)
    acc = torch.randn(xs, device=DEV).bfloat16().contiguous(memory_format=CL) if join else None
    n = xb.numel() // 8
    mask = torch.randint(0, 256, (n,), device=DEV, dtype=torch.int32).to(torch.uint8) if masked else None
    sums = torch.zeros(reps * 2 * xs[1], device=DEV)
    if kind == 'gemm':
        dx = CI.try_backward_data(g, w, xs, (s, s), (p, p), acc=acc, tile=tile, bnb=(sums, xb, mask))
        dx0 = CI.try_backward_data(g, w, xs, (s, s), (p, p), acc=acc, tile=tile)
    else:
        dx = CI.try_conv3x3_backward_data(g, w, xs, (s, s), (p, p), acc=acc, bnb=(sums, xb, mask))
        dx0 = CI.try_conv3x3_backward_data(g, w, xs, (s, s), (p, p), acc=acc)
    assert dx is not None
    assert torch.equal(dx, dx0)     # the statistics do not perturb the stored gradient
    rs, rq = _ref_sums(dx, xb, mask)
    C = xs[1]
    if reps > 1 and xs[2] > 7:   # (2 images of 7x7 are one pixel tile of the wide kernel)
        assert torch.count_nonzero(sums[2 * C:]).item() > 0   # the replicas were used
    sums = sums.view(reps, 2 * C).sum(0)
    assert _rel(sums[:C], rs) < 1e-4, (_rel(sums[:C], rs))
    assert _rel(sums[C:], rq) < 1e-4, (_rel(sums[C:], rq))
    if masked:   # masked store: dx' = dx * keep-bits, same statistics
        s2 = torch.zeros(reps * 2 * C, device=DEV)
        if kind == 'gemm':
            dm = CI.try_backward_data(g, w, xs, (s, s), (p, p), acc=acc, tile=tile, bnb=(s2, xb, mask, True))
        else:
            dm = CI.try_conv3x3_backward_data(g, w, xs, (s, s), (p, p), acc=acc, bnb=(s2, xb, mask, True))
        bits = _bits(mask, dx.permute(0, 2, 3, 1).shape)
        assert torch.equal(dm.permute(0, 2, 3, 1).float(), dx.permute(0, 2, 3, 1).float() * bits)
        assert _rel(s2.view(reps, 2 * C).sum(0), sums) < 1e-5


@pytest.mark.parametrize('tile', [0, 1, 2, 3])
@pytest.mark.parametrize('with_bn', [False, True])
def test_dgrad_subgrid_join(tile, with_bn):
    """1x1 stride-1 data gradient + the compact gradient of a 1x1 stride-2 conv of the same
    input added at the even positions (the ResNet downsample join): against the scattered
    reference, with and without the BN-backward reduction + masked store."""
    torch.manual_seed(3)
    N, H, K, C = 2, 14, 256, 128 if tile != 2 else 64
    g = torch.randn(N, K, H, H, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, 1, 1, device=DEV) * 0.05).bfloat16().contiguous(memory_format=CL)
    acc = torch.randn(N, C, H // 2, H // 2, device=DEV).bfloat16().contiguous(memory_format=CL)
    xs = (N, C, H, H)
    full = torch.zeros(xs, device=DEV).bfloat16().contiguous(memory_format=CL)
    full[:, :, ::2, ::2] = acc
    ref = CI.try_backward_data(g, w, xs, (1, 1), (0, 0), acc=full, tile=tile)
    bnb = None
    if with_bn:
        xb = torch.randn(xs, device=DEV).bfloat16().contiguous(memory_format=CL)
        mask = torch.randint(0, 256, (xb.numel() // 8,), device=DEV, dtype=torch.int32).to(torch.uint8)
        sums = torch.zeros(2 * C, device=DEV)
        bnb = (sums, xb, mask, True)
    dx = CI.try_backward_data(g, w, xs, (1, 1), (0, 0), acc=acc, tile=tile, bnb=bnb, acc_s2=True)
    assert dx is not None
    if not with_bn:
        assert torch.equal(dx, ref)
        return
    bits = _bits(mask, ref.permute(0, 2, 3, 1).shape)
    assert torch.equal(dx.permute(0, 2, 3, 1).float(), ref.permute(0, 2, 3, 1).float() * bits)
    rs, rq = _ref_sums(ref, xb, mask)
    assert _rel(sums[:C], rs) < 1e-4 and _rel(sums[C:], rq) < 1e-4


def test_bn_bwd_sums_pass_matches_reference():
    x = (torch.randn(4, 128, 14, 14, device=DEV) + 1).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(4, 128, 14, 14, device=DEV).bfloat16().contiguous(memory_format=CL)
    mask = torch.randint(0, 256, (x.numel() // 8,), device=DEV, dtype=torch.int32).to(torch.uint8)
    sums = torch.zeros(256, device=DEV)
    KN.bn_bwd_sums(dy, x, mask, sums)
    rs, rq = _ref_sums(dy, x, mask)
    assert _rel(sums[:128], rs) < 1e-4 and _rel(sums[128:], rq) < 1e-4


@pytest.mark.parametrize('relu,residual', [(True, False), (True, True), (False, False)])
def test_bn_backward_from_epilogue_sums_matches_plain(relu, residual):
    """bn_backward with the totals handed in (bsums) against the full backward; the
    totals are zeroed once read (persistent per-layer buffers)."""
    torch.manual_seed(1)
    C = 128
    x = (torch.randn(4, C, 14, 14, device=DEV) * 2 + 0.7).bfloat16().contiguous(memory_format=CL)
    res = torch.randn_like(x).contiguous(memory_format=CL) if residual else None
    sc, bi = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.2
    mask = torch.empty(KN.relu_mask_bytes(x), dtype=torch.uint8, device=DEV) if relu else None
    y, mean, invstd = KN.bn_forward(x, sc, bi, None, None, 0.1, 1e-5, True, relu=relu, residual=res, mask=mask)
    dy = torch.randn_like(x).contiguous(memory_format=CL)
    ref = KN.bn_backward(dy, y, x, sc, mean, invstd, relu=relu, want_dres=residual, bias=bi, mask=mask)
    bs = torch.zeros(2 * C, device=DEV)
    KN.bn_bwd_sums(dy, x, mask, bs)
    out = KN.bn_backward(dy, y, x, sc, mean, invstd, relu=relu, want_dres=residual, bias=bi, mask=mask, bsums=bs)
    assert torch.count_nonzero(bs).item() == 0
    for a, b in zip(out, ref):
        if b is None:
            assert a is None
            continue
        assert _rel(a, b) < 2e-3, _rel(a, b)
    # replicated totals ([R][2C], the first holding the sums, the others partial zeros and
    # garbage that cancels): folded by the finalize kernel, all zeroed
    bs = torch.zeros(3 * 2 * C, device=DEV)
    KN.bn_bwd_sums(dy, x, mask, bs)
    d = torch.randn(2 * C, device=DEV)
    bs[2 * C:4 * C] += d
    bs[4 * C:] -= d
    out = KN.bn_backward(dy, y, x, sc, mean, invstd, relu=relu, want_dres=residual, bias=bi, mask=mask, bsums=bs)
    assert torch.count_nonzero(bs).item() == 0
    for a, b in zip(out, ref):
        if b is None:
            assert a is None
            continue
        assert _rel(a, b) < 2e-3, _rel(a, b)
    # double-buffered totals: coefficients folded in the apply kernel, the other half cleared
    bs = torch.zeros(2 * C, device=DEV)
    other = torch.randn(2 * C, device=DEV)
    KN.bn_bwd_sums(dy, x, mask, bs)
    out = KN.bn_backward(dy, y, x, sc, mean, invstd, relu=relu, want_dres=residual, bias=bi, mask=mask, bsums=bs,
                         bsums_next=other)
    assert torch.count_nonzero(other).item() == 0
    for a, b in zip(out, ref):
        if b is None:
            assert a is None
            continue
        assert _rel(a, b) < 2e-3, _rel(a, b)


def test_persistent_forward_sums_are_rezeroed():
    x = torch.randn(4, 64, 28, 28, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(128, 64, 3, 3, device=DEV) * 0.1).bfloat16().contiguous(memory_format=CL)
    buf = torch.zeros(256, device=DEV)
    sc, bi = torch.rand(128, device=DEV) + 0.5, torch.randn(128, device=DEV)
    ref = None
    for _ in range(3):   # the first call autotunes against scratch, later ones use buf
        y, sums = KC.conv2d_with_stats(x, w, (1, 1), (1, 1), out_sums=buf)
        a, m, i = KN.bn_forward(y, sc, bi, None, None, 0.1, 1e-5, True, relu=True, sums=sums)
        assert torch.count_nonzero(buf).item() == 0
        if ref is None:
            ref = (m.clone(), i.clone())
        assert _rel(m, ref[0]) < 1e-5 and _rel(i, ref[1]) < 1e-5
    a2, m2, i2 = KN.bn_forward(y, sc, bi, None, None, 0.1, 1e-5, True, relu=True)
    assert _rel(m2, ref[0]) < 1e-4 and _rel(i2, ref[1]) < 1e-4


def _resnet_step(fuse_bwd, fuse_stats):
    """first loss and the parameter update of one plain SGD step of ResNet-50 (batch 4)"""
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models import resnet50_imagenet
    from hetu_61a7_amd.ops import node as _node
    _node.G_NODE_ID = 0      # same node ids -> same names and initial weights in both graphs
    os.environ['HETU_FUSE_BN_BWD'] = fuse_bwd if isinstance(fuse_bwd, str) else ('1' if fuse_bwd else '0')
    os.environ['HETU_FUSE_BN_STATS'] = '1' if fuse_stats else '0'
    try:
        B = 4
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        loss, _ = resnet50_imagenet(x, y_, 1000)
        train = ht.optim.SGDOptimizer(learning_rate=1.0).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=3)
        g = torch.Generator(device='cuda')
        g.manual_seed(0)
        X = torch.randn((B, 3, 224, 224), device='cuda', generator=g).bfloat16().contiguous(memory_format=CL)
        Y = torch.nn.functional.one_hot(torch.randint(0, 1000, (B,), device='cuda', generator=g), 1000).bfloat16()
        before = {k: v.detach().float().clone() for k, v in ex.return_tensor_values().items()
                  if isinstance(v, torch.Tensor) and v.is_floating_point()}
        lv = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]
        after = ex.return_tensor_values()
        delta = {k: after[k].detach().float() - v for k, v in before.items() if k in after}
        fused = sum(1 for n in ex.subexecutor['train'].computing_nodes if getattr(n, 'bn_fused', None) is not None)
        return float(np.mean(lv)), delta, fused
    finally:
        os.environ.pop('HETU_FUSE_BN_BWD', None)
        os.environ.pop('HETU_FUSE_BN_STATS', None)


@pytest.mark.parametrize('mode,min_fused', [('1', 15), ('all', 40)])
def test_resnet50_gradients_with_fused_bn_backward_match_unfused(mode, min_fused):
    """One SGD step of ResNet-50 with the BN-backward reductions in the dgrad epilogues
    (and the masked gradient store) updates every parameter as the unfused graph does,
    to bf16 accuracy; the forward is untouched.  mode '1': the joined data gradients only
    (one per bottleneck past the first, whose input is the max-pool output), 'all': every
    eligible one."""
    l0, d0, _ = _resnet_step(False, False)
    l1, d1, nf = _resnet_step(mode, False)
    assert nf >= min_fused, nf
    assert l0 == l1
    num = sum(float((d1[k] - d0[k]).norm()) ** 2 for k in d0)
    den = sum(float(d0[k].norm()) ** 2 for k in d0)
    assert (num / den) ** 0.5 < 0.03, (num / den) ** 0.5
    worst = max((float((d1[k] - d0[k]).norm() / d0[k].norm().clamp_min(1e-12)), k) for k in d0
                if float(d0[k].norm()) > 0)
    assert worst[0] < 0.15, worst     # the stem BN bias (a cancelling sum) sits at ~0.08 from bf16 alone


def test_resnet50_forward_with_fused_bn_statistics():
    """Loss of a random-init ResNet-50 with the forward BN statistics from the conv
    epilogues: the per-shape kernel choice may differ between the two graphs ('fwd' vs
    'fwd_stats' autotune keys), and bf16 rounding differences grow over 50 layers, so
    this is a coarse check; the statistics themselves are checked exactly per kernel
    (test_gemm_gpu.py::test_conv_fused_bn_statistics, test_persistent_forward_sums_are_rezeroed)."""
    l0, _, _ = _resnet_step(False, False)
    l1, _, _ = _resnet_step(False, True)
    assert abs(l0 - l1) <= 2e-2 * max(1.0, abs(l0)), (l0, l1)


def _resnet_grads(use_hipgraph, steps=6):
    """losses and the flat fp32 gradient of every step of ResNet-50 (batch 4, fused BN
    backward for every eligible layer) at learning rate 0: the weights never move, so every
    step computes the same gradient -- up to the atomic-order noise of the fused BN totals.
    (Comparing trajectories instead is hopeless: batch-4 BatchNorm is chaotic, a 2 % change
    in one step's update decorrelates the next step's gradient, profiles/bn_update_repro_r5.txt.)
    The forward statistics take the deterministic two-pass kernel."""
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models import resnet50_imagenet
    from hetu_61a7_amd.ops import node as _node
    _node.G_NODE_ID = 0
    saved = {k: os.environ.get(k) for k in ('HETU_FUSE_BN_BWD', 'HETU_FUSE_BN_STATS')}
    os.environ['HETU_FUSE_BN_BWD'] = 'all'
    os.environ['HETU_FUSE_BN_STATS'] = '0'
    try:
        B = 4
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        loss, _ = resnet50_imagenet(x, y_, 1000)
        train = ht.optim.SGDOptimizer(learning_rate=0.0).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=3,
                         use_hipgraph=use_hipgraph)
        g = torch.Generator(device='cuda')
        g.manual_seed(0)
        X = torch.randn((B, 3, 224, 224), device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
        Y = torch.nn.functional.one_hot(torch.randint(0, 1000, (B,), device='cuda', generator=g), 1000).bfloat16()
        out, grads = [], []
        for _ in range(steps):
            lv = ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0]
            out.append(float(np.mean(lv)))
            op = ex.subexecutor['train'].opt_ops[0]
            grads.append(op.flat.grad[:op.flat.numel].float().clone())
        fused = sum(1 for n in ex.subexecutor['train'].computing_nodes if getattr(n, 'bn_fused', None) is not None)
        return out, grads, fused
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_hipgraph_replays_fused_bn_backward_like_eager():
    """the fused BN-backward totals were double-buffered by a Python
    flip; a captured step froze the flip, so every replay added into the same half and
    zeroed the other.  Small spatial sizes (every layer below 16384 rows: one replica)
    take that path.  With hipGraph replay (3 eager warm-up steps, then capture + 3
    replays) every step's gradient must match the eager run's (a frozen flip doubles and
    triples the BN totals replay after replay)."""
    eager, ge, nf = _resnet_grads(False)
    graph, gg, _ = _resnet_grads(True)
    assert nf >= 20, nf
    np.testing.assert_allclose(graph, eager, rtol=1e-3, atol=1e-3)
    for k, (a, b) in enumerate(zip(gg, ge)):
        rel = float((a - b).norm() / b.norm().clamp_min(1e-20))
        assert rel < 0.05, (k, rel)
