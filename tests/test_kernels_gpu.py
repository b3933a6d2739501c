"""HIP kernel numerics vs plain PyTorch fp32 references (run on MI355X)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from hetu_61a7_amd import _base
from hetu_61a7_amd.kernels import elementwise as KE, norm as KN, softmax as KS, optim as KO
from hetu_61a7_amd.kernels import pool as KP, reduce as KR, sparse as KSP, layernorm as KLN, dropout as KD

DEV = 'cuda'


def test_native_library_loaded():
    assert _base.has_kernels(), 'libhetu_kernels.so must load on the GPU box'


def _tol(dt):
    return dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('op', ['relu', 'sigmoid', 'tanh', 'exp', 'gelu', 'abs', 'neg', 'sqrt', 'add_c', 'mul_c'])
def test_unary(op, dt):
    x = torch.randn(1000003, device=DEV).to(dt)
    if op == 'sqrt':
        x = x.abs() + 0.1
    y = KE.unary(op, x, 0.5)
    ref = KE._ref_unary(op, x.float(), 0.5, 0.0)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('op', ['add', 'sub', 'mul', 'relu_grad', 'gelu_grad', 'tanh_grad'])
def test_binary_modes(op, dt):
    a = torch.randn(512, 768, device=DEV).to(dt)
    b = torch.randn(512, 768, device=DEV).to(dt)
    row = torch.randn(768, device=DEV)
    torch.testing.assert_close(KE.binary(op, a, b).float(), KE._ref_binary(op, a.float(), b.float(), 0.0), **_tol(dt))
    if op in ('add', 'mul', 'sub'):
        torch.testing.assert_close(KE.binary(op, a, row).float(),
                                   KE._ref_binary(op, a.float(), row.to(dt).float(), 0.0), **_tol(dt))


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('relu,res', [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize('N,C,H,W', [(8, 64, 14, 14), (2, 512, 28, 28), (2, 1024, 14, 14), (2, 2048, 7, 7)])
def test_batchnorm_nhwc(dt, relu, res, N, C, H, W):
    # C >= 512 in bf16 puts 512 channels in one stats tile (more than the 256
    # threads that fold it): the ResNet-50 stage 2-4 shapes
    torch.manual_seed(1000 + N + C + H)
    x = torch.randn(N, C, H, W, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    r = torch.randn(N, C, H, W, device=DEV).to(dt).contiguous(memory_format=torch.channels_last) if res else None
    scale = torch.rand(C, device=DEV) + 0.5
    bias = torch.randn(C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y, mean, invstd = KN.bn_forward(x, scale, bias, rm, rv, 0.1, 1e-5, True, relu=relu, residual=r)
    xf = x.float().requires_grad_(True)
    sf = scale.clone().requires_grad_(True)
    bf = bias.clone().requires_grad_(True)
    rf = r.float().requires_grad_(True) if res else None
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    ref = F.batch_norm(xf, rm2, rv2, sf, bf, True, 0.1, 1e-5)
    if res:
        ref = ref + rf
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    torch.testing.assert_close(rm, rm2, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-3)
    dy = torch.randn_like(ref).to(dt).contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    dx, ds, db, dres = KN.bn_backward(dy, y, x, scale, mean, invstd, relu=relu, want_dres=res, bias=bias)
    tol = dict(rtol=5e-2, atol=5e-2) if dt == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    # an output within rounding of 0 can take the other side of the ReLU in the fused kernel
    # (x*a + b folded, bf16 store) than in the fp32 reference: compare where both agree
    agree = ((y.float() > 0) == (ref.detach() > 0)) if relu else torch.ones_like(ref, dtype=torch.bool)
    assert agree.float().mean() > 0.9999
    torch.testing.assert_close(torch.where(agree, dx.float(), xf.grad), xf.grad, **tol)
    torch.testing.assert_close(ds, sf.grad, rtol=2e-2, atol=2e-1 if dt == torch.bfloat16 else 1e-2)
    torch.testing.assert_close(db, bf.grad, rtol=2e-2, atol=2e-1 if dt == torch.bfloat16 else 1e-2)
    if res:
        torch.testing.assert_close(torch.where(agree, dres.float(), rf.grad), rf.grad, **tol)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('res', [False, True])
@pytest.mark.parametrize('N,C,H,W', [(8, 64, 14, 14), (2, 2048, 7, 7), (3, 24, 5, 7)])
def test_batchnorm_relu_keep_bits(dt, res, N, C, H, W):
    """The forward's packed ReLU keep-bits drive the backward exactly as re-reading y does."""
    x = torch.randn(N, C, H, W, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    scale, bias = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mask = torch.full((KN.relu_mask_bytes(x),), 0xAA, dtype=torch.uint8, device=DEV)
    y, mean, invstd = KN.bn_forward(x, scale, bias, rm, rv, 0.1, 1e-5, True, relu=True, residual=r, mask=mask)
    y0, _, _ = KN.bn_forward(x, scale, bias, rm.clone(), rv.clone(), 0.1, 1e-5, True, relu=True, residual=r)
    assert torch.equal(y, y0)
    V = 8 if dt == torch.bfloat16 else 4
    keep = (y.permute(0, 2, 3, 1).reshape(-1, V) > 0).to(torch.int32)
    bits = (keep << torch.arange(V, device=DEV, dtype=torch.int32)).sum(1)
    assert torch.equal(bits.to(torch.uint8), mask)
    dy = torch.randn_like(x)
    a = KN.bn_backward(dy, y, x, scale, mean, invstd, relu=True, want_dres=res, bias=bias, mask=mask)
    b = KN.bn_backward(dy, y, x, scale, mean, invstd, relu=True, want_dres=res, bias=None)   # mask from y
    for u, v in zip(a, b):
        if u is not None:
            torch.testing.assert_close(u.float(), v.float(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_softmax_and_ce(dt):
    x = torch.randn(300, 1000, device=DEV).to(dt)
    lab = F.one_hot(torch.randint(0, 1000, (300,), device=DEV), 1000).float()
    torch.testing.assert_close(KS.softmax(x).float(), torch.softmax(x.float(), -1), **_tol(dt))
    loss, lse = KS.softmax_ce(x, lab)
    ref = -(lab * torch.log_softmax(x.float(), -1)).sum(-1)
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    g = torch.rand(300, device=DEV)
    dx = KS.softmax_ce_backward(x, lab, g, lse)
    refd = g[:, None] * (torch.softmax(x.float(), -1) - lab)
    torch.testing.assert_close(dx.float(), refd, **_tol(dt))
    ids = torch.randint(0, 1000, (300,), device=DEV)
    ids[::7] = -1
    ls, lse2 = KS.softmax_ce_sparse(x, ids, -1)
    valid = ids >= 0
    refs = torch.where(valid, F.cross_entropy(x.float(), ids.clamp_min(0), reduction='none'), torch.zeros(300, device=DEV))
    torch.testing.assert_close(ls, refs, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('N', [30522, 1001, 7, 520])
def test_sparse_softmax_ce_unaligned_rows(dt, N):
    """Vocabulary-wide rows whose starts are not 16-byte aligned (scalar head,
    vector body, scalar tail), forward loss and backward gradient."""
    R = 67
    x = (torch.randn(R, N, device=DEV) * 3).to(dt)
    ids = torch.randint(0, N, (R,), device=DEV)
    ids[::5] = -1
    valid = ids >= 0
    ls, lse = KS.softmax_ce_sparse(x, ids, -1)
    ref = torch.where(valid, F.cross_entropy(x.float(), ids.clamp_min(0), reduction='none'), torch.zeros(R, device=DEV))
    torch.testing.assert_close(ls, ref, rtol=1e-4, atol=1e-4)
    g = torch.rand(R, device=DEV)
    for l in (lse, None):
        dx = KS.softmax_ce_sparse_backward(x, ids, g, l, -1)
        refd = (g * valid.float())[:, None] * (torch.softmax(x.float(), -1) - F.one_hot(ids.clamp_min(0), N).float())
        torch.testing.assert_close(dx.float(), refd, **_tol(dt))


@pytest.mark.parametrize('n', [100003, 100000])   # the unrolled non-temporal kernel, with and without a tail
@pytest.mark.parametrize('mode', ['sgd', 'momentum', 'nesterov', 'adagrad', 'adam', 'adamw', 'lamb'])
def test_flat_optimizer(mode, n):
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    s1 = torch.rand(n, device=DEV)
    s2 = torch.rand(n, device=DEV)
    sh = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    offs = torch.tensor([0, 1000, 50000, n], dtype=torch.int64, device=DEV)
    ws = torch.zeros(6, device=DEV)
    kw = dict(lr=0.01, mu=0.9, beta1=0.9, beta2=0.999, beta1t=0.9 ** 3, beta2t=0.999 ** 3, eps=1e-7, wd=0.01, l2=0.001)
    P2, G2, A, Bs = p.cpu().clone(), g.cpu().clone(), s1.cpu().clone(), s2.cpu().clone()
    KO.optimizer_flat(mode, p, g, s1, s2, sh, seg_off=offs, seg_off_host=offs.cpu().tolist(), norms_ws=ws, **kw)
    KO.optimizer_flat(mode, P2, G2, A, Bs, None, seg_off=None, seg_off_host=offs.cpu().tolist(), **kw)
    torch.testing.assert_close(p.cpu(), P2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(sh.float().cpu(), P2, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('k,s,p,h', [(3, 2, 1, 56), (3, 2, 1, 57), (2, 2, 0, 30), (3, 1, 1, 19)])
def test_pooling(dt, k, s, p, h):
    """max pooling forward / backward (the backward's 2x2-window fast path for windows
    no wider than stride + 1, the general loop otherwise) against torch"""
    x = torch.randn(4, 64, h, h + 1, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    y, idx = KP.maxpool2d(x, k, k, s, s, p, p)
    xf = x.float().requires_grad_(True)
    ref = F.max_pool2d(xf, k, s, p)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    dy = torch.randn_like(ref)
    ref.backward(dy)
    dx = KP.maxpool2d_backward(dy.to(dt), idx, x.shape, k, k, s, s, p, p)
    torch.testing.assert_close(dx.float(), xf.grad, **_tol(dt))
    if (k, s) != (3, 2) or h != 56:
        return
    ya = KP.avgpool2d(x, 2, 2, 2, 2, 0, 0)
    torch.testing.assert_close(ya.float(), F.avg_pool2d(x.float(), 2, 2), **_tol(dt))
    gp = KR.global_avg_pool(x)
    torch.testing.assert_close(gp.float(), x.float().mean((2, 3)), **_tol(dt))


def test_reductions():
    x = torch.randn(64, 1000, 37, device=DEV)
    torch.testing.assert_close(KR.reduce_mid(x), x.sum(1), rtol=1e-4, atol=1e-3)
    # few output columns over a long axis (the MoE gate statistics [T, E] over T): the
    # chunk count is capped so the final pass stays short -- every row still summed once
    for shape in ((1, 65536, 2), (3, 40000, 5), (1, 1000003, 1)):
        x = torch.rand(*shape, device=DEV)
        torch.testing.assert_close(KR.reduce_mid(x), x.double().sum(1).float(), rtol=2e-5, atol=1e-3)
    y = torch.randn(5000, 300, device=DEV)
    torch.testing.assert_close(KR.reduce_last(y), y.sum(1), rtol=1e-4, atol=1e-3)
    # 16-byte vector form (C % 8 == 0 bf16 / C % 4 == 0 fp32) and the scalar form, bf16 rows
    for R, C in ((4096, 2048), (333, 1000), (70, 36), (9, 4104)):
        yb = torch.randn(R, C, device=DEV).bfloat16()
        ref = yb.float().sum(1)
        got = KR.reduce_last(yb, out_dtype=torch.float32)
        torch.testing.assert_close(got, ref, rtol=1e-3, atol=1e-2 * C ** 0.5)
        torch.testing.assert_close(KR.reduce_last(yb, 0.5).float(), 0.5 * ref, rtol=2e-2, atol=2e-2 * C ** 0.5)
    g = torch.randn(32, 16, 128, device=DEV)
    torch.testing.assert_close(KR.sum_to_shape(g, (128,)), g.sum((0, 1)), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_embedding_gather_scatter(dt):
    table = torch.randn(10000, 128, device=DEV).to(dt)
    ids = torch.randint(-5, 10005, (4096,), device=DEV)
    out = KSP.gather_rows(table, ids)
    valid = (ids >= 0) & (ids < 10000)
    ref = torch.where(valid[:, None], table[ids.clamp(0, 9999)].float(), torch.zeros(1, device=DEV))
    torch.testing.assert_close(out.float(), ref)
    dst = torch.zeros(10000, 128, device=DEV)
    src = torch.randn(4096, 128, device=DEV)
    KSP.scatter_add_rows(dst, ids, src)
    ref2 = torch.zeros(10000, 128, device=DEV)
    ref2.index_add_(0, ids[valid], src[valid])
    torch.testing.assert_close(dst, ref2, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_layernorm(dt):
    x = torch.randn(2048, 768, device=DEV).to(dt)
    gm = torch.rand(768, device=DEV) + 0.5
    bt = torch.randn(768, device=DEV)
    y, mean, rstd = KLN.layer_norm(x, gm, bt, 1e-5)
    xf = x.float().requires_grad_(True)
    gf, bf = gm.clone().requires_grad_(True), bt.clone().requires_grad_(True)
    ref = F.layer_norm(xf, (768,), gf, bf, 1e-5)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    dy = torch.randn_like(ref)
    ref.backward(dy)
    dx, dg, db = KLN.layer_norm_backward(dy.to(dt), x, gm, mean, rstd)
    tol = dict(rtol=5e-2, atol=5e-2) if dt == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(dx.float(), xf.grad, **tol)
    torch.testing.assert_close(dg, gf.grad, rtol=2e-2, atol=5e-1 if dt == torch.bfloat16 else 1e-2)
    torch.testing.assert_close(db, bf.grad, rtol=2e-2, atol=5e-1 if dt == torch.bfloat16 else 1e-2)


def test_dropout_mask_recompute():
    x = torch.ones(1 << 20, device=DEV)
    y1 = KD.dropout(x, 0.7, 1234)
    y2 = KD.dropout(x, 0.7, 1234)
    assert torch.equal(y1, y2)
    keep = (y1 != 0).float().mean().item()
    assert abs(keep - 0.7) < 0.01
    torch.testing.assert_close(y1[y1 != 0], torch.full_like(y1[y1 != 0], 1 / 0.7))


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_csr_spmm_spmv(dt):
    import numpy as np
    import scipy.sparse
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.kernels import spmm as KSPM
    rng = np.random.RandomState(0)
    m = scipy.sparse.random(300, 200, density=0.05, random_state=rng, format='csr', dtype=np.float32)
    a = ht.sparse_array(m.data, (m.tocoo().row, m.tocoo().col), (300, 200))
    dense = torch.from_numpy(m.toarray()).to(DEV)
    b = torch.randn(200, 300, device=DEV).to(dt)
    tol = _tol(dt)
    torch.testing.assert_close(KSPM.csrmm(a, b).float(), dense @ b.float(), **tol)
    bt = torch.randn(300, 70, device=DEV).to(dt)
    torch.testing.assert_close(KSPM.csrmm(a, bt, trans_A=True).float(), dense.t() @ bt.float(), **tol)
    # column window [50, 120): B rows indexed relative to 50
    bw = torch.randn(70, 33, device=DEV).to(dt)
    torch.testing.assert_close(KSPM.csrmm(a, bw, col_window=(50, 120)).float(),
                               dense[:, 50:120] @ bw.float(), **tol)
    x = torch.randn(200, device=DEV).to(dt)
    torch.testing.assert_close(KSPM.csrmv(a, x).float(), dense @ x.float(), **tol)


def test_elementwise_offset_views_take_the_scalar_path():
    """Contiguous views at an element offset (not 16-byte aligned) through the
    unary / binary kernels (vector path needs aligned bases)."""
    from hetu_61a7_amd.kernels import elementwise as E
    for dt in (torch.float32, torch.bfloat16):
        base = torch.randn(1 + 4 * 1000, device='cuda').to(dt)
        x = base[1:]                      # 2- or 4-byte aligned only
        assert x.data_ptr() % 16 != 0
        y = E.unary('relu', x)
        assert torch.equal(y.float(), torch.relu(x.float()).to(dt).float())
        b = torch.randn(4, device='cuda').to(dt)
        z = E.binary('add', x.view(1000, 4), b)
        ref = (x.float().view(1000, 4) + b.float()).to(dt).float()
        assert torch.allclose(z.float(), ref, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize('n,nu,dim,dt', [(8192, 2, 768, torch.bfloat16), (8192, 128, 768, torch.float32),
                                         (5000, 4000, 64, torch.bfloat16), (33, 1, 16, torch.float32)])
def test_dedup_rows_heavy_duplication(n, nu, dim, dt):
    """kernels.sparse.dedup_rows (IndexedSlices dedup) spreads heavily duplicated
    ids over private replicas: same sums as torch index_add."""
    from hetu_61a7_amd.kernels.sparse import dedup_rows
    torch.manual_seed(0)
    idx = torch.randint(0, nu, (n,), device='cuda') * 7 + 3
    vals = torch.randn(n, dim, device='cuda').to(dt)
    uniq, merged = dedup_rows(idx, vals)
    ru, inv = torch.unique(idx, sorted=True, return_inverse=True)
    ref = torch.zeros(ru.numel(), dim, device='cuda').index_add_(0, inv, vals.float())
    assert torch.equal(uniq, ru)
    torch.testing.assert_close(merged, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize('n,nrows,dim', [(8192, 2, 768), (8192, 512, 768), (100, 4000, 64)])
def test_dedup_rows_dense_matches_sparse_update(n, nrows, dim):
    """kernels.sparse.dedup_rows_dense (no host sync): summed rows for every hit id,
    -1 for untouched rows, out-of-range ids dropped; an Adam sparse update through
    it equals the update through the unique-id dedup."""
    from hetu_61a7_amd.kernels.sparse import dedup_rows_dense, dedup_rows
    from hetu_61a7_amd.kernels import optim as KO
    torch.manual_seed(0)
    idx = torch.randint(-1, min(nrows, 128), (n,), device='cuda')
    vals = torch.randn(n, dim, device='cuda').to(torch.bfloat16)
    ids, merged = dedup_rows_dense(idx, vals, nrows)
    valid = idx >= 0
    ref = torch.zeros(nrows, dim, device='cuda').index_add_(0, idx[valid], vals[valid].float())
    hit = torch.zeros(nrows, dtype=torch.bool, device='cuda')
    hit[idx[valid]] = True
    assert torch.equal(ids >= 0, hit)
    torch.testing.assert_close(merged[hit], ref[hit], rtol=1e-4, atol=1e-3)
    tabs = [torch.randn(nrows, dim, device='cuda') for _ in range(2)]
    tabs[1].copy_(tabs[0])
    st = [(torch.zeros(nrows, dim, device='cuda'), torch.zeros(nrows, dim, device='cuda')) for _ in range(2)]
    u, m = dedup_rows(idx[valid], vals[valid])
    KO.sparse_update('adam', tabs[0], u, m, st[0][0], st[0][1], lr=0.01, beta1t=0.9, beta2t=0.999)
    KO.sparse_update('adam', tabs[1], ids, merged, st[1][0], st[1][1], lr=0.01, beta1t=0.9, beta2t=0.999)
    torch.testing.assert_close(tabs[1], tabs[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(st[1][1], st[0][1], rtol=1e-5, atol=1e-6)
