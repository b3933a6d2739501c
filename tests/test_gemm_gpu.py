"""Hand-written MFMA GEMM / implicit-GEMM conv vs plain PyTorch fp32."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from hetu_61a7_amd.kernels import gemm_mfma as G, conv_igemm as CI

DEV = 'cuda'
CL = torch.channels_last


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


def _tol(y):
    """bound on the relative-norm error against fp32 math on the same bf16 operands:
    bf16 x bf16 products are exact in fp32 and the fp32 accumulation error is ~1e-7 *
    sqrt(K), so a bf16 output is off by its own rounding (rms ~2^-9 relative) and an fp32
    output by almost nothing.  A dropped K-tail or a 0.5 % systematic error fails."""
    return 4e-3 if y.dtype == torch.bfloat16 else 2e-5


@pytest.mark.parametrize('tile', G.TILES)
@pytest.mark.parametrize('ta', [False, True])
@pytest.mark.parametrize('tb', [False, True])
@pytest.mark.parametrize('mnk', [(256, 256, 256), (200, 136, 72), (1000, 8, 520), (64, 1032, 4096),
                                 (520, 776, 1000), (768, 512, 64)])
def test_gemm_modes(ta, tb, mnk, tile):
    M, N, K = mnk
    a = torch.randn(K, M, device=DEV).bfloat16().t() if ta else torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16().t() if tb else torch.randn(K, N, device=DEV).bfloat16()
    y = G.gemm(a, b, tile=tile)
    assert y is not None
    ref = a.float() @ b.float()
    assert _rel(y, ref) < _tol(y)


@pytest.mark.parametrize('tile', G.TILES)
@pytest.mark.parametrize('act', [None, 'relu', 'gelu'])
def test_gemm_epilogue(act, tile):
    M, N, K = 384, 264, 128
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    cin = torch.randn(M, N, device=DEV)
    y = G.gemm(a, b, bias=bias, act=act, alpha=0.5, beta=2.0, cin=cin, out_dtype=torch.float32, tile=tile)
    ref = 0.5 * (a.float() @ b.float()) + bias + 2.0 * cin
    if act == 'relu':
        ref = torch.relu(ref)
    elif act == 'gelu':
        ref = F.gelu(ref)
    assert _rel(y, ref) < _tol(y)


@pytest.mark.parametrize('tile', G.TILES)
def test_gemm_batched_and_splitk(tile):
    a = torch.randn(6, 128, 64, device=DEV).bfloat16()
    b = torch.randn(6, 128, 64, device=DEV).bfloat16().transpose(1, 2)  # [6, 64, 128]
    y = G.gemm(a, b, tile=tile)
    assert _rel(y, a.float() @ b.float()) < _tol(y)
    x = torch.randn(8192, 96, device=DEV).bfloat16()
    g = torch.randn(8192, 136, device=DEV).bfloat16()
    out = torch.zeros(96, 136, device=DEV)
    G.gemm(x.t(), g, out=out, accumulate=True, splitk=16, tile=tile)
    assert _rel(out, x.float().t() @ g.float()) < _tol(out)
    # split-K through fp32 slabs + reduce (bf16 output)
    y2 = G.gemm(x.t(), g, splitk=4, tile=tile)
    assert _rel(y2, x.float().t() @ g.float()) < _tol(y2)


CONV_SHAPES = [  # N, C, H, K, k, stride, pad
    (4, 64, 14, 64, 1, 1, 0), (4, 64, 14, 128, 3, 1, 1), (4, 128, 15, 64, 3, 2, 1),
    (2, 256, 14, 128, 1, 2, 0), (2, 8, 32, 64, 7, 2, 3), (3, 72, 9, 40, 3, 1, 0),
    (2, 64, 16, 64, 3, 2, 1), (2, 32, 13, 64, 5, 2, 2), (2, 64, 11, 32, 3, 3, 1),
    (2, 64, 13, 128, 3, 2, 1), (2, 192, 9, 64, 3, 1, 1), (2, 128, 7, 192, 3, 1, 1),
    (2, 512, 7, 512, 3, 1, 1)]   # K = 3*3*512 = 4608: the tile-3 (short-K) candidacy edge


# tiles 6 / 7 (the two-ahead K loop) are built for the plain GEMM loaders only
CONV_TILES = [t for t in G.TILES if t not in (6, 7)]


@pytest.mark.parametrize('tile', CONV_TILES)
@pytest.mark.parametrize('shape', CONV_SHAPES)
def test_conv_passes(shape, tile):
    N, C, H, K, k, s, p = shape
    x = torch.randn(N, C, H, H, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, k, k, device=DEV) * 0.1).bfloat16().contiguous(memory_format=CL)
    y = CI.try_forward(x, w, (s, s), (p, p), tile=tile)
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    ref = F.conv2d(xf, wf, None, s, p)
    assert y is not None and y.is_contiguous(memory_format=CL)
    assert _rel(y, ref) < _tol(y)
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    ref.backward(dy.float())
    dx = CI.try_backward_data(dy, w, x.shape, (s, s), (p, p), tile=tile)
    assert dx is not None and _rel(dx, xf.grad) < _tol(dx)
    r = torch.randn_like(x)
    dx2 = CI.try_backward_data(dy, w, x.shape, (s, s), (p, p), acc=r, tile=tile)
    assert dx2 is not None and _rel(dx2, xf.grad + r.float()) < _tol(dx2)
    dw = CI.try_backward_filter(dy, x, w.shape, (s, s), (p, p), tile=tile)
    assert dw is not None and dw.dtype == torch.float32
    assert _rel(dw, wf.grad) < _tol(dw)


@pytest.mark.parametrize('tile', [2, 4])
@pytest.mark.parametrize('shape', [s for s in CONV_SHAPES if s[3] <= 64] + [(3, 64, 56, 64, 3, 1, 1)])
@pytest.mark.parametrize('accumulate', [False, True])
def test_conv_wgrad_64_channel_tiles(shape, tile, accumulate):
    """64-channel weight gradients on the 128x64 tile, as is (2) and with the roles
    swapped (4: filter taps on M, the transposed slab reduce into dw[K][taps])."""
    N, C, H, K, k, s, p = shape
    x = torch.randn(N, C, H, H, device=DEV).bfloat16().contiguous(memory_format=CL)
    wf = torch.zeros(K, C, k, k, device=DEV, requires_grad=True)
    ref = F.conv2d(x.float(), wf, None, s, p)
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    ref.backward(dy.float())
    out = torch.randn(K, C, k, k, device=DEV).contiguous(memory_format=CL)
    base = out.clone()
    dw = CI.try_backward_filter(dy, x, (K, C, k, k), (s, s), (p, p), out=out, accumulate=accumulate, tile=tile)
    assert dw is not None and dw.data_ptr() == out.data_ptr()
    got = out - base if accumulate else out
    assert _rel(got, wf.grad) < (1e-4 if accumulate else 2e-5)


@pytest.mark.parametrize('tile', [t for t in CONV_TILES if t != 5])   # 128x96: no fused statistics
@pytest.mark.parametrize('shape', [(4, 64, 14, 64, 1, 1, 0), (2, 64, 13, 200, 3, 2, 1), (3, 128, 9, 256, 3, 1, 1)])
@pytest.mark.parametrize('reps', [1, 3])
def test_conv_fused_bn_statistics(shape, tile, reps):
    """Per-channel sum / sum of squares of the stored (bf16) conv output, reduced in
    the epilogue, against a torch reduction of the same output (reps > 1: spread over
    that many replicas, Epi::cs_rep)."""
    N, C, H, K, k, s, p = shape
    x = torch.randn(N, C, H, H, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, k, k, device=DEV) * 0.1).bfloat16().contiguous(memory_format=CL)
    st = torch.zeros(reps * 2 * K, device=DEV)
    y = CI.try_forward(x, w, (s, s), (p, p), tile=tile, colstats=st)
    st = st.view(reps, 2 * K).sum(0)
    yf = y.float()
    ref_s = yf.sum((0, 2, 3))
    ref_q = (yf * yf).sum((0, 2, 3))
    assert _rel(st[:K], ref_s) < 1e-4 and _rel(st[K:], ref_q) < 1e-4
    y0 = CI.try_forward(x, w, (s, s), (p, p), tile=tile)
    assert torch.equal(y, y0)


def test_bn_from_fused_statistics_matches_plain_bn():
    from hetu_61a7_amd.kernels import norm as KN, conv as KC
    x = torch.randn(8, 64, 28, 28, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(128, 64, 3, 3, device=DEV) * 0.1).bfloat16().contiguous(memory_format=CL)
    y, sums = KC.conv2d_with_stats(x, w, (1, 1), (1, 1))
    assert sums is not None
    sc, bi = torch.rand(128, device=DEV) + 0.5, torch.randn(128, device=DEV)
    rm1, rv1 = torch.zeros(128, device=DEV), torch.ones(128, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    a, m1, i1 = KN.bn_forward(y, sc, bi, rm1, rv1, 0.1, 1e-5, True, relu=True)
    b, m2, i2 = KN.bn_forward(y, sc, bi, rm2, rv2, 0.1, 1e-5, True, relu=True, sums=sums.clone())
    assert _rel(m2, m1) < 1e-4 and _rel(i2, i1) < 1e-4 and _rel(rv2, rv1) < 1e-4
    assert _rel(b, a) < 1e-2
    s2 = KN.col_sums(y)
    assert _rel(s2, sums) < 1e-4


def test_dgrad_join_timing_leaves_operand_alone():
    """1x1 data gradient with a fused gradient join (acc, dead after the call): the join is
    the epilogue's Cin on every hand-written candidate, and timing the candidates never
    writes the live operand"""
    from hetu_61a7_amd.kernels import conv as KC, autotune
    g = torch.randn(4, 64, 14, 14, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(64, 32, 1, 1, device=DEV) * 0.1).bfloat16().contiguous(memory_format=CL)
    acc = torch.randn(4, 32, 14, 14, device=DEV).bfloat16().contiguous(memory_format=CL)
    ref = torch.einsum('nkhw,kc->nchw', g.float(), w.float().view(64, 32)) + acc.float()
    key = ('dgrad', tuple(g.shape), tuple(w.shape), (1, 1), (0, 0), True)
    autotune._decisions.pop(key, None)
    a = acc.clone(memory_format=CL)
    dx = KC.conv2d_backward_data(g, w, (4, 32, 14, 14), (1, 1), (0, 0), acc=a, acc_inplace=True)
    assert _rel(dx, ref) < _tol(dx)
    assert torch.equal(a, acc)
    assert autotune._decisions[key].startswith('hip')


def test_matmul_join_timing_leaves_operand_alone():
    from hetu_61a7_amd.kernels import gemm as KG, autotune
    a = torch.randn(512, 256, device=DEV).bfloat16()
    b = torch.randn(384, 256, device=DEV).bfloat16()
    acc = torch.randn(512, 384, device=DEV).bfloat16()
    ref = a.float() @ b.float().t() + acc.float()
    key = ('gemm_acc', KG._sig(a), KG._sig(b), False, True)
    autotune._decisions.pop(key, None)
    c = acc.clone()
    y = KG.matmul_acc(a, b, False, True, c, inplace=True)
    assert _rel(y, ref) < _tol(y)
    assert torch.equal(c, acc)
    assert autotune._decisions[key].startswith('hip')


def test_fp32_nchw_three_channel_dgrad_on_hand_written_kernel():
    """The operand mix that aborted MIOpen in round 2 (an NCHW fp32 output gradient, a
    channels-last filter, 3 input channels) now runs on the exact-fp32 MFMA kernel with the
    channels zero-padded to 4 -- there is no library path to fall back to."""
    from hetu_61a7_amd.kernels import conv as KC
    from hetu_61a7_amd import kernels as K
    K.reset_dispatch_stats()
    x = torch.randn(2, 3, 20, 20, device=DEV, requires_grad=True)
    w = (torch.randn(16, 3, 3, 3, device=DEV) * 0.1).contiguous(memory_format=CL)
    y = F.conv2d(x, w, None, 1, 1)
    g = torch.randn_like(y).contiguous()
    y.backward(g)
    dx = KC.conv2d_backward_data(g, w, tuple(x.shape), (1, 1), (1, 1))
    torch.cuda.synchronize()
    assert _rel(dx, x.grad) < 1e-4
    assert not K.FALLBACKS and not K.VENDOR_CALLS


def test_no_library_fallback_raises():
    """a device product no hand-written kernel takes raises instead of calling a library"""
    from hetu_61a7_amd.kernels import gemm as KG, NoKernelError
    a = torch.randn(8, 8, device=DEV).half()
    with pytest.raises(NoKernelError):
        KG.matmul(a, a)


@pytest.mark.parametrize('n,h', [(2, 56), (3, 57), (1, 5), (70, 5)])   # n >= 64: two-pass slab sum
def test_conv3x3_c64_halo_kernel(n, h):
    """3x3/s1/p1 64->64 halo-tile kernel: forward (+ fused BN statistics) and data
    gradient (+ bf16 / fp32 join) against fp32 autograd on the same bf16 operands."""
    x = torch.randn(n, 64, h, 56, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(64, 64, 3, 3, device=DEV) * 0.05).bfloat16().contiguous(memory_format=CL)
    st = torch.zeros(128, device=DEV)
    y = CI.try_conv3x3_forward(x, w, (1, 1), (1, 1), colstats=st)
    assert y is not None and y.is_contiguous(memory_format=CL)
    xf = x.float().requires_grad_(True)
    ref = F.conv2d(xf, w.float(), None, 1, 1)
    assert _rel(y, ref) < _tol(y)
    yf = y.float()
    assert _rel(st[:64], yf.sum((0, 2, 3))) < 1e-4 and _rel(st[64:], (yf * yf).sum((0, 2, 3))) < 1e-4
    st3 = torch.zeros(3 * 128, device=DEV)   # replicated totals: image i into replica i % 3
    assert torch.equal(CI.try_conv3x3_forward(x, w, (1, 1), (1, 1), colstats=st3), y)
    assert _rel(st3.view(3, 128).sum(0), st) < 1e-5
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    ref.backward(dy.float())
    dx = CI.try_conv3x3_backward_data(dy, w, x.shape, (1, 1), (1, 1))
    assert dx is not None and _rel(dx, xf.grad) < _tol(dx)
    for dt in (torch.bfloat16, torch.float32):
        r = torch.randn(x.shape, device=DEV).to(dt).contiguous(memory_format=CL)
        dx2 = CI.try_conv3x3_backward_data(dy, w, x.shape, (1, 1), (1, 1), acc=r)
        assert _rel(dx2, xf.grad + r.float()) < _tol(dx2)
    wf = w.float().requires_grad_(True)
    F.conv2d(x.float(), wf, None, 1, 1).backward(dy.float())
    dw = CI.try_conv3x3_backward_filter(dy, x, w.shape, (1, 1), (1, 1))
    assert dw is not None and dw.dtype == torch.float32 and _rel(dw, wf.grad) < 2e-5
    out = torch.randn(64, 64, 3, 3, device=DEV).contiguous(memory_format=CL)
    base = out.clone()
    CI.try_conv3x3_backward_filter(dy, x, w.shape, (1, 1), (1, 1), out=out, accumulate=True)
    assert _rel(out - base, wf.grad) < 1e-4


@pytest.mark.parametrize('n,c,k,h', [(2, 128, 128, 28), (3, 256, 256, 14), (3, 512, 512, 7), (1, 64, 128, 28),
                                     (2, 128, 256, 14), (1, 192, 128, 56)])
def test_conv3x3_wide_halo_kernel(n, c, k, h):
    """3x3/s1/p1 wide-channel halo kernel: pixel tiles x 128 output channels, one halo per
    64-channel chunk for all 9 taps; forward (+ BN statistics) and data gradient (+ join)."""
    x = torch.randn(n, c, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(k, c, 3, 3, device=DEV) * 0.05).bfloat16().contiguous(memory_format=CL)
    st = torch.zeros(2 * k, device=DEV)
    y = CI.try_conv3x3_forward(x, w, (1, 1), (1, 1), colstats=st)
    assert y is not None and y.is_contiguous(memory_format=CL)
    xf = x.float().requires_grad_(True)
    ref = F.conv2d(xf, w.float(), None, 1, 1)
    assert _rel(y, ref) < _tol(y)
    yf = y.float()
    assert _rel(st[:k], yf.sum((0, 2, 3))) < 1e-4 and _rel(st[k:], (yf * yf).sum((0, 2, 3))) < 1e-4
    st3 = torch.zeros(3 * 2 * k, device=DEV)   # replicated totals: pixel tile t into replica t % 3
    assert torch.equal(CI.try_conv3x3_forward(x, w, (1, 1), (1, 1), colstats=st3), y)
    assert _rel(st3.view(3, 2 * k).sum(0), st) < 1e-5
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    ref.backward(dy.float())
    if c % 128 == 0:
        dx = CI.try_conv3x3_backward_data(dy, w, x.shape, (1, 1), (1, 1))
        assert dx is not None and _rel(dx, xf.grad) < _tol(dx)
        r = torch.randn(x.shape, device=DEV).bfloat16().contiguous(memory_format=CL)
        dx2 = CI.try_conv3x3_backward_data(dy, w, x.shape, (1, 1), (1, 1), acc=r)
        assert _rel(dx2, xf.grad + r.float()) < _tol(dx2)
    else:
        assert CI.try_conv3x3_backward_data(dy, w, x.shape, (1, 1), (1, 1)) is None
    if h in (28, 14, 7):
        wf = w.float().requires_grad_(True)
        F.conv2d(x.float(), wf, None, 1, 1).backward(dy.float())
        out = torch.randn(k, c, 3, 3, device=DEV).contiguous(memory_format=CL)
        base = out.clone()
        dw = CI.try_conv3x3_backward_filter(dy, x, w.shape, (1, 1), (1, 1), out=out, accumulate=True)
        assert dw is not None and dw.data_ptr() == out.data_ptr()
        assert _rel(out - base, wf.grad) < 1e-4
        dw2 = CI.try_conv3x3_backward_filter(dy, x, w.shape, (1, 1), (1, 1))
        assert _rel(dw2, wf.grad) < 2e-5


@pytest.mark.parametrize('mnk', [(64, 2, 768), (768, 2, 64), (64, 768, 768), (3, 5, 7), (1, 1000, 2048)])
@pytest.mark.parametrize('dts', [(torch.bfloat16, torch.bfloat16), (torch.float32, torch.bfloat16),
                                 (torch.float32, torch.float32)])
def test_gemm_small_any_stride(mnk, dts):
    """the one-wave-per-output kernel for the products the MFMA tiles cannot take (N = 2
    heads, strided CLS-token rows): any strides, epilogue as the MFMA kernels"""
    M, N, K = mnk
    a = torch.randn(M, 3 * K, device=DEV).to(dts[0])[:, ::3]           # strided rows and columns
    b = torch.randn(N, K, device=DEV).to(dts[1]).t()                    # transposed view
    bias = torch.randn(N, device=DEV)
    cin = torch.randn(M, N, device=DEV)
    y = G.gemm_small(a, b, bias=bias, act='relu', alpha=0.5, beta=2.0, cin=cin, out_dtype=torch.float32)
    ref = torch.relu(0.5 * (a.float() @ b.float()) + 2.0 * cin + bias)
    assert _rel(y, ref) < 2e-5
    y2 = G.gemm_small(a, b)
    assert y2.dtype == dts[0] and _rel(y2, a.float() @ b.float()) < _tol(y2)


@pytest.mark.parametrize('pmn', [(802816, 64, 64), (50000, 128, 64), (8192, 768, 3072), (1000, 64, 192)])
@pytest.mark.parametrize('accumulate', [False, True])
def test_wgrad_longk(pmn, accumulate):
    """64x64-tile split-K weight gradient over pixel-major operands (1x1 conv / linear
    weight gradients): fp32 result against fp32 math on the same bf16 operands"""
    P_, M, N = pmn
    a = torch.randn(P_, M, device=DEV).bfloat16()
    b = torch.randn(P_, N, device=DEV).bfloat16()
    out = torch.randn(M, N, device=DEV)
    base = out.clone()
    r = G.wgrad_longk(a, b, out, accumulate=accumulate)
    assert r is not None and r.data_ptr() == out.data_ptr()
    ref = a.float().t() @ b.float()
    got = out - base if accumulate else out
    assert _rel(got, ref) < (1e-4 if accumulate else 2e-5)


@pytest.mark.parametrize('n', [1, 2, 5])
def test_gemm_into_few_columns_long_k(n):
    """out[M, n<8] = X^T @ G over a long token axis (the MoE gate's weight gradient):
    G zero-padded to 8 columns on the MFMA tile with a deep K split, against fp32 math;
    and through matmul_into's autotuned choice"""
    from hetu_61a7_amd.kernels import gemm as KG
    torch.manual_seed(5)
    x = torch.randn(8192, 512, device=DEV).bfloat16()
    g = torch.randn(8192, n, device=DEV).bfloat16()
    ref = x.float().t() @ g.float()
    for s in (16, 64):
        out = torch.full((512, n), 7.0, device=DEV)
        assert KG._pad8_into(x.t(), g, out, s) is out
        assert _rel(out, ref) < _tol(out)
    out = torch.empty(512, n, device=DEV)
    KG.matmul_into(x, g, True, False, out)
    assert _rel(out, ref) < _tol(out)


@pytest.mark.parametrize('M,N,K', [(1024, 3072, 768), (8192, 3072, 768), (300, 200, 96)])
def test_matmul_pre_stores_activation_and_pre_activation(M, N, K):
    """one GEMM epilogue storing act(x @ w + b) and the pre-activation (the training GELU
    layer's saved input) -- both equal to the fp32 reference to bf16 accuracy"""
    from hetu_61a7_amd.kernels import gemm as KG
    torch.manual_seed(0)
    a = (torch.randn(M, K, device=DEV) * 0.3).bfloat16()
    w = (torch.randn(K, N, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV) * 0.1
    y, pre = KG.matmul_pre(a, w, False, False, bias, 'gelu')
    ref_pre = a.float() @ w.float() + bias
    ref_y = torch.nn.functional.gelu(ref_pre)
    assert _rel(pre, ref_pre) < _tol(pre)
    assert _rel(y, ref_y) < _tol(y)


@pytest.mark.parametrize('M,N,K', [(4096, 2048, 512), (1000, 256, 200)])
def test_matmul_act_dropout_matches_standalone_dropout(M, N, K):
    """ReLU + dropout in the GEMM epilogue: the same Philox counters as the standalone
    dropout kernel over the [M, N] output, so dropout(relu(a @ w)) computed in two passes is
    the fused result to bf16 accuracy; the backward from the output alone (g / keep where
    out > 0) equals autograd through the two-pass form"""
    from hetu_61a7_amd.kernels import gemm as KG, dropout as KD
    from hetu_61a7_amd.kernels.elementwise import binary
    torch.manual_seed(1)
    keep, seed = 0.9, 4321
    a = (torch.randn(M, K, device=DEV) * 0.5).bfloat16()
    w = (torch.randn(K, N, device=DEV) * 0.05).bfloat16()
    y = KG.matmul_act_dropout(a, w, 'relu', keep, seed)
    ref = KD.dropout(torch.relu(a.float() @ w.float()).contiguous(), keep, seed)
    assert _rel(y, ref) < _tol(y)
    frac = float((y == 0).float().mean())
    assert 0.5 < frac < 0.6, frac          # ~half the ReLU outputs are 0, then 10 % dropped
    g = torch.randn(M, N, device=DEV).bfloat16()
    d = binary('relu_grad_c', y, g, 1.0 / keep)
    m = KD.dropout(torch.ones(M, N, device=DEV), keep, seed) * (a.float() @ w.float() > 0).float()
    assert _rel(d, g.float() * m) < _tol(d)


@pytest.mark.parametrize('tile', [0, 1, 3, 6])
@pytest.mark.parametrize('M,N,K,tb', [(4096, 512, 768, True), (1000, 264, 136, False), (256, 2048, 2048, True)])
def test_gemm_relu_mask_epilogue(M, N, K, tb, tile):
    """The data gradient of a ReLU (+ dropout) output y masked in the GEMM epilogue:
    (g @ w^T) / keep where y > 0, else 0 -- against the plain GEMM and the relu_grad_c
    kernel, and against the fp32 torch product; autotuned entry point too."""
    from hetu_61a7_amd.kernels import gemm as KG
    from hetu_61a7_amd.kernels.elementwise import binary
    torch.manual_seed(2)
    keep = 0.9
    g = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) if tb else torch.randn(K, N, device=DEV)).bfloat16()
    y = torch.relu(torch.randn(M, N, device=DEV)).bfloat16()
    B = w.t() if tb else w
    out = G.gemm_gmask(g, B, y, 1.0 / keep, tile=tile)
    if out is None:
        pytest.skip('tile %d does not take this shape' % tile)
    ref = (g.float() @ B.float()) * (y.float() > 0).float() / keep
    assert _rel(out, ref) < _tol(out)
    assert bool((out[y == 0] == 0).all())
    two = binary('relu_grad_c', y, KG.matmul(g, w, False, tb), 1.0 / keep)
    assert _rel(out, two) < _tol(out)
    auto = KG.matmul_relu_mask(g, w, False, tb, y, 1.0 / keep)
    assert _rel(auto, ref) < _tol(auto)


@pytest.mark.parametrize('tile', [0, 1, 3, 5, 6])
@pytest.mark.parametrize('M,N,K', [(4096, 2048, 512), (1000, 264, 200), (512, 768, 2048)])
def test_dropout_keep_bits_roundtrip(M, N, K, tile):
    """The forward dropout epilogue's keep bits (one byte per 8 outputs) equal out > 0 of
    the output it stores; the backward GEMM masked by those bits equals the one masked by
    the bf16 output, for every tile either side takes"""
    from hetu_61a7_amd.kernels import gemm as KG
    torch.manual_seed(3)
    keep, seed = 0.9, 777
    a = (torch.randn(M, K, device=DEV) * 0.5).bfloat16()
    w = (torch.randn(K, N, device=DEV) * 0.05).bfloat16()
    r = G.gemm_drop_bits(a, w, 'relu', keep, seed, tile=tile)
    if r is None:
        pytest.skip('tile %d does not take this shape' % tile)
    y, bits = r
    ref_y = KG.matmul_act_dropout(a, w, 'relu', keep, seed)
    assert bool((y == ref_y).all())
    unpacked = (bits.view(-1, 1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1
    assert bool((unpacked.view(M, N).bool() == (y > 0)).all())
    g = torch.randn(M, 384, device=DEV).bfloat16()
    w2 = torch.randn(N, 384, device=DEV).bfloat16()
    out = G.gemm_gbits(g, w2.t(), bits, 1.0 / keep, tile=tile)
    if out is None:
        pytest.skip('tile %d does not take the backward shape' % tile)
    ref = G.gemm_gmask(g, w2.t(), y, 1.0 / keep, tile=tile)
    assert bool((out == ref).all())
    y2, mask = KG.matmul_act_dropout_bits(a, w, 'relu', keep, seed)
    assert mask.dtype == torch.uint8 and bool((y2 == ref_y).all())
    auto = KG.matmul_mask(g, w2, False, True, mask, 1.0 / keep)
    assert _rel(auto, (g.float() @ w2.float().t()) * (y > 0).float() / keep) < _tol(auto)


@pytest.mark.parametrize('tile', G.TILES)
@pytest.mark.parametrize('M,N,K,ta,tb', [(4096, 2, 2048, False, False), (4096, 2, 2048, False, True),
                                         (2048, 2, 4096, True, False), (4096, 8, 2048, False, True)])
def test_every_tile_declines_or_matches_narrow_outputs(M, N, K, ta, tb, tile):
    """Narrow outputs (the MoE gate: N = 2 experts): each tile either declines the shape
    (None) or computes it exactly -- the autotuner times every candidate that answers."""
    torch.manual_seed(3)
    a = torch.randn(K, M, device=DEV).bfloat16().t() if ta else torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16().t() if tb else torch.randn(K, N, device=DEV).bfloat16()
    y = G.gemm(a, b, tile=tile)
    if y is None:
        return
    ref = a.float() @ b.float()
    assert _rel(y, ref) < _tol(y)
    out = torch.full((M, N), 7.0, device=DEV)
    r = G.gemm(a, b, out=out, tile=tile)
    if r is not None:
        assert _rel(out, ref) < 2e-5

