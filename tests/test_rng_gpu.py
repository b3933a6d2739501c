"""Graph-safe RNG kernels (csrc/kernels/random.hip, kernels/rng.py) against host
references of the same Philox streams: channel dropout (reference Dropout2d.cu), uniform /
normal fills, arange, and the dense-to-sparse MoE gate (moe.hip dts_gate_k) against the
numpy Philox / softmax / top-k reference for several expert counts, budgets and dtypes."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht
from hetu_61a7_amd.kernels import rng
from hetu_61a7_amd.kernels import moe as KM

pytestmark = pytest.mark.gpu


def _cl(x):
    return x.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('layout', ['nchw', 'cl', '2d'])
def test_dropout2d_matches_host_philox(dtype, layout):
    from hetu_61a7_amd.ops.nn import _dropout2d
    g = torch.Generator().manual_seed(0)
    shape = (6, 40, 7, 5) if layout != '2d' else (33, 70)
    x = torch.randn(shape, generator=g).to(dtype)
    xd = x.cuda()
    if layout == 'cl':
        xd = _cl(xd)
    rng.counter()
    seed = rng.next_seed(777)
    y = _dropout2d(xd, 0.7, seed)
    torch.cuda.synchronize()
    eff = rng.effective_seed(seed)
    ref = _dropout2d(x.float(), 0.7, eff)
    np.testing.assert_allclose(y.float().cpu().numpy(), ref.numpy(), rtol=1e-2 if dtype == torch.bfloat16 else 1e-6,
                               atol=1e-6)
    # whole planes are zero or kept, about 70 % kept
    planes = (y.float().cpu().reshape(shape[0], shape[1], -1) != 0).any(-1).float().mean().item()
    assert 0.55 < planes < 0.85, planes
    # the gradient op regenerates the same planes from the seed
    gy = _dropout2d(torch.ones_like(xd), 0.7, seed)
    torch.cuda.synchronize()
    gref = _dropout2d(torch.ones(shape), 0.7, eff)
    np.testing.assert_allclose(gy.float().cpu().numpy(), gref.numpy(), rtol=1e-2, atol=0)


def test_step_counter_varies_masks_and_replays_them():
    from hetu_61a7_amd.kernels.dropout import dropout
    x = torch.ones(1 << 16, device='cuda')
    rng.set_base_seed(9)
    rng.new_step()
    s1 = rng.next_seed(5)
    a = dropout(x, 0.5, s1)
    a2 = dropout(x, 0.5, s1)          # same step: the backward's regenerated mask
    rng.new_step()
    s2 = rng.next_seed(5)
    assert s1 == s2                   # host seeds repeat per step (replayable launches)
    b = dropout(x, 0.5, s2)
    torch.cuda.synchronize()
    assert torch.equal(a, a2)
    assert not torch.equal(a, b)      # the device counter moved between the steps
    rng.set_base_seed(9)              # a new executor with the same seed: the same stream
    rng.new_step()
    c = dropout(x, 0.5, rng.next_seed(5))
    torch.cuda.synchronize()
    assert torch.equal(a, c)


def test_uniform_normal_arange_full():
    n = 1 << 20
    u = rng.uniform_(torch.empty(n, device='cuda'), -2.0, 3.0, seed=rng.next_seed(11))
    z = rng.normal_(torch.empty(n, device='cuda'), 1.5, 2.0, seed=rng.next_seed(12))
    t = rng.normal_(torch.empty(n, device='cuda'), 0.0, 1.0, trunc=2.0, seed=rng.next_seed(13))
    u, z, t = u.cpu(), z.cpu(), t.cpu()
    assert u.min() >= -2.0 and u.max() < 3.0 and abs(u.mean().item() - 0.5) < 0.02
    assert abs(z.mean().item() - 1.5) < 0.02 and abs(z.std().item() - 2.0) < 0.02
    assert t.abs().max() <= 2.0 and abs(t.std().item() - 0.8796) < 0.01   # std of N(0,1) cut at 2
    a = rng.arange(1000, 3.0, 0.5).cpu()
    np.testing.assert_allclose(a.numpy(), np.arange(1000) * 0.5 + 3.0, rtol=1e-6)
    x = ht.Variable(name='fx')
    f = ht.full_op((3, 5), 2.5)
    r = ht.rand_op((64, 64))
    ar = ht.arange_op(0.0, 10.0, 2.0)
    ex = ht.Executor([f, r, ar], ctx=ht.gpu(0))
    fv, rv, av = ex.run(feed_dict={}, convert_to_numpy_ret_vals=True)
    assert (fv == 2.5).all() and fv.shape == (3, 5)
    assert rv.shape == (64, 64) and 0.0 < rv.min() and rv.max() < 1.0 and abs(rv.mean() - 0.5) < 0.05
    np.testing.assert_allclose(av, [0, 2, 4, 6, 8])
    del x


@pytest.mark.parametrize('E,k', [(2, 1), (2, 2), (16, 1), (16, 2), (16, 16), (64, 1), (64, 2), (64, 16)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_dts_gate_kernel_matches_numpy_reference(E, k, dtype):
    """the HIP gate (Philox Gumbel noise, tempered softmax, top-k with
    lowest-id ties, threshold, per-block histogram) against the numpy reference"""
    T = 4099
    g = torch.Generator().manual_seed(E * 31 + k)
    logits = (torch.randn(T, E, generator=g) * 2).to(dtype)
    inv_tau, thr = 1.0 / 0.7, 0.1
    seed = rng.next_seed(4242 + E)
    val, idx, probs, hist = KM.dts_gate(logits.cuda(), k, inv_tau, thr, seed, noise=True)
    torch.cuda.synchronize()
    rv, ri, rp, rh = KM.dts_gate(logits.float(), k, inv_tau, thr, rng.effective_seed(seed), noise=True)
    p = probs.cpu()
    # __logf / __expf on the device vs libm on the host: the Gumbel transform -log(-log u)
    # amplifies the fast-math error for u next to 1, so a handful of tokens differ more
    bad = ((p - rp).abs() > 1e-5 + 2e-3 * rp.abs()).any(-1)
    assert bad.float().mean() < 2e-3, bad.float().mean()
    np.testing.assert_allclose(p[~bad].numpy(), rp[~bad].numpy(), rtol=2e-3, atol=1e-5)
    gi, gv = idx.cpu(), val.cpu()
    srt = torch.sort(rp, dim=-1, descending=True).values
    near_thr = ((srt[:, :k] - thr).abs() < 1e-4).any(-1) | bad      # a choice on the threshold
    # the chosen (expert, weight) pairs as sets: near-ties may swap the order of two choices
    # (|dp| below the fast-math error) but not the set, except for tokens on the threshold
    key_g = torch.where(gi >= 0, gi, torch.full_like(gi, 10 ** 6))
    key_r = torch.where(ri >= 0, ri, torch.full_like(ri, 10 ** 6))
    sg, og = torch.sort(key_g, -1)
    sr, orr = torch.sort(key_r, -1)
    # a token whose k-th and (k+1)-th probabilities nearly tie may pick either expert
    # (only while the k-th choice is active: below the threshold it is dropped either way)
    edge = (((srt[:, k - 1] - srt[:, k]).abs() < 1e-4 * srt[:, k - 1] + 1e-7) & (srt[:, k - 1] >= thr - 1e-4)
            if k < E else torch.zeros(T, dtype=torch.bool))
    ok = ~near_thr & ~edge
    assert ok.float().mean() > 0.8, ok.float().mean()
    np.testing.assert_array_equal(sg[ok].numpy(), sr[ok].numpy())
    np.testing.assert_allclose(torch.gather(gv, 1, og)[ok].numpy(), torch.gather(rv, 1, orr)[ok].numpy(),
                               rtol=2e-3, atol=1e-5)
    # the histogram counts every token once and agrees with the reference up to the
    # tokens sitting on the threshold
    h = hist.cpu()
    assert int(h.sum()) == T
    assert int((h - rh).abs().sum()) <= 2 * int((~ok).sum())
