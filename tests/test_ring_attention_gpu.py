"""Ring-attention block math on the fused MFMA attention kernels (bf16, D=64):
a sequence split into P key blocks, each (query block, key block) pair run
through ``attention_{fwd,bwd}_blocks`` with strided Q / K / V operands, the
forward merged with logaddexp and the backward handed the GLOBAL out / lse --
must reproduce full-sequence fp32 attention.  This is exactly the per-step
work of ``ring_attention_fwd/bwd`` on each rank; the ring transport itself is
covered by tests/test_ring_attention_cpu.py."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('nblk,S_l', [(2, 64), (4, 128)])
def test_block_merge_matches_full_attention(nblk, S_l):
    from hetu_61a7_amd import _base
    from hetu_61a7_amd.parallel import ring_attention as RA
    assert _base.has_kernels()
    torch.manual_seed(0)
    B, NH, D = 2, 4, 64
    H, S = NH * D, nblk * S_l
    dev = 'cuda'
    qkv = (torch.randn(B, S, 3 * H, device=dev) * 0.5).to(torch.bfloat16)
    mask = torch.zeros(B, S, device=dev)
    mask[1, -5:] = -10000.0
    g = torch.randn(B, S, H, device=dev).to(torch.bfloat16)

    # fp32 reference
    x = qkv.float().requires_grad_(True)
    q, k, v = [x[..., i * H:(i + 1) * H].reshape(B, S, NH, D).transpose(1, 2) for i in range(3)]
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D) + mask.reshape(B, 1, 1, S), -1)
    o_ref = (p @ v).transpose(1, 2).reshape(B, S, H)
    o_ref.backward(g.float())

    scale = 1.0 / math.sqrt(D)
    qb = qkv[:, :S_l].reshape(B * S_l, 3 * H)                    # rank 0's query block
    kvs = [qkv[:, j * S_l:(j + 1) * S_l, H:].reshape(B * S_l, 2 * H).contiguous() for j in range(nblk)]
    ms = [mask[:, j * S_l:(j + 1) * S_l].contiguous() for j in range(nblk)]
    assert all(RA._use_fused(qb[:, :H], kv[:, :H], kv[:, H:], S_l, D, False) for kv in kvs)
    o = torch.zeros(B, S_l, NH, D, device=dev)
    lse = torch.full((B, NH, S_l), float('-inf'), device=dev)
    for kv, m in zip(kvs, ms):
        ob, lb = RA._block_fwd(qb[:, :H], kv[:, :H], kv[:, H:], m, B, S_l, NH, D, scale, False)
        new = torch.logaddexp(lse, lb)
        o = o * torch.exp(lse - new).transpose(1, 2).unsqueeze(-1) + ob.float() * torch.exp(lb - new).transpose(1, 2).unsqueeze(-1)
        lse = new
    out = o.reshape(B * S_l, H).to(torch.bfloat16)
    torch.testing.assert_close(out.float(), o_ref[:, :S_l].reshape(B * S_l, H).detach(), atol=2e-2, rtol=2e-2)

    dout = g[:, :S_l].reshape(B * S_l, H)
    dq = torch.zeros(B * S_l, H, device=dev)
    for j, (kv, m) in enumerate(zip(kvs, ms)):
        gq, gk, gv = RA._block_bwd(dout, qb[:, :H], kv[:, :H], kv[:, H:], out, lse, m, B, S_l, NH, D, scale, False)
        dq += gq.float()
        # rank 0's queries' share of key block j's gradient: reference with only those queries
        x2 = qkv.float().requires_grad_(True)
        q2, k2, v2 = [x2[..., i * H:(i + 1) * H].reshape(B, S, NH, D).transpose(1, 2) for i in range(3)]
        p2 = torch.softmax(q2[:, :, :S_l] @ k2.transpose(-1, -2) * scale + mask.reshape(B, 1, 1, S), -1)
        (p2 @ v2).transpose(1, 2).reshape(B, S_l, H).backward(g[:, :S_l].float())
        ref_k = x2.grad[:, j * S_l:(j + 1) * S_l, H:2 * H].reshape(B * S_l, H)
        ref_v = x2.grad[:, j * S_l:(j + 1) * S_l, 2 * H:].reshape(B * S_l, H)
        torch.testing.assert_close(gk.float(), ref_k, atol=3e-2, rtol=3e-2)
        torch.testing.assert_close(gv.float(), ref_v, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(dq, x.grad[:, :S_l, :H].reshape(B * S_l, H), atol=3e-2, rtol=3e-2)


def test_single_rank_ring_attention_op_gpu():
    """P == 1 ring attention through the executor on cuda:0 (fused path)."""
    import numpy as np
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.parallel import comm as C
    from hetu_61a7_amd.parallel.ring_attention import ring_attention_op
    from hetu_61a7_amd.kernels import attention as KA
    B, S, NH, D = 2, 128, 4, 64
    H = NH * D
    comm = C.init_process_group(use_gpu=True)
    x = ht.Variable(name='qkv', trainable=False)
    gout = ht.Variable(name='gout', trainable=False)
    out = ring_attention_op(x, None, B, S, NH, comm=comm)
    loss = ht.reduce_sum_op(ht.mul_op(out, gout), None)
    (dx,) = ht.gradients(loss, [x])
    ex = ht.Executor([out, dx], ctx=ht.gpu(0), mixed_precision='bf16')
    rng = np.random.RandomState(0)
    qkv = (rng.randn(B * S, 3 * H) * 0.5).astype(np.float32)
    g = rng.randn(B * S, H).astype(np.float32)
    o, d = ex.run(feed_dict={x: qkv, gout: g}, convert_to_numpy_ret_vals=True)
    qt = torch.tensor(qkv, device='cuda').to(torch.bfloat16)
    o_ref, lse = KA.attention_fwd(qt, None, B, S, NH)
    d_ref = KA.attention_bwd(torch.tensor(g, device='cuda'), qt, o_ref, lse, None, B, S, NH)
    np.testing.assert_allclose(o, o_ref.float().cpu().numpy(), atol=3e-2, rtol=3e-2)
    np.testing.assert_allclose(d, d_ref.float().cpu().numpy(), atol=5e-2, rtol=5e-2)
    C.destroy()


class _ThreadRing:
    """in-process P-rank point-to-point transport for one thread per rank: sends are
    queued device copies, receives block until the peer's send arrives"""

    def __init__(self, P):
        import queue
        self.P = P
        self.q = {(a, b): queue.Queue() for a in range(P) for b in range(P)}

    def comm(self, rank):
        ring = self

        class _C:
            nrank = ring.P

            def batch_p2p(self, ops):
                for kind, t, peer in ops:
                    if kind == 'send':
                        c = t.clone()
                        torch.cuda.synchronize()
                        ring.q[(self.rank, peer)].put(c)
                for kind, t, peer in ops:
                    if kind == 'recv':
                        t.copy_(ring.q[(peer, self.rank)].get(timeout=60))
                torch.cuda.synchronize()
                return []
        c = _C()
        c.rank = rank
        return c


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize('causal', [False, True])
def test_ring_attention_flash_path_four_ranks(causal):
    """ring_attention_fwd / _bwd on the flash kernels (S/P = 100: no fused-kernel shape), four
    ranks as threads over an in-process ring: every rank's output and dQKV match full-sequence
    fp32 attention (causal: the diagonal block masked, blocks above it skipped)."""
    import threading
    from hetu_61a7_amd import _base
    from hetu_61a7_amd.parallel import ring_attention as RA
    assert _base.has_kernels()
    torch.manual_seed(0)
    P, B, NH, D, S_l = 4, 2, 2, 64, 100
    H, S = NH * D, P * S_l
    qkv = (torch.randn(B, S, 3 * H, device='cuda') * 0.5).to(torch.bfloat16)
    mask = torch.zeros(B, S, device='cuda')
    mask[1, -7:] = -10000.0
    g = torch.randn(B, S, H, device='cuda').to(torch.bfloat16)
    x = qkv.float().requires_grad_(True)
    q, k, v = [x[..., i * H:(i + 1) * H].reshape(B, S, NH, D).transpose(1, 2) for i in range(3)]
    s = q @ k.transpose(-1, -2) / math.sqrt(D) + mask.reshape(B, 1, 1, S)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device='cuda').triu_(1), float('-inf'))
    o_ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, H)
    o_ref.backward(g.float())
    assert RA._flash_ring_ok(qkv[:, :S_l].reshape(B * S_l, 3 * H).contiguous(), NH)

    ring = _ThreadRing(P)
    res, errs = {}, []

    def rank_main(r):
        try:
            torch.cuda.set_device(0)
            qb = qkv[:, r * S_l:(r + 1) * S_l].reshape(B * S_l, 3 * H).contiguous()
            mb = mask[:, r * S_l:(r + 1) * S_l].contiguous()
            c = ring.comm(r)
            out, lse = RA.ring_attention_fwd(qb, mb, c, B, S_l, NH, causal)
            dq = RA.ring_attention_bwd(g[:, r * S_l:(r + 1) * S_l].reshape(B * S_l, H).contiguous(), qb, mb, out,
                                       lse, c, B, S_l, NH, causal)
            torch.cuda.synchronize()
            res[r] = (out, dq)
        except Exception as e:       # noqa: BLE001 -- surfaced below
            errs.append((r, repr(e)))
    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    for r in range(P):
        out, dq = res[r]
        sl = slice(r * S_l, (r + 1) * S_l)
        assert _rel(out, o_ref[:, sl].reshape(B * S_l, H)) < 2e-2, r
        assert _rel(dq, x.grad[:, sl].reshape(B * S_l, 3 * H)) < 3e-2, r
