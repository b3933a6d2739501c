"""Ring attention (context parallel) over 2- and 3-rank gloo groups vs
full-sequence attention on one process: forward and dqkv, with an additive
key mask, causal and non-causal."""
import socket

import numpy as np
import pytest
import torch


def _ref(B, S, NH, D, seed, causal):
    rng = np.random.RandomState(seed)
    H = NH * D
    qkv = torch.tensor(rng.randn(B * S, 3 * H).astype(np.float32) * 0.5, requires_grad=True)
    mask = torch.zeros(B, S)
    mask[-1, -3:] = -10000.0
    x = qkv.reshape(B, S, 3, NH, D)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = q @ k.transpose(-1, -2) / np.sqrt(D) + mask.reshape(B, 1, 1, S)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float('-inf'))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * S, H)
    g = torch.tensor(rng.randn(B * S, H).astype(np.float32))
    o.backward(g)
    return qkv.detach(), mask, g, o.detach(), qkv.grad


def _worker(rank, world, port, causal, q):
    import os
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HETU_USE_CONFIG='0')
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.parallel.ring_attention import ring_attention_op
    from hetu_61a7_amd.parallel import comm as C
    B, S, NH, D = 2, 12 * world, 3, 8
    qkv, mask, g, o_ref, dqkv_ref = _ref(B, S, NH, D, 0, causal)
    S_l = S // world
    rows = np.concatenate([np.arange(b * S + rank * S_l, b * S + (rank + 1) * S_l) for b in range(B)])
    comm = C.init_process_group(use_gpu=False)
    x = ht.Variable(name='qkv', trainable=False)
    m = ht.Variable(name='mask', trainable=False)
    gout = ht.Variable(name='gout', trainable=False)
    out = ring_attention_op(x, m, B, S_l, NH, comm=comm, causal=causal)
    loss = ht.reduce_sum_op(ht.mul_op(out, gout), None)
    (dx,) = ht.gradients(loss, [x])
    ex = ht.Executor([out, dx], ctx=ht.cpu(0))
    o, d = ex.run(feed_dict={x: qkv.numpy()[rows], m: mask.numpy()[:, rank * S_l:(rank + 1) * S_l],
                             gout: g.numpy()[rows]}, convert_to_numpy_ret_vals=True)
    q.put((rank, float(np.abs(o - o_ref.numpy()[rows]).max()),
           float(np.abs(d - dqkv_ref.numpy()[rows]).max())))
    C.destroy()


@pytest.mark.parametrize('world,causal', [(2, False), (2, True), (3, True)])
def test_ring_attention_matches_full_attention(world, causal):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, causal, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, eo, ed in res:
        assert eo < 1e-5 and ed < 1e-5, (rank, eo, ed)
