"""Pipeline parallel (GPipe / PipeDream 1F1B) on CPU with gloo: parameters after
training must match a single-process baseline (reference
examples/runner/parallel/validate_results.py pattern)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

B, M, STEPS, LR = 16, 4, 2, 0.05


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rng = np.random.RandomState(0)
    X = rng.randn(B, 12).astype(np.float32)
    Y = np.eye(3, dtype=np.float32)[rng.randint(0, 3, B)]
    return X, Y


def _build(ht, stages):
    """3-layer MLP; stages = list of device groups (one per layer block)."""
    rng = np.random.RandomState(5)
    ws = [(rng.randn(12, 16) * .3).astype(np.float32), (rng.randn(16, 16) * .3).astype(np.float32),
          (rng.randn(16, 3) * .3).astype(np.float32)]
    blocks = {1: [[0, 1, 2]], 2: [[0, 1], [2]], 3: [[0], [1], [2]]}[len(stages)]
    h = None
    x = y_ = None
    for si, ctx in enumerate(stages):
        with ht.context(ctx):
            if si == 0:
                x = ht.Variable(name='x')
                h = x
            for li in blocks[si]:
                W = ht.Variable(name='w%d' % li, value=ws[li])
                b = ht.Variable(name='b%d' % li, value=np.zeros(ws[li].shape[1], np.float32))
                h = ht.linear_op(h, W, b)
                if li < 2:
                    h = ht.relu_op(h)
            if si == len(stages) - 1:
                y_ = ht.Variable(name='y_')
                loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(h, y_), [0])
                train = ht.optim.SGDOptimizer(LR).minimize(loss)
    return x, y_, loss, train


def _baseline(lr_scale):
    import hetu_61a7_amd as ht
    X, Y = _data()
    x, y_, loss, train = _build(ht, [ht.cpu(0)])
    train.optimizer.learning_rate = LR * lr_scale
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    for _ in range(STEPS):
        ex.run('train', feed_dict={x: X, y_: Y})
    return {n.name: v.numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items() if n.trainable}


def _worker(rank, world, port, kind, nstages, q, steps=STEPS):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HETU_USE_CONFIG='0')
    import hetu_61a7_amd as ht
    X, Y = _data()
    nrep = world // nstages
    stages = [[ht.gpu(s * nrep + r) for r in range(nrep)] if nrep > 1 else ht.gpu(s) for s in range(nstages)]
    x, y_, loss, train = _build(ht, stages)
    ex = ht.Executor({'train': [loss, train]}, pipeline=kind)
    sub = ex.subexecutor['train']
    rep = sub.replica
    shard = slice(rep * (B // nrep), (rep + 1) * (B // nrep))
    losses = []
    for _ in range(steps):
        res = ex.run('train', feed_dict={x: X[shard], y_: Y[shard]}, batch_num=M, convert_to_numpy_ret_vals=True)
        losses.append([r[0] for r in res if r is not None and r[0] is not None])
    params = {n.name: v.numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items() if n.trainable}
    q.put((rank, params, losses, sub.p2p.hdr_syncs, len(sub.recv_msgs['F']) + len(sub.recv_msgs['B'])))
    from hetu_61a7_amd.parallel import comm
    comm.destroy()


@pytest.mark.parametrize('kind,world,nstages', [('gpipe', 2, 2), ('pipedream_flush', 2, 2),
                                                ('pipedream_flush', 3, 3), ('gpipe', 4, 2)])
def test_pipeline_matches_single_process(kind, world, nstages):
    nrep = world // nstages
    # per replica: M micro-batch mean grads summed; replicas summed -> lr * M * nrep on the full batch
    base = _baseline(M * nrep)
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kind, nstages, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for _, params, _, _, _ in res:
        merged.update(params)
    assert set(merged) == set(base)
    for k, v in base.items():
        np.testing.assert_allclose(merged[k], v, rtol=1e-4, atol=1e-5, err_msg=k)


def _stash_reference(nstages, steps):
    """Explicit PipeDream (weight stashing, per-micro-batch update) simulation in torch
    autograd: micro-batch b's forward on stage s sees the stage's weights after
    max(0, b - warm_s) of its own updates (warm_s = nstages - s - 1 warm-up forwards,
    1F1B afterwards), its backward differentiates THOSE weights, and each stage applies
    its micro-batch gradients to its latest weights in micro-batch order."""
    import torch
    X, Y = _data()
    rng = np.random.RandomState(5)
    ws = [(rng.randn(12, 16) * .3).astype(np.float32), (rng.randn(16, 16) * .3).astype(np.float32),
          (rng.randn(16, 3) * .3).astype(np.float32)]
    layer_stage = {2: [0, 0, 1], 3: [0, 1, 2]}[nstages]
    hist = [[torch.tensor(w, dtype=torch.float64)] for w in ws]          # versions per layer
    bias = [[torch.zeros(w.shape[1], dtype=torch.float64)] for w in ws]
    mb = B // M
    for _ in range(steps):
        base = [len(h) - 1 for h in hist]                               # version at step start
        for b in range(M):
            params = []
            for li in range(3):
                warm = min(nstages - layer_stage[li] - 1, M)
                v = base[li] + max(0, b - warm)
                W = hist[li][v].clone().requires_grad_(True)
                c = bias[li][v].clone().requires_grad_(True)
                params.append((W, c))
            h = torch.tensor(X[b * mb:(b + 1) * mb], dtype=torch.float64)
            for li, (W, c) in enumerate(params):
                h = h @ W + c
                if li < 2:
                    h = torch.relu(h)
            y = torch.tensor(Y[b * mb:(b + 1) * mb], dtype=torch.float64)
            loss = -(y * torch.log_softmax(h, 1)).sum(1).mean()
            loss.backward()
            for li, (W, c) in enumerate(params):
                hist[li].append(hist[li][-1] - LR * W.grad)
                bias[li].append(bias[li][-1] - LR * c.grad)
    out = {}
    for li in range(3):
        out['w%d' % li] = hist[li][-1].numpy()
        out['b%d' % li] = bias[li][-1].numpy()
    return out


@pytest.mark.parametrize('nstages', [2, 3])
def test_pipedream_weight_stashing_matches_reference(nstages):
    """Asynchronous PipeDream: final weights equal the explicit weight-stash
    simulation, and the receiver host-synchronises on a shape header once per
    message edge per step -- not once per micro-batch."""
    steps = 2
    ref = _stash_reference(nstages, steps)
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, nstages, port, 'pipedream', nstages, q, steps))
          for r in range(nstages)]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for _, params, _, syncs, nrecv in res:
        merged.update(params)
        assert syncs == nrecv * steps, (syncs, nrecv)
    for k, v in ref.items():
        np.testing.assert_allclose(merged[k], v, rtol=1e-4, atol=1e-5, err_msg=k)


class _FifoComm(object):
    """in-process stand-in for the RCCL p2p group: sends queue tensors, recvs pop them"""

    def __init__(self, box):
        self.box = box

    def batch_p2p(self, ops):
        class _Done(object):
            def wait(self):
                return None
        for kind, t, peer in ops:
            if kind == 'send':
                self.box.append(t.clone())
            else:
                src = self.box.pop(0)
                assert src.shape == t.shape, 'payload recv posted with a stale shape'
                t.copy_(src)
        return [_Done() for _ in ops]


def test_p2p_shape_change_within_step():
    """a short last micro-batch: static mode refuses at the sender (instead of the
    receiver posting a stale-shape recv); dynamic mode carries a header per message"""
    import torch
    from hetu_61a7_amd.parallel.pipeline_exec import _P2P
    box = []
    snd, rcv = _P2P('cpu', _FifoComm(box)), _P2P('cpu', _FifoComm(box))
    a, b = torch.ones(4, 3), torch.full((2, 3), 2.0)
    snd.send_many([('act', a, 1)])
    assert torch.equal(rcv.recv_many([('act', 0)])[0], a)
    with pytest.raises(ValueError, match='changed shape'):
        snd.send_many([('act', b, 1)])
    box.clear()
    snd, rcv = _P2P('cpu', _FifoComm(box), dynamic=True), _P2P('cpu', _FifoComm(box), dynamic=True)
    for t in (a, b, a):
        snd.send_many([('act', t, 1)])
        assert torch.equal(rcv.recv_many([('act', 0)])[0], t)
    assert rcv.hdr_syncs == 3
