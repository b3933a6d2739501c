"""Eight-rank rehearsals (gloo, CPU) of the bench entry points the driver runs on an
8-GPU node (reference examples/runner/parallel/all_mlp_tests.sh:14-30 checks every
parallel layout against the single-process losses, validate_results.py:11-18):

* ResNet-50 data parallel over 8 ranks (bench.py's default model and its exact
  Executor call): with the same batch on every rank, SUM all-reduce and lr / 8 give the
  single-process update, so losses and weights match one process;
* BERT with a forced Galvatron plan of 2 pipeline stages x 4 data-parallel replicas
  (bench.py --model bert --pp 2): the replicas slice one global batch, so the weights
  match one process training on that global batch;
* MoE top-2 with expert parallelism over 8 ranks (2 experts per rank, all-to-all).

Every rank runs one thread; shapes are tiny."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

WORLD = 8


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(target, world, *args, timeout=420):
    port = _port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    import queue
    import time
    res, t0 = [], time.time()
    while len(res) < len(ps):
        try:
            res.append(q.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
            assert not dead, 'a rank died: exit codes %s' % dead
            assert time.time() - t0 < timeout, 'rehearsal timed out'
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    return sorted(res, key=lambda t: t[0])


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port), HETU_USE_CONFIG='0', OMP_NUM_THREADS='1')
    import torch
    torch.set_num_threads(1)


def _resnet_worker(rank, world, port, q):
    _env(rank, world, port)
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models import resnet50_imagenet
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    loss, _ = resnet50_imagenet(x, y_, 10)
    # bench.py: MomentumOptimizer(0.1 / world), DataParallel('allreduce') when world > 1
    train = ht.optim.MomentumOptimizer(learning_rate=0.1 / world, momentum=0.9).minimize(loss)
    kw = dict(bucket_mb=4, seed=1234)
    if world > 1:
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
    else:
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), **kw)
    rng = np.random.RandomState(7)                 # the same batch on every rank
    X = rng.randn(1, 3, 224, 224).astype(np.float32)
    Y = np.eye(10, dtype=np.float32)[rng.randint(0, 10, 1)]
    losses = [float(np.asarray(ex.run('train', feed_dict={x: X, y_: Y}, convert_to_numpy_ret_vals=True)[0])
                    .reshape(-1)[0]) for _ in range(3)]
    params = {n.name: v.detach().numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items()
              if n.trainable and ('fc' in n.name or n.name.startswith('stem'))}
    info = {}
    if world > 1:
        from hetu_61a7_amd.parallel import comm
        info = comm.stats()
        info['buckets'] = len(train.buckets)
        comm.destroy()
    q.put((rank, losses, params, info))


def test_resnet50_dp8_matches_single_process():
    ref = _run(_resnet_worker, 1)[0]
    res = _run(_resnet_worker, WORLD)
    for rank, losses, params, info in res:
        assert info['world'] == WORLD and info['buckets'] > 1
        np.testing.assert_allclose(losses, ref[1], rtol=2e-4, atol=1e-5, err_msg='rank %d' % rank)
        for k, v in ref[2].items():
            np.testing.assert_allclose(params[k], v, rtol=2e-4, atol=2e-6, err_msg='%s rank %d' % (k, rank))
    for _, _, p, _ in res[1:]:                                         # replicas bitwise identical
        for k in p:
            np.testing.assert_array_equal(p[k], res[0][2][k])


def _bert_worker(rank, world, port, q, pp, batch):
    _env(rank, world, port)
    import types
    from hetu_61a7_amd.models.bert import BertConfig, bert_bench
    cfg = BertConfig(vocab_size=256, hidden_size=32, num_hidden_layers=4, num_attention_heads=2,
                     intermediate_size=64, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                     max_position_embeddings=16, seq_len=16, batch_size=batch)
    # SGD: the pipeline sums its micro-batch gradients and the replicas SUM-all-reduce, so
    # the update is world x the mean gradient: lr / world reproduces one process on the
    # global batch (the reference scales lr by 1/N the same way)
    args = types.SimpleNamespace(batch=batch, dtype='fp32', bucket_mb=1, zero=0, pp=pp, bert_config=cfg,
                                 optimizer='sgd', lr=0.5 / world)
    step, samples, conf, _, _ = bert_bench(args, world, rank, rank)
    for _ in range(2):
        step()
    ex = step.executor
    params = {n.name: v.detach().numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items()
              if getattr(n, 'trainable', False) and hasattr(v, 'detach')}
    if world > 1:
        from hetu_61a7_amd.parallel import comm
        comm.destroy()
    q.put((rank, conf, samples, params))


def test_bert_pp2_dp4_plan_matches_single_process():
    ref = _run(_bert_worker, 1, None, 8)[0]
    res = _run(_bert_worker, WORLD, 2, 1)
    assert res[0][1]['plan']['pp'] == 2 and res[0][1]['parallelism'].startswith('pp2 x dp4')
    assert res[0][2] == ref[2] == 8                                  # global batch 1 x 8 GPUs
    merged = {}
    for _, _, _, params in res:
        for k, v in params.items():
            if k in merged:                                          # data-parallel replicas agree
                np.testing.assert_allclose(v, merged[k], rtol=1e-5, atol=1e-7, err_msg=k)
            else:
                merged[k] = v
    merged.pop('cls_decoder_weight', None)                           # the last stage's tied copy
    assert set(merged) == set(ref[3])
    for k, v in ref[3].items():
        np.testing.assert_allclose(merged[k], v, rtol=2e-3, atol=2e-5, err_msg=k)


def _moe_worker(rank, world, port, q):
    _env(rank, world, port)
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.layers.moe import TopKGate, Expert, MoELayer
    T, d, n_local = 16, 8, 2
    E = n_local * world
    X = np.random.RandomState(100 + rank).randn(T, d).astype(np.float32)
    x = ht.Variable(name='x')
    experts = [Expert(d, 16, activation='relu', name='expert_%d' % (rank * n_local + i)) for i in range(n_local)]
    y, l_aux = MoELayer(TopKGate(d, T, E, k=2, capacity_factor=float(E)), experts, T, d, all2all_size=world)(x)
    loss = ht.add_op(ht.reduce_mean_op(ht.mul_op(y, y), [0, 1]), ht.mul_byconst_op(l_aux, 0.01))
    train = ht.optim.SGDOptimizer(0.05).minimize(loss)
    ex = ht.Executor({'train': [loss, y, train]}, comm_mode='AllReduce')
    outs = [float(np.asarray(ex.run('train', feed_dict={x: X}, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
            for _ in range(4)]
    gate = {n.name: v.detach().numpy().copy() for n, v in ex.config.placeholder_to_arr_map.items()
            if n.trainable and 'expert' not in n.name}
    from hetu_61a7_amd.parallel import comm
    comm.destroy()
    q.put((rank, outs, gate))


def test_moe_expert_parallel_eight_ranks():
    res = _run(_moe_worker, WORLD)
    for rank, outs, _ in res:
        assert np.isfinite(outs).all() and outs[-1] < outs[0], (rank, outs)
    for _, _, g in res[1:]:                                          # the data-parallel gate agrees
        for k in g:
            np.testing.assert_allclose(g[k], res[0][2][k], rtol=1e-6, atol=1e-7)
