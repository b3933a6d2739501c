"""CTR models on Criteo-shaped data (reference ``examples/ctr/models/``:
``wdl_criteo.py:8-42``, ``deepfm_criteo.py``, ``dcn_criteo.py``, ``dc_criteo.py``,
``wdl_adult.py``) plus a synthetic Criteo source for the benchmark.

Criteo layout: 13 dense features, 26 categorical fields whose ids index one
shared embedding table of ``feature_dimension`` rows (33,762,577 for the full
Kaggle set).  On MI355X the whole 17.3 GB table fits in one GPU's HBM, so in
the AllReduce configuration the table is GPU-resident with row-sparse updates;
in PS / Hybrid modes it lives in the PS server's host DRAM behind the HET cache
(the reference's ``ctx=ht.cpu(0)`` placement).
"""
from __future__ import annotations

import numpy as np

from .. import init
from .. import ops as ht
from .. import optimizer as optim

CRITEO_ROWS = 33762577
N_DENSE, N_SPARSE = 13, 26


def _embedding(name, rows, width, stddev=0.01):
    return init.random_normal([rows, width], stddev=stddev, name=name)


def wdl_criteo(dense_input, sparse_input, y_, feature_dimension=CRITEO_ROWS, embedding_size=128,
               learning_rate=0.01, optimizer=None):
    E = _embedding('snd_order_embedding', feature_dimension, embedding_size)
    sp = ht.embedding_lookup_op(E, sparse_input)
    sp = ht.array_reshape_op(sp, (-1, N_SPARSE * embedding_size))
    W1 = init.random_normal([N_DENSE, 256], stddev=0.01, name='W1')
    W2 = init.random_normal([256, 256], stddev=0.01, name='W2')
    W3 = init.random_normal([256, 256], stddev=0.01, name='W3')
    W4 = init.random_normal([256 + N_SPARSE * embedding_size, 1], stddev=0.01, name='W4')
    r1 = ht.relu_op(ht.matmul_op(dense_input, W1))
    r2 = ht.relu_op(ht.matmul_op(r1, W2))
    y3 = ht.matmul_op(r2, W3)
    y4 = ht.concat_op(sp, y3, axis=1)
    y = ht.sigmoid_op(ht.matmul_op(y4, W4))
    loss = ht.reduce_mean_op(ht.binarycrossentropy_op(y, y_), [0])
    opt = optimizer or optim.SGDOptimizer(learning_rate=learning_rate)
    return loss, y, y_, opt.minimize(loss)


def dfm_criteo(dense_input, sparse_input, y_, feature_dimension=CRITEO_ROWS, embedding_size=128,
               learning_rate=0.01, optimizer=None):
    E1 = _embedding('fst_order_embedding', feature_dimension, 1)
    FM_W = init.random_normal([N_DENSE, 1], stddev=0.01, name='dense_parameter')
    sp1 = ht.embedding_lookup_op(E1, sparse_input)
    y1 = ht.matmul_op(dense_input, FM_W) + ht.reduce_sum_op(sp1, axes=1)
    E2 = _embedding('snd_order_embedding', feature_dimension, embedding_size)
    sp2 = ht.embedding_lookup_op(E2, sparse_input)
    s = ht.reduce_sum_op(sp2, axes=1)
    sum_sq = ht.mul_op(s, s)
    sq_sum = ht.reduce_sum_op(ht.mul_op(sp2, sp2), axes=1)
    y2 = ht.reduce_sum_op((sum_sq + -1 * sq_sum) * 0.5, axes=1, keepdims=True)
    flat = ht.array_reshape_op(sp2, (-1, N_SPARSE * embedding_size))
    W1 = init.random_normal([N_SPARSE * embedding_size, 256], stddev=0.01, name='W1')
    W2 = init.random_normal([256, 256], stddev=0.01, name='W2')
    W3 = init.random_normal([256, 1], stddev=0.01, name='W3')
    r1 = ht.relu_op(ht.matmul_op(flat, W1))
    r2 = ht.relu_op(ht.matmul_op(r1, W2))
    y3 = ht.matmul_op(r2, W3)
    y = ht.sigmoid_op(y1 + y2 + y3)
    loss = ht.reduce_mean_op(ht.binarycrossentropy_op(y, y_), [0])
    opt = optimizer or optim.SGDOptimizer(learning_rate=learning_rate)
    return loss, y, y_, opt.minimize(loss)


def _cross_layer(x0, x1, width):
    w = init.random_normal(shape=(width, 1), stddev=0.01, name='weight')
    b = init.random_normal(shape=(width,), stddev=0.01, name='bias')
    x1w = ht.matmul_op(x1, w)
    y = ht.mul_op(x0, ht.broadcastto_op(x1w, x0))
    return y + x1 + ht.broadcastto_op(b, y)


def dcn_criteo(dense_input, sparse_input, y_, feature_dimension=CRITEO_ROWS, embedding_size=128,
               learning_rate=0.003, num_cross=3, optimizer=None):
    E = _embedding('snd_order_embedding', feature_dimension, embedding_size)
    sp = ht.array_reshape_op(ht.embedding_lookup_op(E, sparse_input), (-1, N_SPARSE * embedding_size))
    x = ht.concat_op(sp, dense_input, axis=1)
    width = N_SPARSE * embedding_size + N_DENSE
    c = x
    for _ in range(num_cross):
        c = _cross_layer(x, c, width)
    W1 = init.random_normal([width, 256], stddev=0.01, name='W1')
    W2 = init.random_normal([256, 256], stddev=0.01, name='W2')
    W3 = init.random_normal([256, 256], stddev=0.01, name='W3')
    W4 = init.random_normal([256 + width, 1], stddev=0.01, name='W4')
    r1 = ht.relu_op(ht.matmul_op(x, W1))
    r2 = ht.relu_op(ht.matmul_op(r1, W2))
    y3 = ht.matmul_op(r2, W3)
    y = ht.sigmoid_op(ht.matmul_op(ht.concat_op(c, y3, axis=1), W4))
    loss = ht.reduce_mean_op(ht.binarycrossentropy_op(y, y_), [0])
    opt = optimizer or optim.SGDOptimizer(learning_rate=learning_rate)
    return loss, y, y_, opt.minimize(loss)


def _residual_layer(x0, input_dim, hidden_dim):
    w1 = init.random_normal(shape=(input_dim, hidden_dim), stddev=0.1, name='weight_1')
    b1 = init.random_normal(shape=(hidden_dim,), stddev=0.1, name='bias_1')
    w2 = init.random_normal(shape=(hidden_dim, input_dim), stddev=0.1, name='weight_2')
    b2 = init.random_normal(shape=(input_dim,), stddev=0.1, name='bias_2')
    h = ht.matmul_op(x0, w1)
    h = ht.relu_op(h + ht.broadcastto_op(b1, h))
    o = ht.matmul_op(h, w2)
    o = o + ht.broadcastto_op(b2, o)
    return ht.relu_op(o + x0)


def dc_criteo(dense_input, sparse_input, y_, feature_dimension=CRITEO_ROWS, embedding_size=8,
              learning_rate=0.001, num_layers=5, optimizer=None):
    E = _embedding('snd_order_embedding', feature_dimension, embedding_size)
    sp = ht.array_reshape_op(ht.embedding_lookup_op(E, sparse_input), (-1, N_SPARSE * embedding_size))
    x = ht.concat_op(sp, dense_input, axis=1)
    d = N_SPARSE * embedding_size + N_DENSE
    for _ in range(num_layers):
        x = _residual_layer(x, d, d)
    W4 = init.random_normal([d, 1], stddev=0.1, name='W4')
    y = ht.sigmoid_op(ht.matmul_op(x, W4))
    loss = ht.reduce_mean_op(ht.binarycrossentropy_op(y, y_), [0])
    opt = optimizer or optim.SGDOptimizer(learning_rate=learning_rate)
    return loss, y, y_, opt.minimize(loss)


def wdl_adult(X_deep, X_wide, y_, dim_wide=809, lr=5 / 128):
    """Adult census Wide&Deep: 8 categorical fields (8-wide embeddings of 50
    rows) + 4 continuous fields, wide part concatenated before the output."""
    W = init.random_normal([dim_wide + 20, 2], stddev=0.1, name='W')
    W1 = init.random_normal([68, 50], stddev=0.1, name='W1')
    b1 = init.random_normal([50], stddev=0.1, name='b1')
    W2 = init.random_normal([50, 20], stddev=0.1, name='W2')
    b2 = init.random_normal([20], stddev=0.1, name='b2')
    deep = None
    for i in range(8):
        E = init.random_normal([50, 8], stddev=0.1, name='Embedding_deep_%d' % i)
        now = ht.array_reshape_op(ht.embedding_lookup_op(E, X_deep[i]), (-1, 8))
        deep = now if deep is None else ht.concat_op(deep, now, 1)
    for i in range(4):
        deep = ht.concat_op(deep, ht.array_reshape_op(X_deep[i + 8], (-1, 1)), 1)
    m1 = ht.matmul_op(deep, W1)
    h1 = ht.relu_op(m1 + ht.broadcastto_op(b1, m1))
    m2 = ht.matmul_op(h1, W2)
    h2 = ht.relu_op(m2 + ht.broadcastto_op(b2, m2))
    pred = ht.matmul_op(ht.concat_op(X_wide, h2, 1), W)
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(pred, y_), [0])
    train_op = optim.SGDOptimizer(learning_rate=lr).minimize(loss)
    return loss, pred, y_, train_op


CTR_MODELS = {'wdl': wdl_criteo, 'wdl_criteo': wdl_criteo, 'dfm': dfm_criteo, 'deepfm': dfm_criteo,
              'dcn': dcn_criteo, 'dc': dc_criteo}


def synthetic_criteo(n, feature_dimension=CRITEO_ROWS, seed=0, zipf=1.05):
    """Criteo-shaped synthetic batch source: dense ~ N(0,1) [n,13], sparse ids
    [n,26] drawn per field from a Zipf-like distribution over disjoint id ranges
    (the skew is what makes the HET cache effective), labels in {0,1}."""
    rng = np.random.default_rng(seed)
    dense = rng.standard_normal((n, N_DENSE)).astype(np.float32)
    per = feature_dimension // N_SPARSE
    ranks = rng.zipf(zipf + 1e-9, size=(n, N_SPARSE)) if zipf > 1 else rng.integers(1, per, (n, N_SPARSE))
    ranks = np.minimum(ranks - 1, per - 1)
    offs = (np.arange(N_SPARSE, dtype=np.int64) * per)[None, :]
    sparse = (offs + ranks).astype(np.int64)
    labels = (rng.random((n, 1)) < 0.25).astype(np.float32)
    return dense, sparse, labels


def wdl_criteo_bench(args, world, rank, local):
    """Benchmark step for the BASELINE Wide&Deep-Criteo configuration: full
    33.76M x 128 embedding on the PS (host DRAM) behind an LFUOpt HET cache with
    bound 3 (reference examples/ctr/tests/hybrid_wdl_criteo.sh), dense MLP on
    the GPU (RCCL all-reduce when world > 1), SGD lr 0.01, per-worker batch 128.
    Returns (step_fn, samples_per_step, config, metric, finish_fn)."""
    import torch
    import hetu_61a7_amd as ht
    rows = int(getattr(args, 'criteo_rows', 0) or CRITEO_ROWS)
    B = args.batch or 128
    nb = 64
    # id distribution: Zipf a=1.05 per field (the skew real CTR data has), or a uniform
    # control run (``--ids uniform``: every lookup is a cold row -- the cache's worst case)
    dist = getattr(args, 'ids', 'zipf')
    # rehearsal knobs (tests/test_rehearse8_cpu.py): CPU context, BSP, every worker on the
    # same batches, no cache, another lr / embedding width
    cpu = bool(getattr(args, 'rehearse_cpu', False))
    same = bool(getattr(args, 'same_data', False))
    emb = int(getattr(args, 'emb', 0) or 128)
    lr = float(getattr(args, 'lr', 0) or 0.01)
    bsp = int(getattr(args, 'bsp', -1))
    import numpy as np
    inter = int(getattr(args, 'interleave_workers', 0) or 0)
    if same:
        dense, sparse, labels = synthetic_criteo(B * nb, rows, seed=100, zipf=1.05 if dist == 'zipf' else 0)
        if world > 1:
            # the dataloader shards its data over the workers (contiguous 1/world slices): tile
            # the block so that every worker's shard -- and so every batch -- is the same
            dense, sparse, labels = (np.concatenate([a] * world, 0) for a in (dense, sparse, labels))
    elif inter > 1:
        # the single-worker reference of a ``inter``-worker job (rehearsal): the same global
        # data, reordered so that this worker's batch j (of inter x the per-worker batch) is
        # the concatenation of every worker's batch j
        b0 = B // inter
        dense, sparse, labels = synthetic_criteo(b0 * nb * inter, rows, seed=100, zipf=1.05 if dist == 'zipf' else 0)
        S = b0 * nb
        order = np.concatenate([np.arange(r * S + j * b0, r * S + (j + 1) * b0)
                                for j in range(nb) for r in range(inter)])
        dense, sparse, labels = dense[order], sparse[order], labels[order]
    else:
        # one global data set (identical on every worker) that the dataloader shards: every
        # worker reads distinct ids, as the reference's run_hetu.py workers read their shard
        dense, sparse, labels = synthetic_criteo(B * nb * world, rows, seed=100, zipf=1.05 if dist == 'zipf' else 0)
    # dataloader-fed inputs, as the reference's run_hetu.py: the executor knows the
    # next batch's sparse ids and prefetches their rows with this step's push
    xd = ht.dataloader_op([ht.Dataloader(dense, B, 'train')])
    xs = ht.dataloader_op([ht.Dataloader(sparse, B, 'train')])
    y_ = ht.dataloader_op([ht.Dataloader(labels, B, 'train')])
    loss, y, _, train = wdl_criteo(xd, xs, y_, feature_dimension=rows, embedding_size=emb, learning_rate=lr)
    # comm mode: 'PS' (BASELINE config 3, reference examples/ctr/tests/ps_wdl_criteo.sh: the
    # dense MLP parameters live on the server too, pushed and pulled every step) or
    # 'Hybrid' (dense parameters all-reduced on the GPUs, embeddings on the PS)
    comm = getattr(args, 'comm', None) or 'PS'
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0) if cpu else ht.gpu(local), comm_mode=comm,
                     cstable_policy=getattr(args, 'cache', 'LFUOpt'), cache_bound=3, bsp=bsp,
                     mixed_precision=None if cpu else args.dtype, seed=1234,
                     prefetch=getattr(args, 'prefetch', True) and bsp < 0)
    from ..ps import table as _pst
    clock = {'wall': [], 'wait': []}

    losses = []

    def step():
        import time
        t0, w0 = time.perf_counter(), _pst.WAIT_S[0]
        r = ex.run('train')
        if cpu:
            losses.append(float(r[0].asnumpy().reshape(-1)[0]) if hasattr(r[0], 'asnumpy') else float(r[0]))
        clock['wall'].append(time.perf_counter() - t0)
        clock['wait'].append(_pst.WAIT_S[0] - w0)

    tables = [t for t in ex.config.placeholder_to_arr_map.values() if getattr(t, 'cache', None) is not None]
    for t in tables:
        t.cache.perf_enabled = True

    def extra():
        """HET cache statistics over every step so far (warm-up included)"""
        tot = {}
        for t in tables:
            for k, v in t.cache.perf.items():
                tot[k] = tot.get(k, 0) + v
        unique, miss = tot.get('unique', 0), tot.get('miss', 0)
        k = max(1, min(int(getattr(args, 'steps', 0) or 0) or len(clock['wall']), len(clock['wall'])))
        wall, wait = sum(clock['wall'][-k:]), sum(clock['wait'][-k:])
        return {'ids': dist, 'cache_lookups_unique': int(unique), 'cache_misses': int(miss),
                'cache_hit_rate': round(1.0 - miss / unique, 4) if unique else None,
                'prefetch_hits': int(sum(t.prefetch_hits for t in tables)),
                # host-side step breakdown over the timed steps: the time run() blocked on
                # PS / cache tickets and staging copies, and the rest (graph walk, kernel
                # launches, host work of the lookups / pushes); run() returns before the
                # GPU finishes, so 'wall' can sit below the bench's synchronised ms_per_step
                'step_breakdown_ms': {'wall': round(wall * 1e3 / k, 3),
                                      'ps_wait': round(wait * 1e3 / k, 3),
                                      'host_other': round((wall - wait) * 1e3 / k, 3)}}
    step.extra = extra
    step.losses = losses
    step.executor = ex

    def finish():
        from ..ps import worker
        for op in ex.subexecutor['train'].opt_ops:
            if getattr(op, 'ps_dense', None) is not None:
                op.ps_dense.drain()
        ex.config.ps_comm.BarrierWorker()
        worker.worker_finish()

    par = ('ps: dense + embeddings on PS (1 server) + HET cache lfuopt/3, %d worker(s)' % world if comm == 'PS'
           else 'hybrid: PS(1 server)+HET cache lfuopt/3 + dp%d' % world)
    cfg = {'model': 'Wide&Deep (Criteo-shaped, %d x 128 embedding)' % rows, 'global_batch': B * world,
           'seq_len': None, 'parallelism': par, 'comm_mode': comm,
           'optimizer': 'sgd', 'per_gpu_batch': B}
    return step, B * world, cfg, 'samples/sec (whole node) Wide&Deep-Criteo PS + HET cache', finish
