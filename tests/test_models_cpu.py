"""Model-zoo smoke tests on the CPU backend: each model builds, runs a few
training steps and its loss goes down (reference examples/rec/hetu_ncf.py,
examples/nlp/hetu_transformer.py)."""
import numpy as np

import hetu_61a7_amd as ht


def test_ncf_trains():
    from hetu_61a7_amd.models import neural_mf
    rng = np.random.RandomState(0)
    users = rng.randint(0, 50, 256)
    items = rng.randint(0, 80, 256)
    y = ((users + items) % 2).astype(np.float32).reshape(-1, 1)
    u, i, y_ = (ht.Variable(name=n, trainable=False) for n in ('u', 'i', 'y'))
    loss, _, train = neural_mf(u, i, y_, 50, 80, learning_rate=0.5)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=1)
    ls = [float(ex.run('train', feed_dict={u: users, i: items, y_: y}, convert_to_numpy_ret_vals=True)[0])
          for _ in range(40)]
    assert np.isfinite(ls).all() and ls[-1] < ls[0]


def test_transformer_trains():
    from hetu_61a7_amd.models.transformer import Transformer, TransformerConfig, synthetic_batch
    hp = TransformerConfig(vocab_size=64, d_model=32, d_ff=64, num_blocks=1, num_heads=4, maxlen1=8,
                           maxlen2=9, dropout_rate=0.0, batch_size=4)
    names = ('xs', 'src_mask', 'ys', 'tgt_mask', 'labels')
    ph = {n: ht.Variable(name=n, trainable=False) for n in names}
    loss, _ = Transformer(hp).train(*(ph[n] for n in names))
    train = ht.optim.AdamOptimizer(3e-3).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=2)
    b = synthetic_batch(hp)
    feed = {ph[n]: b[n] for n in names}
    ls = [float(ex.run('train', feed_dict=feed, convert_to_numpy_ret_vals=True)[0]) for _ in range(15)]
    assert np.isfinite(ls).all() and ls[-1] < 0.9 * ls[0]
