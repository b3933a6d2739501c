"""Neural collaborative filtering (reference examples/rec/hetu_ncf.py; MovieLens).

GMF + MLP towers over one user table and one item table whose rows hold both
the GMF factors (first ``embed_dim``) and the MLP half-input; SGD lr 0.01,
sigmoid + BCE.  The embedding tables are the row-sparse parameters that the
PS / Hybrid modes place on the parameter server (``examples/rec/ps_ncf.sh``,
``hybrid_ncf.sh``).
"""
from __future__ import annotations

from .. import initializers as init
from .. import ops as ht
from .. import optimizer as optim


def neural_mf(user_input, item_input, y_, num_users, num_items, embed_dim=8,
              layers=(64, 32, 16, 8), learning_rate=0.01):
    width = embed_dim + layers[0] // 2
    user_emb = init.random_normal((num_users, width), stddev=0.01, name='user_embed')
    item_emb = init.random_normal((num_items, width), stddev=0.01, name='item_embed')
    user_latent = ht.embedding_lookup_op(user_emb, user_input)
    item_latent = ht.embedding_lookup_op(item_emb, item_input)
    mf_user = ht.slice_op(user_latent, (0, 0), (-1, embed_dim))
    mlp_user = ht.slice_op(user_latent, (0, embed_dim), (-1, -1))
    mf_item = ht.slice_op(item_latent, (0, 0), (-1, embed_dim))
    mlp_item = ht.slice_op(item_latent, (0, embed_dim), (-1, -1))
    W1 = init.random_normal((layers[0], layers[1]), stddev=0.1, name='W1')
    W2 = init.random_normal((layers[1], layers[2]), stddev=0.1, name='W2')
    W3 = init.random_normal((layers[2], layers[3]), stddev=0.1, name='W3')
    W4 = init.random_normal((embed_dim + layers[3], 1), stddev=0.1, name='W4')
    mf_vector = ht.mul_op(mf_user, mf_item)
    h = ht.concat_op(mlp_user, mlp_item, axis=1)
    h = ht.relu_op(ht.matmul_op(h, W1))
    h = ht.relu_op(ht.matmul_op(h, W2))
    h = ht.relu_op(ht.matmul_op(h, W3))
    y = ht.sigmoid_op(ht.matmul_op(ht.concat_op(mf_vector, h, axis=1), W4))
    loss = ht.reduce_mean_op(ht.binarycrossentropy_op(y, y_), [0])
    train_op = optim.SGDOptimizer(learning_rate=learning_rate).minimize(loss)
    return loss, y, train_op
