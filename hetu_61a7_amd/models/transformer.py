"""Encoder-decoder Transformer (reference examples/nlp/hetu_transformer.py,
hparams.py: d_model 512, d_ff 2048, 6 blocks, 8 heads, maxlen 100, dropout 0.3,
label smoothing 0.1; IWSLT de-en).

Same structure as the reference -- token embedding shared with the output
projection, sinusoidal positions, post-LN blocks, label-smoothed cross entropy
-- built from this framework's fused pieces: the QKV projections are one
``linear_op`` (bf16 MFMA GEMM with bias epilogue), attention is the single
``attention_op`` (padding mask as an additive [B, 1, 1, S] tensor, causal mask
inside the op), LayerNorm is the one-pass wave64 kernel.
"""
from __future__ import annotations

import numpy as np

from .. import initializers as init
from .. import ops as ht


class TransformerConfig(object):
    def __init__(self, vocab_size=32000, d_model=512, d_ff=2048, num_blocks=6, num_heads=8,
                 maxlen1=100, maxlen2=100, dropout_rate=0.3, smoothing=0.1, batch_size=32):
        self.vocab_size, self.d_model, self.d_ff = vocab_size, d_model, d_ff
        self.num_blocks, self.num_heads = num_blocks, num_heads
        self.maxlen1, self.maxlen2 = maxlen1, maxlen2
        self.dropout_rate, self.smoothing, self.batch_size = dropout_rate, smoothing, batch_size


def _dense(x, din, dout, name, act=None):
    w = init.xavier_normal((din, dout), name=name + '_weights')
    b = init.zeros((dout,), name=name + '_bias')
    return ht.linear_op(x, w, b, activation=act)


def _ln(x, d, name):
    return ht.layer_normalization_op(x, init.ones((d,), name=name + '_scale'),
                                     init.zeros((d,), name=name + '_bias'), eps=1e-8)


def _dropout(x, p):
    return ht.dropout_op(x, 1.0 - p) if p else x


def _positions(T, E):
    pe = np.array([[pos / np.power(10000, (i & -2) / E) for i in range(E)] for pos in range(T)])
    pe[:, 0::2] = np.sin(pe[:, 0::2])
    pe[:, 1::2] = np.cos(pe[:, 1::2])
    return pe.astype(np.float32)


class Transformer(object):
    def __init__(self, hp: TransformerConfig):
        self.hp = hp
        self.embeddings = init.xavier_normal((hp.vocab_size, hp.d_model), name='embedding_table')
        self._n = 0

    def _name(self, s):
        self._n += 1
        return '%s%d' % (s, self._n)

    def _mha(self, q_in, kv_in, Tq, Tk, mask, causal):
        hp = self.hp
        B, D, nh = hp.batch_size, hp.d_model, hp.num_heads
        hd = D // nh
        q2 = ht.array_reshape_op(q_in, (B * Tq, D))
        kv2 = ht.array_reshape_op(kv_in, (B * Tk, D))
        q = _dense(q2, D, D, self._name('q'))
        k = _dense(kv2, D, D, self._name('k'))
        v = _dense(kv2, D, D, self._name('v'))
        heads = lambda t, T: ht.transpose_op(ht.array_reshape_op(t, (B, T, nh, hd)), (0, 2, 1, 3))
        o = ht.attention_op(heads(q, Tq), heads(k, Tk), heads(v, Tk), mask, dropout=hp.dropout_rate,
                            causal=causal)
        o = ht.array_reshape_op(ht.transpose_op(o, (0, 2, 1, 3)), (B, Tq, D))
        return _ln(o + q_in, D, self._name('attn_ln'))

    def _ff(self, x, T):
        hp = self.hp
        B, D = hp.batch_size, hp.d_model
        h = ht.array_reshape_op(x, (B * T, D))
        h = _dense(h, D, hp.d_ff, self._name('ff1'), act='relu')
        h = ht.array_reshape_op(_dense(h, hp.d_ff, D, self._name('ff2')), (B, T, D))
        return _ln(h + x, D, self._name('ff_ln'))

    def _embed(self, ids, T):
        hp = self.hp
        e = ht.mul_byconst_op(ht.embedding_lookup_op(self.embeddings, ids), hp.d_model ** 0.5)
        pos = ht.Variable(name=self._name('position_enc'),
                          value=np.tile(_positions(T, hp.d_model), (hp.batch_size, 1, 1)), trainable=False)
        return _dropout(e + pos, hp.dropout_rate)

    @staticmethod
    def _additive(mask01, B, T):
        m = ht.array_reshape_op(mask01, (B, 1, 1, T))
        return ht.mul_byconst_op(ht.addbyconst_op(m, -1.0), 1e9)

    def encode(self, xs, src_mask):
        hp = self.hp
        T = hp.maxlen1
        m = self._additive(src_mask, hp.batch_size, T)
        enc = self._embed(xs, T)
        for _ in range(hp.num_blocks):
            enc = self._mha(enc, enc, T, T, m, False)
            enc = self._ff(enc, T)
        return enc, m

    def decode(self, ys, tgt_mask, memory, src_add):
        hp = self.hp
        T = hp.maxlen2 - 1
        m = self._additive(tgt_mask, hp.batch_size, T)
        dec = self._embed(ys, T)
        for _ in range(hp.num_blocks):
            dec = self._mha(dec, dec, T, T, m, True)
            dec = self._mha(dec, memory, T, hp.maxlen1, src_add, False)
            dec = self._ff(dec, T)
        dec = ht.array_reshape_op(dec, (hp.batch_size * T, hp.d_model))
        return ht.matmul_op(dec, self.embeddings, trans_B=True)  # tied output projection

    def train(self, xs, src_mask, ys, tgt_mask, labels):
        """labels: [B*(maxlen2-1)] int ids; returns (mean label-smoothed loss, logits)."""
        hp = self.hp
        memory, src_add = self.encode(xs, src_mask)
        logits = self.decode(ys, tgt_mask, memory, src_add)
        onehot = ht.one_hot_op(labels, hp.vocab_size)
        smooth = ht.addbyconst_op(ht.mul_byconst_op(onehot, 1.0 - hp.smoothing), hp.smoothing / hp.vocab_size)
        loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(logits, smooth), [0])
        return loss, logits


def synthetic_batch(hp: TransformerConfig, seed=0):
    rng = np.random.default_rng(seed)
    B, T1, T2 = hp.batch_size, hp.maxlen1, hp.maxlen2 - 1
    xs = rng.integers(4, hp.vocab_size, (B, T1)).astype(np.int64)
    ys = rng.integers(4, hp.vocab_size, (B, T2)).astype(np.int64)
    lx = rng.integers(T1 // 2, T1 + 1, B)
    ly = rng.integers(T2 // 2, T2 + 1, B)
    sm = (np.arange(T1)[None] < lx[:, None]).astype(np.float32)
    tm = (np.arange(T2)[None] < ly[:, None]).astype(np.float32)
    xs[sm == 0] = 0
    ys[tm == 0] = 0
    labels = np.roll(ys, -1, axis=1).reshape(-1)
    return dict(xs=xs, src_mask=sm, ys=ys, tgt_mask=tm, labels=labels)
