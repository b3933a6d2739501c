"""BERT (reference ``examples/nlp/bert/hetu_bert.py``, config ``bert_config.py``).

Same architecture and parameter naming scheme as the reference (embeddings
word/position/token-type + LayerNorm, N x [self-attention, add&LN, GELU FFN,
add&LN], tanh pooler, MLM head tied to the word embedding, NSP head), written
MI355X-first:

* hidden states stay 2-D ``[B*S, H]`` between layers, so every projection is one
  plain bf16 GEMM with the bias (and GELU) fused in the epilogue
  (``linear_op(..., activation='gelu')``) instead of reshape->matmul->broadcast-add;
* Q, K and V come from ONE fused [H, 3H] projection;
* attention is the single ``attention_op`` (QK^T/PV on the MFMA batched GEMM,
  masked softmax + recompute-dropout kernels);
* the pretraining losses are sparse-label softmax-CE (one wave64 kernel, ignore
  index -1) rather than softmax followed by cross-entropy.
"""
from __future__ import annotations

import contextlib

import numpy as np

from .. import init
from .. import ops as ht
from .. import optimizer as optim
from ..context import context as _context


def _stage_ctx(placement, layer):
    """Context of planner layer ``layer`` (0 = embeddings, 1..L = encoder
    layers, L+1 = heads) under ``placement`` (a callable layer -> device group),
    or a no-op when the model is not pipelined."""
    if placement is None:
        return contextlib.nullcontext()
    return _context(placement(layer))


class BertConfig(object):
    def __init__(self, vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act='gelu', hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02, batch_size=64, seq_len=128, fused_attention=True, vocab_multiple=64,
                 max_predictions_per_seq=None):
        self.vocab_size = vocab_size
        # max_predictions_per_seq (the original BERT's data contract: at most this many
        # labelled positions per sequence): the MLM head runs over the labelled rows only,
        # compacted into that many slots per sequence (ops/mlm.py) -- same loss and
        # gradients; None scores every position as the reference does
        self.max_predictions_per_seq = max_predictions_per_seq
        # the word-embedding table / MLM decoder are padded to a multiple of vocab_multiple
        # rows (Megatron's make-vocab-size-divisible-by): 30522 -> 30528 keeps every MLM-head
        # GEMM leading dimension a multiple of the MFMA loaders' 16-byte chunks.  The pad
        # columns carry a -1e4 decoder bias, so their softmax weight is exactly 0 in fp32:
        # the loss, the gradients of the real rows and the pad rows' zero gradient are those
        # of the unpadded model.  vocab_multiple=1 disables it.
        self.vocab_multiple = max(1, int(vocab_multiple))
        self.fused_attention = fused_attention   # packed-QKV HIP attention (else op-by-op graph)
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.intermediate_size = intermediate_size
        self.hidden_act = hidden_act
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.initializer_range = initializer_range
        self.batch_size = batch_size
        self.seq_len = seq_len

    @property
    def padded_vocab_size(self):
        m = self.vocab_multiple
        return -(-self.vocab_size // m) * m

    @classmethod
    def base(cls, **kw):
        return cls(**kw)

    @classmethod
    def large(cls, **kw):
        d = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)
        d.update(kw)
        return cls(**d)


def _w(name, shape, cfg):
    return init.truncated_normal(shape, stddev=cfg.initializer_range, name=name)


def _zeros(name, n):
    return init.zeros((n,), name=name)


def _ones(name, n):
    return init.ones((n,), name=name)


def _dense(x, din, dout, name, cfg, act=None):
    W = _w(name + '_weight', (din, dout), cfg)
    b = _zeros(name + '_bias', dout)
    return ht.linear_op(x, W, b, activation=act)


def _ln(x, h, name):
    return ht.layer_normalization_op(x, _ones(name + '_scale', h), _zeros(name + '_bias', h), eps=1e-12)


def _drop_add_ln(x, res, h, name, p):
    """LN(dropout(x) + res) as one fused kernel each way."""
    return ht.dropout_add_layernorm_op(x, res, _ones(name + '_scale', h), _zeros(name + '_bias', h),
                                       keep_prob=1.0 - p, eps=1e-12)


def _dropout(x, p):
    return ht.dropout_op(x, 1.0 - p) if p > 0 else x


class BertLayer(object):
    def __init__(self, cfg, idx):
        self.cfg, self.idx = cfg, idx

    def __call__(self, h2d, mask):
        c = self.cfg
        B, S, H = c.batch_size, c.seq_len, c.hidden_size
        nh, hd = c.num_attention_heads, H // c.num_attention_heads
        p = 'layer%d_' % self.idx
        qkv = _dense(h2d, H, 3 * H, p + 'attention_qkv', c)                  # [B*S, 3H]
        if c.fused_attention:
            # one HIP kernel each way straight off the packed projection
            ctxl = ht.packed_attention_op(qkv, mask, B, S, nh, dropout=c.attention_probs_dropout_prob)
            a = _dense(ctxl, H, H, p + 'attention_output', c)
            a = _drop_add_ln(a, h2d, H, p + 'attention_LayerNorm', c.hidden_dropout_prob)
            f = _dense(a, H, c.intermediate_size, p + 'intermediate', c, act=c.hidden_act)
            f = _dense(f, c.intermediate_size, H, p + 'output', c)
            return _drop_add_ln(f, a, H, p + 'output_LayerNorm', c.hidden_dropout_prob)
        mask = ht.array_reshape_op(mask, (B, 1, 1, S))
        qkv = ht.array_reshape_op(qkv, (B, S, 3, nh, hd))
        qkv = ht.transpose_op(qkv, (2, 0, 3, 1, 4))                           # [3, B, nh, S, hd]
        q = ht.slice_op(qkv, (0, 0, 0, 0, 0), (1, B, nh, S, hd))
        k = ht.slice_op(qkv, (1, 0, 0, 0, 0), (1, B, nh, S, hd))
        v = ht.slice_op(qkv, (2, 0, 0, 0, 0), (1, B, nh, S, hd))
        q, k, v = [ht.array_reshape_op(t, (B, nh, S, hd)) for t in (q, k, v)]
        ctxl = ht.attention_op(q, k, v, mask, dropout=c.attention_probs_dropout_prob)
        ctxl = ht.array_reshape_op(ht.transpose_op(ctxl, (0, 2, 1, 3)), (B * S, H))
        a = _dense(ctxl, H, H, p + 'attention_output', c)
        a = _drop_add_ln(a, h2d, H, p + 'attention_LayerNorm', c.hidden_dropout_prob)
        f = _dense(a, H, c.intermediate_size, p + 'intermediate', c, act=c.hidden_act)
        f = _dense(f, c.intermediate_size, H, p + 'output', c)
        return _drop_add_ln(f, a, H, p + 'output_LayerNorm', c.hidden_dropout_prob)


class BertModel(object):
    def __init__(self, cfg: BertConfig, placement=None):
        self.cfg = cfg
        self.placement = placement
        H = cfg.hidden_size
        with _stage_ctx(placement, 0):
            self.word_embeddings = _w('word_embeddings', (cfg.padded_vocab_size, H), cfg)
            self.position_embeddings = _w('position_embeddings', (cfg.max_position_embeddings, H), cfg)
            self.token_type_embeddings = _w('token_type_embeddings', (cfg.type_vocab_size, H), cfg)
        self.layers = [BertLayer(cfg, i) for i in range(cfg.num_hidden_layers)]

    def __call__(self, input_ids, token_type_ids, attention_mask):
        """input_ids / token_type_ids: [B, S] ints; attention_mask: [B, S] of {0,1}.
        Returns (sequence_output [B*S, H], pooled_output [B, H])."""
        c = self.cfg
        B, S, H = c.batch_size, c.seq_len, c.hidden_size
        pl = self.placement
        with _stage_ctx(pl, 0):
            pos = ht.Variable('position_ids', value=np.tile(np.arange(S, dtype=np.int64), (B, 1)),
                              trainable=False)
            e = ht.embedding_lookup_op(self.word_embeddings, input_ids) + \
                ht.embedding_lookup_op(self.position_embeddings, pos) + \
                ht.embedding_lookup_op(self.token_type_embeddings, token_type_ids)
            e = ht.array_reshape_op(e, (B * S, H))
            h = _dropout(_ln(e, H, 'embeddings_LayerNorm'), c.hidden_dropout_prob)
        for i, layer in enumerate(self.layers):
            with _stage_ctx(pl, i + 1):
                # additive key mask [B, S]: 0 keep, -10000 masked (built on
                # every stage from the fed mask, so it never crosses a stage boundary)
                if i == 0:
                    m = ht.array_reshape_op(attention_mask, (B, S))
                    m = ht.mul_byconst_op(ht.addbyconst_op(m, -1.0), 10000.0)
                elif pl is not None and pl(i + 1) != pl(i):
                    from ..ops.node import shadow_ids
                    with shadow_ids():
                        m = ht.array_reshape_op(attention_mask, (B, S))
                        m = ht.mul_byconst_op(ht.addbyconst_op(m, -1.0), 10000.0)
                h = layer(h, m)
        with _stage_ctx(pl, len(self.layers) + 1):
            first = ht.array_reshape_op(ht.slice_op(ht.array_reshape_op(h, (B, S, H)), (0, 0, 0), (B, 1, H)),
                                        (B, H))
            pooled = ht.tanh_op(_dense(first, H, H, 'pooler_dense', c))
        return h, pooled


class BertPreTrainingHeads(object):
    def __init__(self, cfg, word_embeddings):
        self.cfg, self.E = cfg, word_embeddings

    def __call__(self, seq, pooled):
        c = self.cfg
        H = c.hidden_size
        t = _dense(seq, H, H, 'cls_transform_dense', c, act=c.hidden_act)
        t = _ln(t, H, 'cls_transform_LayerNorm')
        V, Vp = c.vocab_size, c.padded_vocab_size
        if Vp == V:
            bias = _zeros('cls_lm_bias', V)
        else:
            bias = ht.Variable('cls_lm_bias', value=np.concatenate([np.zeros(V, np.float32),
                                                                    np.full(Vp - V, -1e4, np.float32)]))
        scores = ht.linear_op(t, self.E, bias, trans_B=True)            # tied decoder: [B*S, V]
        nsp = _dense(pooled, H, 2, 'cls_seq_relationship', c)
        return scores, nsp


class BertForPreTraining(object):
    def __init__(self, cfg, placement=None):
        self.cfg = cfg
        self.placement = placement
        self.bert = BertModel(cfg, placement)
        head = len(self.bert.layers) + 1
        if placement is not None and placement(head) != placement(0):
            # pipelined: the MLM decoder lives on the last stage, so it holds its own copy
            # of the tied 30522 x H table instead of shipping it across stages every step;
            # ``tied_to`` keeps the copies equal (same initial values, gradients summed
            # between the two stages each step: pipeline_exec ties)
            from ..ops.node import shadow_ids
            with _stage_ctx(placement, head), shadow_ids():
                E = _w('cls_decoder_weight', (cfg.padded_vocab_size, cfg.hidden_size), cfg)
            E.tied_to = self.bert.word_embeddings
        else:
            E = self.bert.word_embeddings
        self.cls = BertPreTrainingHeads(cfg, E)

    def __call__(self, input_ids, token_type_ids, attention_mask, masked_lm_labels=None,
                 next_sentence_label=None):
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        with _stage_ctx(self.placement, len(self.bert.layers) + 1):
            C = self.cfg.max_predictions_per_seq
            if C and masked_lm_labels is not None:
                # the labelled rows only (C slots per sequence); the mean of the per-slot
                # losses times C / S equals the reference's mean over all B*S rows (unlabelled
                # rows contribute 0): ``mlm_mean_scale``
                pos = ht.masked_positions_op(masked_lm_labels, C)
                self.masked_positions = pos
                seq = ht.take_rows_op(seq, pos)
                labels = ht.take_rows_op(masked_lm_labels, pos, fill_neg1=True)
            else:
                labels = masked_lm_labels
            scores, nsp = self.cls(seq, pooled)
            out = [scores, nsp]
            if masked_lm_labels is not None and next_sentence_label is not None:
                mlm = ht.softmaxcrossentropy_sparse_op(scores, labels, ignored_index=-1)
                # per-slot losses: their mean times C / S is the reference's mean over all rows
                self.mlm_mean_scale = float(C) / self.cfg.seq_len if C else 1.0
                ns = ht.softmaxcrossentropy_sparse_op(nsp, next_sentence_label, ignored_index=-1)
                out += [mlm, ns]
        return out


class BertForMaskedLM(BertForPreTraining):
    def __call__(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None):
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        scores, _ = self.cls(seq, pooled)
        if masked_lm_labels is None:
            return [scores]
        return [scores, ht.softmaxcrossentropy_sparse_op(scores, masked_lm_labels, ignored_index=-1)]


class BertForNextSentencePrediction(BertForPreTraining):
    def __call__(self, input_ids, token_type_ids=None, attention_mask=None, next_sentence_label=None):
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        _, nsp = self.cls(seq, pooled)
        if next_sentence_label is None:
            return [nsp]
        return [nsp, ht.softmaxcrossentropy_sparse_op(nsp, next_sentence_label, ignored_index=-1)]


class BertForSequenceClassification(object):
    """GLUE fine-tuning head (reference test_glue_hetu_bert.py)."""

    def __init__(self, cfg, num_labels=2):
        self.cfg, self.num_labels = cfg, num_labels
        self.bert = BertModel(cfg)

    def __call__(self, input_ids, token_type_ids, attention_mask, labels=None):
        _, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        logits = _dense(_dropout(pooled, self.cfg.hidden_dropout_prob), self.cfg.hidden_size,
                        self.num_labels, 'classifier', self.cfg)
        if labels is None:
            return logits
        # (loss, logits) like the reference (hetu_bert.py:853-865); the fused
        # sparse softmax-CE kernel replaces its softmax_op -> crossentropy_sparse_op
        return ht.softmaxcrossentropy_sparse_op(logits, labels, ignored_index=-1), logits


def plan_placement(plan, ctx_of_ranks=None):
    """layer -> device group of its pipeline stage under a Galvatron ``Plan``
    (``parallel.galvatron``); ``ctx_of_ranks`` maps a rank list to a context
    (default: the stage's GPUs)."""
    def placement(layer):
        s = next(i for i, (a, b) in enumerate(plan.stages) if a <= layer < b)
        ranks = plan.stage_ranks(s)
        if ctx_of_ranks is not None:
            return ctx_of_ranks(ranks)
        devs = plan.stage_devices(s)
        return devs if len(devs) > 1 else devs[0]
    return placement


def bert_pretrain_graph(cfg, lr=1e-5, optimizer=None, plan=None, placement=None):
    """Placeholders + loss + train op for BERT pretraining (reference
    train_hetu_bert.py: Adam lr 1e-5, loss = mean MLM + mean NSP).

    ``plan`` (a Galvatron ``Plan`` over the L+2 planner layers of
    ``galvatron.bert_layers``) or an explicit ``placement`` puts every layer in
    its pipeline stage's device context; run the result with
    ``Executor(..., pipeline='gpipe' | 'pipedream')``."""
    if plan is not None and placement is None and plan.pp > 1:
        placement = plan_placement(plan)
    with _stage_ctx(placement, 0):
        input_ids = ht.Variable(name='input_ids', trainable=False)
        token_type_ids = ht.Variable(name='token_type_ids', trainable=False)
        attention_mask = ht.Variable(name='attention_mask', trainable=False)
    with _stage_ctx(placement, cfg.num_hidden_layers + 1):
        mlm_labels = ht.Variable(name='masked_lm_labels', trainable=False)
        nsp_labels = ht.Variable(name='next_sentence_label', trainable=False)
    model = BertForPreTraining(cfg, placement)
    _, _, mlm, nsp = model(input_ids, token_type_ids, attention_mask, mlm_labels, nsp_labels)
    with _stage_ctx(placement, cfg.num_hidden_layers + 1):
        mlm_mean = ht.reduce_mean_op(mlm, [0])
        if getattr(model, 'mlm_mean_scale', 1.0) != 1.0:
            mlm_mean = ht.mul_byconst_op(mlm_mean, model.mlm_mean_scale)
        loss = mlm_mean + ht.reduce_mean_op(nsp, [0])
        opt = optimizer or optim.AdamOptimizer(learning_rate=lr)
        train = opt.minimize(loss)
    feeds = dict(input_ids=input_ids, token_type_ids=token_type_ids, attention_mask=attention_mask,
                 masked_lm_labels=mlm_labels, next_sentence_label=nsp_labels)
    return feeds, loss, train


def synthetic_bert_batch(cfg, seed=0, mask_prob=0.15):
    """Random ids; each token labelled with probability ``mask_prob`` -- or, with
    ``cfg.max_predictions_per_seq`` set, exactly min(max_predictions_per_seq,
    max(1, round(S * mask_prob))) labelled positions per sequence, as the original BERT's
    create_pretraining_data draws them"""
    rng = np.random.default_rng(seed)
    B, S = cfg.batch_size, cfg.seq_len
    ids = rng.integers(min(1000, cfg.vocab_size // 2), cfg.vocab_size, (B, S)).astype(np.int64)
    types = np.zeros((B, S), np.int64)
    types[:, S // 2:] = 1
    mask = np.ones((B, S), np.float32)
    C = getattr(cfg, 'max_predictions_per_seq', None)
    if C:
        n = min(int(C), max(1, int(round(S * mask_prob))))
        sel = np.argsort(rng.random((B, S)), axis=1)[:, :n]
        lab = np.zeros((B, S), bool)
        np.put_along_axis(lab, sel, True, axis=1)
        mlm = np.where(lab, ids, -1).astype(np.int64)
    else:
        mlm = np.where(rng.random((B, S)) < mask_prob, ids, -1).astype(np.int64)
    nsp = rng.integers(0, 2, (B,)).astype(np.int64)
    return dict(input_ids=ids, token_type_ids=types, attention_mask=mask, masked_lm_labels=mlm,
                next_sentence_label=nsp)


def bert_bench(args, world, rank, local):
    """Benchmark step for BASELINE config 4 (reference
    examples/nlp/bert/scripts/train_hetu_bert_base_dp.sh: BERT-base, seq 128,
    batch 64 per GPU, Adam lr 1e-5, MLM + NSP pretraining), bf16 compute,
    synthetic token ids.  On N > 1 GPUs the Galvatron planner picks the DP x PP
    layout for the node (``galvatron.plan_bert``; ``args.pp`` forces the pipeline
    degree) and the step runs EXACTLY that plan:

    * pp = 1: data parallel, bucketed RCCL all-reduce;
    * pp > 1: every planner layer goes to its stage's device group
      (``plan_placement``), the stages run the GPipe schedule over the plan's
      micro-batches, each stage is data parallel over its ``N / pp`` replicas
      (replica r of stage s talks to replica r of stage s+1) and all-reduces its
      gradients over the replica group.

    Tensor parallelism inside a layer is left to the dispatch lowering
    (``parallel.lowering``); the bench caps the planner at tp = 1
    (``HETU_GALVATRON_MAX_TP`` raises it).  Weak scaling: the global batch is
    ``batch * N`` in every layout.  ``args.bert_config`` (tests) replaces BERT-base.
    Returns (step_fn, samples_per_step, config, metric, finish_fn)."""
    import os
    import torch
    import hetu_61a7_amd as H
    from ..parallel.galvatron import GalvatronPlanner, Hardware, bert_layers
    B = args.batch or 64
    # the MLM head over the labelled positions only, 20 slots per sequence (the original
    # BERT's max_predictions_per_seq; HETU_BERT_MAX_PRED=0 scores every position)
    max_pred = int(os.environ.get('HETU_BERT_MAX_PRED', '20')) or None
    cfg = getattr(args, 'bert_config', None) or BertConfig.base(batch_size=B, seq_len=128,
                                                                 max_predictions_per_seq=max_pred)
    cfg.batch_size = B
    specs = bert_layers(cfg.hidden_size, cfg.num_hidden_layers, cfg.seq_len, cfg.vocab_size)
    planner = GalvatronPlanner(specs, hw=Hardware(gpus=world), max_tp=int(os.environ.get('HETU_GALVATRON_MAX_TP', '1')))
    force_pp = getattr(args, 'pp', None)
    plan = planner.search(B * world, pp_options=[force_pp] if force_pp else None)
    if max(plan.tp) > 1:
        raise NotImplementedError('bench: tensor-parallel layers (planner chose %s) are not wired into the '
                                  'BERT bench graph' % plan.short())
    on_gpu = torch.cuda.is_available()
    dev = torch.device('cuda', local) if on_gpu else torch.device('cpu')
    kw = dict(mixed_precision=args.dtype if on_gpu else None, seed=1234,
              bucket_mb=getattr(args, 'bucket_mb', 32), zero=getattr(args, 'zero', 0))
    opt = None
    if getattr(args, 'optimizer', None) == 'sgd':          # tests: gradient-exact comparisons
        opt = optim.SGDOptimizer(learning_rate=getattr(args, 'lr', 1e-2))
    if plan.pp > 1:
        kw.pop('zero')
        # one replica's batch is global / (N / pp) = B * pp, fed as plan.micro_batches
        # micro-batches: the graph is built for one micro-batch
        cfg.batch_size = B * plan.pp // plan.micro_batches
        feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-5, plan=plan, optimizer=opt)
        ex = H.Executor({'train': [loss, train]}, pipeline='gpipe', **kw)
        sub = ex.subexecutor['train']
        replica, m = sub.replica, plan.micro_batches
        parallelism = 'pp%d x dp%d (galvatron plan: %s)' % (plan.pp, world // plan.pp, plan.short())
    else:
        feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-5, optimizer=opt)
        if world > 1:
            ex = H.Executor({'train': [loss, train]}, dist_strategy=H.dist.DataParallel('allreduce'), **kw)
        else:
            ex = H.Executor({'train': [loss, train]}, ctx=H.gpu(local) if on_gpu else H.cpu(0), **kw)
        replica, m = rank, None
        parallelism = 'dp%d (galvatron plan: %s)' % (world, plan.short())
    # one global synthetic batch, each data-parallel replica takes its contiguous slice, so
    # every layout (dp N, pp x dp, one process) trains on the same global batch
    import copy
    gcfg = copy.copy(cfg)
    rb = B * plan.pp if plan.pp > 1 else cfg.batch_size
    gcfg.batch_size = B * world
    full = synthetic_bert_batch(gcfg, seed=10)
    batch = {k: v[replica * rb:(replica + 1) * rb] for k, v in full.items()}
    fd = {feeds[k]: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in batch.items()}

    def step():
        if m is None:
            return ex.run('train', feed_dict=fd)
        return ex.run('train', feed_dict=fd, batch_num=m)

    conf = {'model': 'BERT-base (L12 H768 A12, MLM+NSP)', 'global_batch': B * world, 'seq_len': cfg.seq_len,
            'parallelism': parallelism, 'optimizer': 'adam', 'per_gpu_batch': B,
            'mlm_head': ('labelled positions only, max_predictions_per_seq %d' % cfg.max_predictions_per_seq
                         if getattr(cfg, 'max_predictions_per_seq', None) else 'every position'),
            'plan': {'pp': plan.pp, 'micro_batches': plan.micro_batches, 'stages': plan.stages,
                     'est_ms': round(plan.time * 1e3, 3)}}
    step.executor = ex
    step.plan = plan

    def finish():
        from ..ops.mlm import MaskedPositionsOp
        for sub in getattr(ex, 'subexecutor', {}).values():
            for n in getattr(sub, 'topo_order', ()):
                if isinstance(n, MaskedPositionsOp):
                    n.check()      # no sequence had more labels than slots
    return step, B * world, conf, 'samples/sec (whole node) BERT-base pretraining', finish
