"""GLUE fine-tuning (reference examples/nlp/bert/test_glue_hetu_bert.py):
``BertForSequenceClassification`` (BERT encoder -> pooled [CLS] -> dropout ->
linear) trained with Adam + L2 on sentence(-pair) classification batches.

There is no network here for the GLUE files, so batches are synthetic with
the task's shape (``--task_name`` sst-2 / cola / mrpc: 2 labels, mnli: 3).  The
label is marked by the tokens after [CLS], so fine-tuning has something
learnable and the printed accuracy climbs.

    python examples/nlp/bert/test_glue_hetu_bert.py --task_name mnli --gpu_id 0
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.bert import BertConfig, BertForSequenceClassification  # noqa: E402

NUM_LABELS = {'sst-2': 2, 'cola': 2, 'mrpc': 2, 'mnli': 3}


def glue_batch(task, B, S, vocab, num_labels, rng):
    ids = rng.integers(1000, vocab, (B, S)).astype(np.int64)
    ids[:, 0] = 101                                            # [CLS]
    lens = rng.integers(S // 2, S + 1, B)
    mask = (np.arange(S)[None, :] < lens[:, None]).astype(np.float32)
    types = np.zeros((B, S), np.int64)
    if task in ('mrpc', 'mnli'):                               # sentence pairs
        types[:, S // 2:] = 1
    labels = rng.integers(0, num_labels, B).astype(np.int64)
    ids[:, 1:1 + S // 4] = 1000 + labels[:, None]              # label-marking tokens
    return dict(input_ids=ids, token_type_ids=types, attention_mask=mask, label_ids=labels)


def finetune(args):
    num_labels = NUM_LABELS[args.task_name]
    cfg = BertConfig(vocab_size=args.vocab_size, hidden_size=args.hidden_size,
                     num_hidden_layers=args.num_hidden_layers, num_attention_heads=args.num_attention_heads,
                     intermediate_size=4 * args.hidden_size, hidden_act=args.hidden_act,
                     hidden_dropout_prob=args.dropout_prob, attention_probs_dropout_prob=args.dropout_prob,
                     batch_size=args.train_batch_size, seq_len=args.seq_length,
                     max_position_embeddings=max(512, args.seq_length))
    model = BertForSequenceClassification(cfg, num_labels=num_labels)
    input_ids = ht.Variable(name='input_ids', trainable=False)
    token_type_ids = ht.Variable(name='token_type_ids', trainable=False)
    attention_mask = ht.Variable(name='attention_mask', trainable=False)
    label_ids = ht.Variable(name='label_ids', trainable=False)
    loss, logits = model(input_ids, token_type_ids, attention_mask, label_ids)
    loss = ht.reduce_mean_op(loss, [0])
    opt = ht.optim.AdamOptimizer(learning_rate=args.lr, beta1=0.9, beta2=0.999, epsilon=1e-8,
                                 l2reg=args.adam_weight_decay)
    train_op = opt.minimize(loss)
    ctx = ht.cpu(0) if args.gpu_id < 0 else ht.gpu(args.gpu_id)
    kw = dict(seed=1234)
    if args.gpu_id >= 0 and not args.fp32:
        kw['mixed_precision'] = 'bf16'
    ex = ht.Executor([loss, logits, train_op], ctx=ctx, **kw)
    rng = np.random.default_rng(0)
    accs = []
    for ep in range(args.epochs):
        for i in range(args.batches):
            t0 = time.time()
            b = glue_batch(args.task_name, args.train_batch_size, args.seq_length, args.vocab_size, num_labels, rng)
            fd = {input_ids: b['input_ids'], token_type_ids: b['token_type_ids'],
                  attention_mask: b['attention_mask'], label_ids: b['label_ids']}
            lo, lg = ex.run(feed_dict=fd, convert_to_numpy_ret_vals=True)[:2]
            acc = float(np.mean(np.argmax(np.asarray(lg, np.float32), 1) == b['label_ids']))
            accs.append(acc)
            print('[Epoch %d] (Iteration %d): Loss = %.3f, Accuracy = %.4f Time = %.3f'
                  % (ep, i, float(np.asarray(lo).reshape(-1)[0]), acc, time.time() - t0), flush=True)
    return accs


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpu_id', type=int, default=0, help='-1 = CPU')
    p.add_argument('--train_batch_size', type=int, default=16)
    p.add_argument('--task_name', default='sst-2', choices=sorted(NUM_LABELS))
    p.add_argument('--vocab_size', type=int, default=30522)
    p.add_argument('--hidden_size', type=int, default=768)
    p.add_argument('--num_hidden_layers', type=int, default=12)
    p.add_argument('-a', '--num_attention_heads', type=int, default=12)
    p.add_argument('-s', '--seq_length', type=int, default=128)
    p.add_argument('-e', '--epochs', type=int, default=10)
    p.add_argument('--batches', type=int, default=20, help='batches per epoch (synthetic)')
    p.add_argument('--lr', type=float, default=1e-5)
    p.add_argument('--adam_weight_decay', type=float, default=0.01)
    p.add_argument('--hidden_act', default='gelu')
    p.add_argument('--dropout_prob', type=float, default=0.1)
    p.add_argument('--fp32', action='store_true')
    return finetune(p.parse_args(argv))


if __name__ == '__main__':
    main()
