"""Which parameters differ after one step between the full MLM head and the
masked-position head (GPU): SGD, fp32 and bf16."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import hetu_61a7_amd as ht
from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
from hetu_61a7_amd.ops import node as _node

for mp in (None, 'bf16'):
    res, init = {}, None
    for C in (None, 20):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=2000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                         intermediate_size=256, batch_size=8, seq_len=128, max_position_embeddings=128,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, max_predictions_per_seq=20)
        batch = synthetic_bert_batch(cfg, seed=1)
        cfg.max_predictions_per_seq = C
        feeds, loss, train = bert_pretrain_graph(cfg, lr=0.1, optimizer=ht.optim.SGDOptimizer(0.1))
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=2, mixed_precision=mp, use_hipgraph=False)
        pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
        if init is None:
            init = {k: v.detach().clone() for k, v in pm.items()}
        else:
            for k, v in pm.items():
                v.copy_(init[k])
        fd = {feeds[k]: torch.from_numpy(v).cuda() for k, v in batch.items()}
        l = float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
        res[C] = (l, {k: (v.detach().float().cpu() - init[k].float().cpu()) for k, v in pm.items()})
    print('mixed_precision', mp, 'loss full %.6f gathered %.6f' % (res[None][0], res[20][0]))
    rows = []
    for k, d0 in res[None][1].items():
        d1 = res[20][1][k]
        rel = float((d1 - d0).norm() / d0.norm().clamp_min(1e-12))
        rows.append((rel, k, float(d0.norm()), float(d1.norm())))
    for r in sorted(rows, reverse=True)[:8]:
        print('  %-40s rel %.3e  |d_full| %.3e  |d_gath| %.3e' % (r[1], r[0], r[2], r[3]))
