"""Masked-LM head over the labelled positions only (ops/mlm.py): the compacted graph
gives the same loss and the same gradients as scoring every position (CPU, fp32)."""
import numpy as np

import hetu_61a7_amd as ht
from hetu_61a7_amd.kernels import mlm as KM


def test_masked_positions_slots_in_position_order():
    import torch
    lab = torch.tensor([[-1, 5, -1, 7, 9], [-1, -1, -1, -1, 3], [1, 2, 3, 4, 5]])
    ovf = torch.zeros(1, dtype=torch.int32)
    idx = KM.masked_positions(lab, 3, ovf)
    assert idx.tolist() == [1, 3, 4, 9, -1, -1, 10, 11, 12]
    assert int(ovf[0]) == 5                      # the third sequence has 5 > 3 labels
    x = torch.arange(15, dtype=torch.float32).reshape(15, 1).repeat(1, 2)
    t = KM.take_rows(x, idx)
    assert t[:, 0].tolist() == [1, 3, 4, 9, 0, 0, 10, 11, 12]
    back = KM.put_rows(t, idx, 15)
    assert back[:, 0].tolist() == [0, 1, 0, 3, 4, 0, 0, 0, 0, 9, 10, 11, 12, 0, 0]


def _run(max_pred):
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    _node.G_NODE_ID = 0
    cfg = BertConfig(vocab_size=500, hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                     intermediate_size=64, batch_size=3, seq_len=16, max_position_embeddings=16,
                     hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, max_predictions_per_seq=4)
    batch = synthetic_bert_batch(cfg, seed=4)           # exactly 2 labels per sequence (round(16*0.15))
    cfg.max_predictions_per_seq = max_pred
    feeds, loss, train = bert_pretrain_graph(cfg, lr=0.1, optimizer=ht.optim.SGDOptimizer(0.1))
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0), seed=2)
    pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
    return ex, pm, {feeds[k]: v for k, v in batch.items()}


def test_gathered_head_matches_full_head():
    ex_a, pa, fa = _run(None)
    ex_b, pb, fb = _run(4)
    for k in pa:
        pb[k].copy_(pa[k])
    la = [float(np.asarray(ex_a.run('train', feed_dict=fa, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
          for _ in range(3)]
    lb = [float(np.asarray(ex_b.run('train', feed_dict=fb, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
          for _ in range(3)]
    np.testing.assert_allclose(lb, la, rtol=1e-5, atol=1e-6)
    for k in pa:        # every parameter, after three SGD steps
        np.testing.assert_allclose(pb[k].numpy(), pa[k].numpy(), rtol=1e-4, atol=1e-6)
