"""mlm_gather.hip against the CPU reference of kernels/mlm.py, and the BERT pretraining
graph with the masked-position MLM head against the full head on the GPU (bf16)."""
import numpy as np
import pytest
import torch

import hetu_61a7_amd as ht
from hetu_61a7_amd.kernels import mlm as KM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('B,S,C,H', [(64, 128, 20, 768), (3, 100, 7, 24), (5, 200, 40, 64)])
def test_masked_rows_kernels_match_reference(B, S, C, H):
    g = torch.Generator().manual_seed(B * S)
    lab = torch.where(torch.rand(B, S, generator=g) < 0.12, torch.randint(0, 1000, (B, S), generator=g),
                      torch.full((B, S), -1, dtype=torch.int64))
    lab[0, :] = 1                                       # an overflowing sequence (S > C labels)
    ovf_c = torch.zeros(1, dtype=torch.int32)
    ref = KM.masked_positions(lab, C, ovf_c)
    from hetu_61a7_amd.kernels.tensor import zeros
    ovf = zeros((1,), torch.int32, 'cuda')
    idx = KM.masked_positions(lab.cuda(), C, ovf)
    assert torch.equal(idx.cpu(), ref)
    for dt in (torch.int32, torch.float32):                   # fp32: mixed-precision label feeds
        assert torch.equal(KM.masked_positions(lab.to(dt).cuda(), C, zeros((1,), torch.int32, 'cuda')).cpu(), ref)
    assert int(ovf_c[0]) == S and int(ovf.cpu()[0]) > C      # the device flag: some overflowing count
    x = torch.randn(B * S, H, generator=g).bfloat16()
    t = KM.take_rows(x.cuda(), idx)
    assert torch.equal(t.cpu(), KM.take_rows(x, ref))
    for dt in (torch.int64, torch.int32, torch.float32):     # fp32: mixed-precision label feeds
        lg = KM.take_rows(lab.reshape(-1).to(dt).cuda(), idx, fill_neg1=True)
        assert torch.equal(lg.cpu(), KM.take_rows(lab.reshape(-1).to(dt), ref, fill_neg1=True)), dt
    back = KM.put_rows(t, idx, B * S)
    assert torch.equal(back.cpu(), KM.put_rows(t.cpu(), ref, B * S))


def test_bert_masked_position_head_trains_like_full_head():
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    out, init = {}, None
    for C in (None, 20):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=2000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                         intermediate_size=256, batch_size=8, seq_len=128, max_position_embeddings=128,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, max_predictions_per_seq=20)
        batch = synthetic_bert_batch(cfg, seed=1)
        cfg.max_predictions_per_seq = C
        feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-3)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=2, mixed_precision='bf16')
        pm = {n.name: t for n, t in ex.config.placeholder_to_arr_map.items() if n.trainable}
        if init is None:
            init = {k: v.detach().clone() for k, v in pm.items()}
        else:
            for k, v in pm.items():
                v.copy_(init[k])
            # the bf16 compute shadows of the flat parameters follow their masters (the two
            # graphs number their nodes differently, so their own initial values differ)
            for op in ex.subexecutor['train'].opt_ops:
                f = op.flat
                if f is not None and f.shadow is not None and f.shadow.shape == f.param.shape:
                    f.shadow.copy_(f.param)
        fd = {feeds[k]: torch.from_numpy(v).cuda() for k, v in batch.items()}
        out[C] = [float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
                  for _ in range(6)]
    np.testing.assert_allclose(out[20], out[None], rtol=2e-2)
    assert out[20][-1] < out[20][0]
