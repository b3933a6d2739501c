"""Fused transformer kernels on the GPU vs torch fp32 references."""
import pytest
import torch

from test_fused_ln_cpu import fused_ln_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('N', [768, 1024, 64, 2048])
@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_fp32(N, keep):
    fused_ln_check('cuda', torch.float32, R=300, N=N, keep=keep, tol=2e-5)


@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_bf16(keep):
    fused_ln_check('cuda', torch.bfloat16, R=257, N=768, keep=keep)


@pytest.mark.parametrize('S', [32, 64, 96, 128, 256])
@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_packed_attention_bf16(S, keep):
    from test_bert_cpu import packed_attention_check
    packed_attention_check('cuda', torch.bfloat16, B=3, S=S, NH=2, D=64, keep=keep, tol=2.5e-2)


def test_bert_fused_attention_gpu_bf16_trains():
    import numpy as np
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.models.bert import BertConfig, bert_pretrain_graph, synthetic_bert_batch
    from hetu_61a7_amd.ops import node as _node
    out, init = [], None
    for fused in (False, True):
        _node.G_NODE_ID = 0
        cfg = BertConfig(vocab_size=2000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                         intermediate_size=256, batch_size=4, seq_len=64, max_position_embeddings=64,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, fused_attention=fused)
        feeds, loss, train = bert_pretrain_graph(cfg, lr=1e-3)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), seed=2, mixed_precision='bf16')
        from hetu_61a7_amd.utils.checkpoint import state_dict, load_dict
        if init is None:
            init = state_dict(ex)
        else:
            load_dict(ex, init)      # fp32 masters AND their bf16 compute copies
        fd = {feeds[k]: v for k, v in synthetic_bert_batch(cfg, seed=1).items()}
        out.append([float(np.asarray(ex.run('train', feed_dict=fd, convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0])
                    for _ in range(6)])
    np.testing.assert_allclose(out[0], out[1], rtol=3e-2, atol=3e-2)
    assert out[1][-1] < out[1][0]
