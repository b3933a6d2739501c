"""WordPiece tokenizer parity with the HuggingFace reference implementation
(transformers.BertTokenizer, pure-python, same local vocab file)."""
import pytest

from hetu_61a7_amd.tokenizers import BertTokenizer

VOCAB = ['[PAD]', '[UNK]', '[CLS]', '[SEP]', '[MASK]', 'the', 'quick', 'brown', 'fox', 'jump', '##s',
         '##ed', 'over', 'lazy', 'dog', '.', ',', '!', 'un', '##aff', '##able', 'runn', '##ing', 'hello',
         'world', '中', '国', 'cafe', "'", 's', 'a']
TEXTS = ["The quick brown fox jumps over the lazy dog.", "unaffable running, HELLO world!",
         "中国 café's fox", "\tweird   spacing\x00 and control", "jumped, jumping!"]


@pytest.fixture
def vocab_file(tmp_path):
    p = tmp_path / 'vocab.txt'
    p.write_text('\n'.join(VOCAB) + '\n', encoding='utf-8')
    return str(p)


def test_wordpiece_matches_transformers(vocab_file):
    tr = pytest.importorskip('transformers')
    ref = tr.BertTokenizer(vocab_file, do_lower_case=True)
    ours = BertTokenizer(vocab_file, do_lower_case=True)
    for t in TEXTS:
        assert ours.tokenize(t) == ref.tokenize(t), t
        assert ours.convert_tokens_to_ids(ours.tokenize(t)) == ref.convert_tokens_to_ids(ref.tokenize(t))


def test_encode_pair(vocab_file):
    tok = BertTokenizer(vocab_file)
    ids, types, mask = tok.encode('the fox', 'lazy dog', max_seq_len=10)
    assert tok.convert_ids_to_tokens(ids[:8]) == ['[CLS]', 'the', 'fox', '[SEP]', 'lazy', 'dog', '[SEP]', '[PAD]']
    assert types[:7] == [0, 0, 0, 0, 1, 1, 1] and sum(mask) == 7
