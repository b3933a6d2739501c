"""BERT WordPiece tokenizer (reference ``python/hetu/tokenizers/bert_tokenizer.py``).

Pipeline: text cleanup (control chars dropped, whitespace normalised) ->
optional lower-casing + accent stripping -> split on whitespace, punctuation
and around CJK ideographs -> greedy longest-match-first WordPiece with the
``##`` continuation prefix.  Vocabularies are read from local files only (no
downloads: ``from_pretrained`` takes a directory or a vocab.txt path).
"""
from __future__ import annotations

import collections
import os
import unicodedata
from typing import Dict, Iterable, List, Optional

VOCAB_NAME = 'vocab.txt'


def load_vocab(vocab_file: str) -> Dict[str, int]:
    vocab = collections.OrderedDict()
    with open(vocab_file, 'r', encoding='utf-8') as f:
        for i, line in enumerate(f):
            tok = line.rstrip('\n').strip()
            if tok or line.strip() == '':
                vocab[tok] = i
    return vocab


def whitespace_tokenize(text: str) -> List[str]:
    text = text.strip()
    return text.split() if text else []


def _is_whitespace(ch):
    if ch in (' ', '\t', '\n', '\r'):
        return True
    return unicodedata.category(ch) == 'Zs'


def _is_control(ch):
    if ch in ('\t', '\n', '\r'):
        return False
    return unicodedata.category(ch).startswith('C')


def _is_punctuation(ch):
    cp = ord(ch)
    # ASCII non-alphanumerics are punctuation for BERT even when Unicode disagrees ($, ^, `)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return unicodedata.category(ch).startswith('P')


def _is_cjk(cp):
    return (0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0x20000 <= cp <= 0x2A6DF or
            0x2A700 <= cp <= 0x2B73F or 0x2B740 <= cp <= 0x2B81F or 0x2B820 <= cp <= 0x2CEAF or
            0xF900 <= cp <= 0xFAFF or 0x2F800 <= cp <= 0x2FA1F)


class BasicTokenizer(object):
    def __init__(self, do_lower_case=True, never_split=('[UNK]', '[SEP]', '[PAD]', '[CLS]', '[MASK]')):
        self.do_lower_case = do_lower_case
        self.never_split = set(never_split)

    def tokenize(self, text: str) -> List[str]:
        text = self._clean(text)
        text = ''.join(' %s ' % c if _is_cjk(ord(c)) else c for c in text)
        out = []
        for tok in whitespace_tokenize(text):
            if tok not in self.never_split:
                if self.do_lower_case:
                    tok = tok.lower()
                    tok = ''.join(c for c in unicodedata.normalize('NFD', tok) if unicodedata.category(c) != 'Mn')
                out.extend(self._split_punc(tok))
            else:
                out.append(tok)
        return whitespace_tokenize(' '.join(out))

    def _split_punc(self, tok):
        if tok in self.never_split:
            return [tok]
        pieces, cur = [], []
        for c in tok:
            if _is_punctuation(c):
                if cur:
                    pieces.append(''.join(cur))
                    cur = []
                pieces.append(c)
            else:
                cur.append(c)
        if cur:
            pieces.append(''.join(cur))
        return pieces

    @staticmethod
    def _clean(text):
        out = []
        for c in text:
            cp = ord(c)
            if cp == 0 or cp == 0xFFFD or _is_control(c):
                continue
            out.append(' ' if _is_whitespace(c) else c)
        return ''.join(out)


class WordpieceTokenizer(object):
    def __init__(self, vocab, unk_token='[UNK]', max_input_chars_per_word=100):
        self.vocab = vocab
        self.unk_token = unk_token
        self.max_chars = max_input_chars_per_word

    def tokenize(self, text: str) -> List[str]:
        out = []
        for word in whitespace_tokenize(text):
            if len(word) > self.max_chars:
                out.append(self.unk_token)
                continue
            start, sub = 0, []
            while start < len(word):
                end = len(word)
                piece = None
                while start < end:
                    cand = word[start:end]
                    if start > 0:
                        cand = '##' + cand
                    if cand in self.vocab:
                        piece = cand
                        break
                    end -= 1
                if piece is None:
                    sub = None
                    break
                sub.append(piece)
                start = end
            out.extend([self.unk_token] if sub is None else sub)
        return out


class BertTokenizer(object):
    def __init__(self, vocab_file, do_lower_case=True, max_len=None, do_basic_tokenize=True,
                 never_split=('[UNK]', '[SEP]', '[PAD]', '[CLS]', '[MASK]')):
        if not os.path.isfile(vocab_file):
            raise ValueError("Can't find a vocabulary file at path '%s'" % vocab_file)
        self.vocab = load_vocab(vocab_file)
        self.ids_to_tokens = collections.OrderedDict((i, t) for t, i in self.vocab.items())
        self.do_basic_tokenize = do_basic_tokenize
        self.basic_tokenizer = BasicTokenizer(do_lower_case, never_split) if do_basic_tokenize else None
        self.wordpiece_tokenizer = WordpieceTokenizer(self.vocab)
        self.max_len = max_len if max_len is not None else int(1e12)

    def tokenize(self, text: str) -> List[str]:
        if not self.do_basic_tokenize:
            return self.wordpiece_tokenizer.tokenize(text)
        out = []
        for tok in self.basic_tokenizer.tokenize(text):
            out.extend(self.wordpiece_tokenizer.tokenize(tok))
        return out

    def convert_tokens_to_ids(self, tokens: Iterable[str]) -> List[int]:
        ids = [self.vocab.get(t, self.vocab.get('[UNK]')) for t in tokens]
        if len(ids) > self.max_len:
            raise ValueError('sequence length %d exceeds max_len %d' % (len(ids), self.max_len))
        return ids

    def convert_ids_to_tokens(self, ids: Iterable[int]) -> List[str]:
        return [self.ids_to_tokens[i] for i in ids]

    def encode(self, text_a: str, text_b: Optional[str] = None, max_seq_len: Optional[int] = None):
        """[CLS] a [SEP] (b [SEP]) -> (input_ids, token_type_ids, attention_mask), padded."""
        a = self.tokenize(text_a)
        b = self.tokenize(text_b) if text_b else []
        if max_seq_len is not None:
            budget = max_seq_len - (3 if b else 2)
            while len(a) + len(b) > budget:
                (a if len(a) >= len(b) else b).pop()
        toks = ['[CLS]'] + a + ['[SEP]'] + (b + ['[SEP]'] if b else [])
        types = [0] * (len(a) + 2) + [1] * (len(b) + 1 if b else 0)
        ids = self.convert_tokens_to_ids(toks)
        mask = [1] * len(ids)
        if max_seq_len is not None:
            pad = max_seq_len - len(ids)
            ids += [self.vocab.get('[PAD]', 0)] * pad
            types += [0] * pad
            mask += [0] * pad
        return ids, types, mask

    def save_vocabulary(self, vocab_path):
        if os.path.isdir(vocab_path):
            vocab_path = os.path.join(vocab_path, VOCAB_NAME)
        with open(vocab_path, 'w', encoding='utf-8') as f:
            for tok, _ in sorted(self.vocab.items(), key=lambda kv: kv[1]):
                f.write(tok + '\n')
        return vocab_path

    @classmethod
    def from_pretrained(cls, path, **kwargs):
        """Local directory containing vocab.txt, or the vocab file itself."""
        vf = os.path.join(path, VOCAB_NAME) if os.path.isdir(path) else path
        return cls(vf, **kwargs)
