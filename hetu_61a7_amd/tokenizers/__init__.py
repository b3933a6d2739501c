from .bert_tokenizer import BertTokenizer, BasicTokenizer, WordpieceTokenizer, load_vocab
