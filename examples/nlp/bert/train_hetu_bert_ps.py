"""Reference entry point examples/nlp/bert/train_hetu_bert_ps.py: BERT pretraining (MLM + NSP), data parallel through the parameter server (launch with heturun -s 1 -w N).
Same flags as examples/nlp/train_hetu_bert.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from train_hetu_bert import main  # noqa: E402

if __name__ == '__main__':
    main(['--ps'] + sys.argv[1:])
