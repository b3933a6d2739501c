"""Reference entry point examples/moe/test_moe_base.py: the MoE benchmark with the
'base' gate (same flags as test_moe.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_moe import main  # noqa: E402

if __name__ == '__main__':
    main(['--gate', 'base'] + sys.argv[1:])
