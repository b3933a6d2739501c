import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (ROCm device)')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_runtest_logstart(nodeid, location):
    # one flushed line per test on stderr, so that a native abort (HIP/MIOpen
    # SIGABRT) leaves the failing test id as the last line of the log
    if os.environ.get('HETU_TEST_TRACE', '1') != '0':
        sys.stderr.write('\n[test-start] %s\n' % nodeid)
        sys.stderr.flush()


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)
