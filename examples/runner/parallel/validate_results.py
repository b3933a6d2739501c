"""Every saved layout must reproduce the single-process baseline (reference
examples/runner/parallel/validate_results.py): ``results/<tag>_rank<r>.npy`` vs
``results/base.npy`` within rtol 1e-4.  The ranks of one layout that saved
losses are averaged first: data-parallel replicas each hold the mean loss of
their equal batch shard, whose average is the full-batch loss."""
import glob
import os
import re
import sys
from collections import defaultdict

import numpy as np


def main(path=None, rtol=1e-4):
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'results')
    base = np.load(os.path.join(path, 'base.npy'))
    groups = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(path, '*_rank*.npy'))):
        groups[re.sub(r'_rank\d+\.npy$', '', os.path.basename(f))].append(np.load(f))
    bad = 0
    for tag, arrs in sorted(groups.items()):
        r = np.mean(arrs, axis=0)
        ok = r.shape == base.shape and np.allclose(r, base, rtol=rtol, atol=1e-6)
        bad += not ok
        print('%-24s ranks %d  %s' % (tag, len(arrs), 'ok' if ok else 'MISMATCH %s vs %s' % (r, base)))
    return bad


if __name__ == '__main__':
    sys.exit(1 if main(*(sys.argv[1:2])) else 0)
