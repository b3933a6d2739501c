"""Reproducibility of ResNet-50 (batch 4) parameter updates across executors in one process:
for each BN-fusion setting, two eager runs; prints step losses and the relative difference
of the per-step updates (BN parameters / the rest).  CPU runs are bitwise reproducible."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import torch  # noqa: E402

import test_bn_fusion_gpu as T  # noqa: E402


def rel(a, b, sel):
    num = sum(float((a[n] - b[n]).norm()) ** 2 for n in b if sel(n))
    den = sum(float(b[n].norm()) ** 2 for n in b if sel(n))
    return (num / max(den, 1e-30)) ** 0.5


def main():
    for stats, bwd in (('0', '0'), ('1', '0'), ('0', 'all'), ('1', 'all')):
        os.environ['HETU_FUSE_BN_STATS'] = stats
        runs = []
        for _ in range(2):
            os.environ['HETU_FUSE_BN_BWD'] = bwd
            src = T._resnet_updates.__code__
            losses, ups, _ = T._resnet_updates(False, steps=2, lr=1e-3)
            runs.append((losses, ups))
        print('stats=%s bwd=%s losses %s | %s' % (stats, bwd, [round(x, 5) for x in runs[0][0]],
                                                 [round(x, 5) for x in runs[1][0]]), flush=True)
        for k in range(2):
            print('   step %d: bn %.4f other %.4f' % (k, rel(runs[0][1][k], runs[1][1][k], lambda n: 'bn' in n),
                                                     rel(runs[0][1][k], runs[1][1][k], lambda n: 'bn' not in n)),
                  flush=True)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
