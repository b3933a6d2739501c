"""Per-BatchNorm backward segments of two rocprofv3 kernel traces (last full step), side by
side: each segment = the kernels since the previous bn_bwd_apply up to and including the
next one (the data-gradient conv feeding that BN, its partial/finalize passes, the apply),
weight-gradient kernels excluded.  Usage: bn_layer_diff.py A.csv B.csv"""
import csv
import re
import sys

WGRAD = ('ConvWgradB', 'BufMN, BufMN', 'BufMN<true, 4>, BufMN<true, 4>', 'wgrad', 'splitk_reduce', 'opt_flat',
         'reduce_', 'bn_stats', 'bn_apply<', 'stem')


def segments(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    ks = []
    for r in rows:
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').replace('hetu::', '')
        n = n.replace('gemm::', '').replace('__hip_bfloat16', 'bf16')
        n = re.sub(r'\(.*', '', n)
        ks.append((n, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
    idx = [i for i, k in enumerate(ks) if 'maxpool_fwd_vec' in k[0]]
    step = ks[idx[-2]:idx[-1]]
    start = [i for i, k in enumerate(step) if 'sce_bwd' in k[0]][0]
    segs, cur = [], []
    for n, d in step[start:]:
        if any(w in n for w in WGRAD) and 'bn_bwd' not in n:
            continue
        cur.append((n, d))
        if 'bn_bwd_apply' in n:
            segs.append(cur)
            cur = []
    return segs


def short(n):
    n = n.replace('gemm_kernel', 'gk').replace('<true, 4>', '').replace('gemm_big_kernel', 'big')
    return re.sub(r'<bf16, ', '<', n)[:44]


def main():
    a, b = segments(sys.argv[1]), segments(sys.argv[2])
    ta = tb = 0.0
    for i in range(max(len(a), len(b))):
        sa = a[i] if i < len(a) else []
        sb = b[i] if i < len(b) else []
        da, db = sum(d for _, d in sa), sum(d for _, d in sb)
        ta += da
        tb += db
        print('#%-3d %8.0f %8.0f %+7.0f   %s  ||  %s' % (i, da, db, da - db,
              ' + '.join('%s %.0f' % (short(n), d) for n, d in sa),
              ' + '.join('%s %.0f' % (short(n), d) for n, d in sb)))
    print('total %.0f %.0f %+.0f us' % (ta, tb, ta - tb))


if __name__ == '__main__':
    main()
