"""Per-(kernel, grid) steady-state times from a rocprofv3 kernel trace: the last N steps
(delimited by the once-per-step optimizer kernel), grouped by kernel family and launch
grid so the same kernel on different shapes stays apart.

    python scripts/prof_shapes.py run_kernel_trace.csv [--steps 3] [--marker opt_flat] [--top 60]
"""
import argparse
import collections
import csv
import re


def family(name):
    n = name.replace('(anonymous namespace)::', '').replace('hetu::gemm::', '').replace('hetu::attn::', '')
    n = n.replace('hetu::', '').replace('__hip_bfloat16', 'bf16')
    n = re.sub(r'\(.*', '', n)
    return re.sub(r'^void ', '', n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--marker', default='opt_flat')
    ap.add_argument('--top', type=int, default=60)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    sel = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        key = (family(r['Kernel_Name']), '%sx%sx%s' % (r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z']))
        agg[key][0] += 1
        agg[key][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    total = sum(v[1] for v in agg.values())
    print('steps=%d  kernel time %.3f ms/step  launches %d/step' % (a.steps, total / a.steps / 1e3, len(sel) // a.steps))
    print('%-70s %-18s %7s %9s %9s' % ('kernel', 'grid', 'n/step', 'us/call', 'ms/step'))
    for (k, g), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print('%-70s %-18s %7.1f %9.1f %9.3f' % (k, g, c / a.steps, us / c, us / a.steps / 1e3))


if __name__ == '__main__':
    main()
