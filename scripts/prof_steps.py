#!/usr/bin/env python3
"""Steady-state per-step kernel breakdown from a rocprofv3 kernel_trace.csv.

Steps are delimited by the fused optimizer kernel (one launch per step); the
last ``--last`` complete steps are summarised, so warm-up and autotuning
launches do not pollute the numbers.

    python scripts/prof_steps.py gpurun_out/prof/run_kernel_trace.csv --last 3
"""
import argparse
import csv
import re
from collections import defaultdict


def classify(n):
    if n.startswith('igemm_fwd') or ('conv' in n.lower() and 'fwd' in n):
        return 'conv_fwd (MIOpen)'
    if n.startswith('igemm_bwd'):
        return 'conv_dgrad (MIOpen)'
    if n.startswith('igemm_wrw'):
        return 'conv_wgrad (MIOpen)'
    if n.startswith('Cijk'):
        return 'gemm (hipBLASLt)'
    m = re.search(r'hetu::gemm::gemm_kernel<hetu::gemm::(\w+), hetu::gemm::(\w+), (true|false)', n)
    if m:
        return 'hetu::gemm<%s,%s,%s>' % m.groups()
    if 'hetu::gemm' in n and '<' in n:
        return n.split('(')[0].replace('hetu::gemmf::', '').replace('hetu::gemm::', '').replace('void ', '')[:60]
    m = re.search(r'hetu::(\w+?)(<|\()', n)
    if m:
        return 'hetu::' + m.group(1)
    if 'at::native' in n:
        m = re.search(r'at::native::(?:\w+::)?(\w+)', n)
        return 'torch::' + (m.group(1) if m else 'other')
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--last', type=int, default=3)
    ap.add_argument('--marker', default='opt_flat')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--context', action='append', default=[],
                    help='category substring: list each launch of it in the last step with its neighbours')
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    if len(ends) < a.last + 1:
        raise SystemExit('only %d step markers found' % len(ends))
    lo, hi = ends[-a.last - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    cat, cnt = defaultdict(float), defaultdict(int)
    busy = 0.0
    for r in sel:
        t = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        c = classify(r['Kernel_Name'])
        cat[c] += t
        cnt[c] += 1
        busy += t
    wall = (int(sel[-1]['End_Timestamp']) - int(sel[0]['Start_Timestamp'])) / 1e6
    print('steps=%d  wall %.3f ms/step  kernel-busy %.3f ms/step  launches %.0f/step' %
          (a.last, wall / a.last, busy / a.last, len(sel) / a.last))
    print('%-52s %9s %7s %6s' % ('category', 'ms/step', 'calls', '%'))
    for c, t in sorted(cat.items(), key=lambda kv: -kv[1])[:a.top]:
        print('%-52s %9.3f %7.1f %6.1f' % (c, t / a.last, cnt[c] / a.last, 100 * t / busy))
    last = rows[ends[-2] + 1:ends[-1] + 1]
    for want in a.context:
        print('\n# launches of %r in the last step (prev | this | next)' % want)
        for i, r in enumerate(last):
            if want.lower() in classify(r['Kernel_Name']).lower():
                dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
                nb = lambda j: classify(last[j]['Kernel_Name']) if 0 <= j < len(last) else '-'
                print('%4d  %-40s | %-30s %7.1f us grid %s | %s' % (
                    i, nb(i - 1)[:40], classify(r['Kernel_Name'])[:30], dur,
                    r.get('Grid_Size', r.get('Grid_Size_X', '?')), nb(i + 1)[:40]))


if __name__ == '__main__':
    main()
