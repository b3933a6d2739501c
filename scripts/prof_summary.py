#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv into categories (per step)."""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
cat = defaultdict(float)
cnt = defaultdict(int)
tot = 0.0


def classify(n):
    if n.startswith('igemm_fwd') or 'conv' in n.lower() and 'fwd' in n:
        return 'conv_fwd (MIOpen)'
    if n.startswith('igemm_bwd'):
        return 'conv_dgrad (MIOpen)'
    if n.startswith('igemm_wrw'):
        return 'conv_wgrad (MIOpen)'
    if n.startswith('Cijk'):
        return 'gemm (hipBLASLt)'
    m = re.search(r'hetu::(\w+?)(<|\()', n)
    if m:
        return 'hetu::' + m.group(1)
    if 'at::native' in n:
        m = re.search(r'at::native::(?:\w+::)?(\w+)', n)
        return 'torch::' + (m.group(1) if m else 'other')
    return n[:60]


for r in rows:
    t = float(r['TotalDurationNs'])
    c = classify(r['Name'])
    cat[c] += t
    cnt[c] += int(r['Calls'])
    tot += t
print('%-48s %10s %8s %6s' % ('category', 'ms/step', 'calls', '%'))
for c, t in sorted(cat.items(), key=lambda kv: -kv[1]):
    print('%-48s %10.3f %8d %6.1f' % (c, t / 1e6 / steps, cnt[c] / steps, 100 * t / tot))
print('%-48s %10.3f' % ('TOTAL', tot / 1e6 / steps))
