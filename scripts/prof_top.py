#!/usr/bin/env python3
"""Top kernels of a rocprofv3 kernel_stats.csv, per step: prof_top.py CSV STEPS [N]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
tot = sum(float(r['TotalDurationNs']) for r in rows) / steps / 1e6
print('total kernel ms/step %.3f' % tot)
print('%-100s %7s %8s %8s' % ('kernel', 'calls', 'ms/step', 'avg_us'))
for r in rows[:n]:
    print('%-100s %7d %8.3f %8.1f' % (r['Name'][:100], int(r['Calls']) / steps, float(r['TotalDurationNs']) / steps / 1e6,
                                      float(r['AverageNs']) / 1e3))
