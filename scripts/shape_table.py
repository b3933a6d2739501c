"""Per-shape before/after table from two autotune dumps (HETU_AUTOTUNE_DUMP): the round-3
choice (hand-written vs library, per-shape timing) against the round-4 hand-written-only
choice.  Keys that changed form (dgrad -> dgrad_bn when the BN reduction is fused, the 30522
vocabulary padded to 30528) are matched by shape.

    python scripts/shape_table.py before.txt after.txt > table.md
"""
import re
import sys


def load(p):
    d = {}
    for line in open(p):
        if ' -> ' not in line:
            continue
        k, rest = line.split(' -> ', 1)
        choice = rest.split()[0]
        times = {a: float(b) for a, b in re.findall(r'(\w+)=([\d.]+)us', rest)}
        d[k.strip()] = (choice, times)
    return d


def norm(k):
    k = k.replace("('dgrad_bn',", "('dgrad',").replace("('fwd_stats',", "('fwd',").replace('30522', '30528')
    return k


def main(a, b):
    r3, r4 = load(a), load(b)
    r3n = {norm(k): v for k, v in r3.items()}
    print('| shape (autotune key) | before: choice | before: us | before: best library us | after: hand-written choice | after: us |')
    print('|---|---|---|---|---|---|')
    tot3 = tot4 = 0.0
    for k, (c4, t4) in r4.items():
        old = r3n.get(norm(k))
        u4 = t4.get(c4)
        if old is None:
            print('| `%s` | (new key) | | | %s | %s |' % (k, c4, '%.1f' % u4 if u4 else ''))
            continue
        c3, t3 = old
        u3 = t3.get(c3)
        lib = [v for n, v in t3.items() if not n.startswith('hip')]
        print('| `%s` | %s | %s | %s | %s | %s |' % (k, c3, '%.1f' % u3 if u3 else '', '%.1f' % min(lib) if lib else '',
                                                   c4, '%.1f' % u4 if u4 else ''))
        if u3 and u4:
            tot3 += u3
            tot4 += u4
    print('\nSum over shapes timed in both (one call each): before %.0f us, after %.0f us.' % (tot3, tot4))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
