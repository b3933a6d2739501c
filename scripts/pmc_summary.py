"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) per kernel family.

    python scripts/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_mem gpurun_out/pmc_wr > profiles/x.txt

Per kernel family (template arguments and parameter lists stripped) it sums the
counters over every dispatch and derives:
  calls/ms = dispatches / summed dispatch time per step with --steps S (the --pmc run
             serialises dispatches), else over the whole window
  clk_GHz  = GRBM_GUI_ACTIVE / 8 / time (GRBM is summed over the 8 XCDs)
  mfma_pk  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8): the
             fraction of the chip's matrix-pipe cycles that were busy, i.e. the
             fraction of dense bf16 MFMA peak at the running clock
  wait     = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt/barrier)
  lds_cf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  rd_TB/s  = 2 * FETCH_SIZE KB / time (FETCH_SIZE reads 1/2 of a wide coalesced
             stream on gfx950, MI355X_MICROARCH.md); wr_TB/s = WRITE_SIZE KB / time
  TF/s     = 512 * SQ_INSTS_VALU_MFMA_MOPS_BF16 / time (4th directory, optional)
"""
import collections
import csv
import glob
import os
import re
import sys


def family(name):
    n = name.replace('(anonymous namespace)::', '').replace('hetu::gemm::', '').replace('hetu::attn::', '')
    n = n.replace('hetu::', '').replace('__hip_bfloat16', 'bf16').replace('HIP_vector_type<float, 4u>', 'float4')
    n = re.sub(r'\(.*', '', n)
    n = re.sub(r'^void ', '', n)
    if n.startswith('igemm_'):
        return n.split('_gtcx')[0] + ' (MIOpen)'
    return n[:90]


STEPS = 1
LAST = 0   # --last N: only the N most recent dispatches of each pass (steady state, no autotune)
MARKER = ''   # --marker K: the window is the last --steps steps, delimited by kernel K (once per step)


def load(d):
    """-> ({family: {counter: sum}}, {family: n_dispatches}, {family: summed dispatch ns})"""
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = {}
    rows = [r for f in files for r in csv.DictReader(open(f))]
    if MARKER:
        # exactly STEPS steps: the dispatches after the (STEPS+1)-th last launch of the
        # once-per-step marker kernel up to and including the last one
        ids = sorted({int(r['Dispatch_Id']) for r in rows if MARKER in r['Kernel_Name']})
        if len(ids) < STEPS + 1:
            raise SystemExit('only %d %s dispatches' % (len(ids), MARKER))
        lo, hi = ids[-STEPS - 1], ids[-1]
        rows = [r for r in rows if lo < int(r['Dispatch_Id']) <= hi]
    elif LAST:
        ids = sorted({int(r['Dispatch_Id']) for r in rows})[-LAST:]
        keep = set(ids)
        rows = [r for r in rows if int(r['Dispatch_Id']) in keep]
    for r in rows:
        if True:
            k = family(r['Kernel_Name'])
            agg[k][r['Counter_Name']] += float(r['Counter_Value'])
            seen[r['Dispatch_Id']] = (k, int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    calls, ns = collections.Counter(), collections.defaultdict(float)
    for k, t in seen.values():
        calls[k] += 1
        ns[k] += t
    return agg, calls, ns


def main(dirs):
    sq, calls, ns = load(dirs[0])
    mem = load(dirs[1]) if len(dirs) > 1 else ({}, {}, {})
    wr = load(dirs[2]) if len(dirs) > 2 else ({}, {}, {})
    mops = load(dirs[3]) if len(dirs) > 3 else ({}, {}, {})
    rows = sorted(sq.items(), key=lambda kv: -ns[kv[0]])
    print('%-64s %6s %8s %8s %8s %8s %8s %8s %7s %7s' % ('kernel family', 'calls', 'ms', 'clk_GHz', 'mfma_pk',
                                                         'wait', 'lds_cf', 'rd_TB/s', 'wr_TB/s', 'TF/s'))
    for k, c in rows[:40]:
        t = ns[k] * 1e-9
        cyc = c.get('GRBM_GUI_ACTIVE', 0) / 8.0                      # summed over 8 XCDs
        clk = cyc / t / 1e9 if t else float('nan')
        mf = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024.0 * cyc) if cyc else float('nan')
        wc = c.get('SQ_WAVE_CYCLES', 0)
        wait = c.get('SQ_WAIT_ANY', 0) / wc if wc else float('nan')
        lds = mem[0].get(k, {}).get('SQ_LDS_IDX_ACTIVE', 0)
        lc = c.get('SQ_LDS_BANK_CONFLICT', 0) / lds if lds else float('nan')
        tm = mem[2].get(k, 0) * 1e-9
        rd = 2 * mem[0].get(k, {}).get('FETCH_SIZE', 0) * 1024 / tm / 1e12 if tm else float('nan')
        tw = wr[2].get(k, 0) * 1e-9
        w = wr[0].get(k, {}).get('WRITE_SIZE', 0) * 1024 / tw / 1e12 if tw else float('nan')
        tmo = mops[2].get(k, 0) * 1e-9
        tf = 512 * mops[0].get(k, {}).get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0) / tmo / 1e12 if tmo else float('nan')
        print('%-64s %6.4g %8.3f %8.2f %8.3f %8.3f %8.3f %8.2f %7.2f %7.0f' % (k[:64], calls[k] / STEPS, t * 1e3 / STEPS,
                                                                             clk, mf, wait,
                                                                             lc, rd, w, tf))
    # HBM traffic of the whole window (the --last dispatches; per step with --steps S)
    rd_b = sum(2 * c.get('FETCH_SIZE', 0) * 1024 for c in mem[0].values()) if mem[0] else 0.0
    wr_b = sum(c.get('WRITE_SIZE', 0) * 1024 for c in wr[0].values()) if wr[0] else 0.0
    if rd_b or wr_b:
        print('\n# HBM bytes per %s: read %.2f GB, write %.2f GB, total %.2f GB' %
              ('step' if STEPS > 1 else 'window', rd_b / STEPS / 1e9, wr_b / STEPS / 1e9, (rd_b + wr_b) / STEPS / 1e9))
    # every counter of every pass, per dispatch (raw sums / calls), for the top families
    print('\n# raw counters per dispatch')
    for k, c in rows[:12]:
        allc = dict(c)
        for d in (mem, wr):
            allc.update(d[0].get(k, {}) if d[0] else {})
        n = max(calls[k], 1)
        print('%s: %s' % (k[:64], ', '.join('%s=%.4g' % (cn, v / n) for cn, v in sorted(allc.items()))))


if __name__ == '__main__':
    a = sys.argv[1:]
    while a and a[0] in ('--last', '--steps', '--marker'):
        if a[0] == '--last':
            LAST = int(a[1])
        elif a[0] == '--marker':
            MARKER = a[1]
        else:
            STEPS = int(a[1])
        a = a[2:]
    main(a)
