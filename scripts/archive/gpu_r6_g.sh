#!/bin/bash
# attention LDS stride A/B: fused attention tests, kernel timings, one PMC pass over the
# attention kernels (lds_cf), then the steady-state PMC passes of BERT and ResNet-50
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py \
  tests/test_ring_attention_gpu.py tests/test_fused_gpu.py tests/test_models_gpu.py -k "attn or attention or bert or transformer or flash or ring or seqblock" > $O/r6g_tests.txt 2>&1
rc=$?; tail -3 $O/r6g_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 180 python -u scripts/bench_attn.py > $O/r6g_attn.txt 2>&1 || exit $?
cat $O/r6g_attn.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  -d $O/r6g_attn_pmc -o run --output-format csv -- python3 $R/scripts/bench_attn.py > $O/r6g_attn_pmc.log 2>&1 || exit $?
python3 -c "
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.Counter())
for f in glob.glob('$O/r6g_attn_pmc/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r'\(.*', '', r['Kernel_Name'])
        if 'attn' in k or 'flash' in k:
            agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in sorted(agg.items()):
    a = c['SQ_LDS_IDX_ACTIVE']
    print('%-60s lds_cf %.3f wait %.3f' % (k[:60], c['SQ_LDS_BANK_CONFLICT'] / a if a else float('nan'),
          c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES'] if c['SQ_WAVE_CYCLES'] else float('nan')))
" > $O/r6g_attn_lds.txt; cat $O/r6g_attn_lds.txt
rm -rf $O/r6g_attn_pmc
cd $R
PMC_MODEL=bert bash scripts/gpu_pmc_steady.sh && PMC_MODEL=resnet50 bash scripts/gpu_pmc_steady.sh
