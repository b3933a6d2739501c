#!/bin/bash
# Round-5: same-box A/B of the GELU dual-store epilogue on BERT-base (interleaved), then
# steady-state rocprofv3 kernel traces of BERT, ResNet-50 and MoE.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  for g in 1 0; do
    HETU_GELU_EPILOGUE=$g timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5i_bert_gelu$g.$i.json 2> gpurun_out/r5i_bert_gelu$g.$i.err
    rc=$?; echo "gelu_epilogue=$g run $i: $(tail -1 gpurun_out/r5i_bert_gelu$g.$i.json | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
  done
done
bash scripts/gpu_r5_h.sh
