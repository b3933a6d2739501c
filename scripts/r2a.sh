set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S diag_bs2_bf16 180 python -u scripts/diag_smoke.py 2 bf16 &&
$S diag_bs2_bf16_vendor 180 env HETU_CONV=vendor python -u scripts/diag_smoke.py 2 bf16 &&
$S diag_bs2_fp32 180 python -u scripts/diag_smoke.py 2 none &&
$S diag_bs32_bf16 180 python -u scripts/diag_smoke.py 32 bf16 &&
$S convbias_serial 180 env AMD_SERIALIZE_KERNEL=3 python -u -m pytest tests -m gpu -x -v -k "conv_bias" --timeout 120 --timeout-method thread &&
$S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5
