export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S diag_bert 300 python -u scripts/diag_torch_ops.py 0 bert &&
$S diag_moe 300 python -u scripts/diag_torch_ops.py 0 moe
