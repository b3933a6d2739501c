export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S diag_ops 300 python -u scripts/diag_torch_ops.py
