export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S wdl_ops_cpu 300 python -u scripts/wdl_ops.py cpu &&
$S wdl_ops_gpu 300 python -u scripts/wdl_ops.py gpu
