export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
