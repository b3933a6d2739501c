export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
PYTHONPATH=$PWD $S diag_bs2 300 python -u scripts/diag_layers.py 2 fused
