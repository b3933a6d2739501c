export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5 &&
$S bench_bert 300 python bench.py --model bert --steps 20 --warmup 5 &&
$S bench_moe 300 python bench.py --model moe --steps 20 --warmup 5 &&
$S bench_wdl 300 python bench.py --model wdl --steps 60 --warmup 10
