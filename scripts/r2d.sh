export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_models 400 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread &&
$S bench_bert 300 python bench.py --model bert --steps 20 --warmup 5 &&
$S bench_moe 300 python bench.py --model moe --steps 20 --warmup 5 &&
$S bench_wdl 300 python bench.py --model wdl --steps 60 --warmup 10 &&
cd /tmp && $GRAFT_REPO_ROOT/scripts/gpu_step.sh prof_resnet 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3
