export TMPDIR=/tmp
S=scripts/gpu_step.sh
PYTHONPATH=$PWD $S test_sce 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 30 --warmup 5 > ../gpurun_out/ab_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 30 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
done
grep -h value gpurun_out/ab_old_*.log gpurun_out/ab_new_*.log | cut -c1-140
