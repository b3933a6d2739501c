export TMPDIR=/tmp
S=scripts/gpu_step.sh
PYTHONPATH=$PWD $S test_bn 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "batchnorm or bn" || exit 1
PYTHONPATH=$PWD $S bench_bn 300 python -u scripts/bench_bn.py gpurun_out/bench_bn_r2aj.txt || exit 1
for i in 1 2; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 30 --warmup 5 > ../gpurun_out/ab_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
done
grep -h total gpurun_out/bench_bn_r2aj.txt
grep -h value gpurun_out/ab_old_*.log gpurun_out/ab_new_*.log | cut -c1-110
