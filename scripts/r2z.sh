export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && $GRAFT_REPO_ROOT/scripts/gpu_step.sh prof_resnet 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2z -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 &&
cd $GRAFT_REPO_ROOT && python scripts/prof_steps.py gpurun_out/prof_r2z/run_kernel_trace.csv --last 3 --context copyBuffer --context manual_unroll --context reduce_kernel --context vectorized_elementwise > gpurun_out/resnet_steady_r2z.txt 2>&1 && rm -f gpurun_out/prof_r2z/run_kernel_trace.csv
