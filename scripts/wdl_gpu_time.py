"""Device time of the Wide&Deep PS bench step: kernels per step and their summed
duration (torch.profiler activity trace over 20 steady steps), against the wall time per
step -- how much of the step the GPU is busy once the host path is short.

    python scripts/wdl_gpu_time.py            (HETU_PIECEWISE_GRAPH=0 shows every kernel)
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    server = bench.start_ps_server(1, 0)            # before this process touches the GPU
    import torch
    from torch.profiler import profile, ProfilerActivity
    sys.argv = ['bench.py', '--model', 'wdl', '--steps', '1', '--warmup', '0']
    args = bench.parse()
    from hetu_61a7_amd.models.ctr import wdl_criteo_bench
    step = wdl_criteo_bench(args, 1, 0, 0)[0]
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(n):
            step()
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    tot, cnt = collections.Counter(), collections.Counter()
    for e in prof.events():
        if 'CUDA' not in str(e.device_type):
            continue
        k = e.name.split('(')[0][:90]
        tot[k] += e.device_time_total if hasattr(e, 'device_time_total') else e.cuda_time_total
        cnt[k] += 1
    busy = sum(tot.values()) / n / 1e3
    print('steps %d  wall %.3f ms/step (profiled)  kernels %.1f/step  device busy %.3f ms/step'
          % (n, wall, sum(cnt.values()) / n, busy))
    for k, v in tot.most_common(25):
        print('%8.1f us/step  %5.1f/step  %s' % (v / n, cnt[k] / n, k))
    from hetu_61a7_amd.ps import worker
    worker.worker_finish()
    server.wait(timeout=60)


if __name__ == '__main__':
    main()
