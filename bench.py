#!/usr/bin/env python3
"""Flagship benchmark: ResNet-50 (ImageNet-shaped, synthetic data, random init)
data-parallel training on N MI355X GPUs, bf16 compute with fp32 master weights,
bucketed RCCL all-reduce overlapped with backward.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

Prints ONE JSON line on rank 0.  ``value`` is whole-job samples/s (all ranks),
``scaling`` is weak (fixed per-GPU batch).  Secondary BASELINE configs:
``--model wdl`` (Wide&Deep-Criteo, PS + HET cache), ``--model bert`` (BERT-base
pretraining, Galvatron-planned DP), ``--model moe`` (top-2 MoE, expert
all-to-all; ``--moe-gate dts`` for the dense-to-sparse gate).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--batch', type=int, default=None, help='per-GPU batch (256 resnet50, 128 wdl)')
    p.add_argument('--criteo-rows', type=int, default=0, help='embedding rows (default: full Criteo 33762577)')
    p.add_argument('--cache', default='LFUOpt')
    p.add_argument('--no-prefetch', dest='prefetch', action='store_false',
                   help='wdl: do not prefetch the next batch rows with the push')
    p.add_argument('--model', default='resnet50', choices=['resnet50', 'wdl', 'bert', 'moe', 'logreg'])
    p.add_argument('--moe-gate', default='topk', choices=['topk', 'dts'])
    p.add_argument('--moe-local-experts', type=int, default=2,
                   help='moe: experts per GPU (the reference scripts: 2; the DTS schedule run: 16)')
    p.add_argument('--dts-schedule', default=None,
                   help='moe dts: "tau0,decay,tau_min" temperature schedule; every step is then timed '
                        'alone and the JSON reports ms/step per expert budget and the budget changes')
    p.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    p.add_argument('--bucket-mb', type=float, default=32)
    p.add_argument('--zero', type=int, default=0, help='1: ZeRO-1 sharded optimizer state over the DP group')
    p.add_argument('--pp', type=int, default=None, help='bert: force the Galvatron pipeline degree')
    p.add_argument('--comm', default='PS', choices=['PS', 'Hybrid'],
                   help='wdl: PS = dense parameters on the server too (BASELINE config 3), Hybrid = RCCL dense')
    p.add_argument('--ids', default='zipf', choices=['zipf', 'uniform'],
                   help='wdl: sparse id distribution (uniform = cache worst-case control)')
    p.add_argument('--op-profile', default=None, help='write per-op-type GPU time (ms) to this file')
    p.add_argument('--grad-wire', default=os.environ.get('HETU_GRAD_WIRE', 'fp32'), choices=['fp32', 'bf16'],
                   help='DP gradient all-reduce wire format (bf16: fp32 accumulation)')
    p.add_argument('--comm-trace', action='store_true',
                   help='report the last step\'s all-reduce bucket timeline in the JSON config')
    p.add_argument('--rehearse-cpu', action='store_true',
                   help='run the model on the CPU (fp32, gloo between ranks): a dry run of the multi-GPU '
                        'launch that prints the same JSON line (tests/test_rehearse8_cpu.py)')
    return p.parse_args()


def start_ps_server(world, local):
    """One PS server process per node, started by local rank 0 BEFORE any GPU
    initialisation in this process (the server never touches the GPU)."""
    import subprocess
    os.environ.setdefault('DMLC_PS_ROOT_PORT', str(int(os.environ.get('MASTER_PORT', '29500')) + 7))
    os.environ['DMLC_NUM_WORKER'] = str(world)
    os.environ.setdefault('DMLC_NUM_SERVER', '1')
    os.environ.setdefault('HETU_PS_HEAP_GB', '24')
    if local != 0:
        return None
    env = dict(os.environ, DMLC_ROLE='server')
    return subprocess.Popen([sys.executable, '-m', 'hetu_61a7_amd.ps'], env=env)


def _progress(rank, world, msg):
    """per-rank progress on stderr for multi-rank runs (a stalled rank is then visible
    by its last line, and faulthandler dumps every rank's stack if it stalls)"""
    if world > 1:
        print('[bench rank %d/%d %.1fs] %s' % (rank, world, time.perf_counter() - _T0, msg), file=sys.stderr,
              flush=True)


_T0 = time.perf_counter()

_VENDOR_MARKS = ('Cijk', 'igemm', 'SubTensorOp', 'naive_conv', 'MIOpen', 'miopen', 'ck::', '_ZN2ck', 'gridwise_')


def _kernel_census(step):
    """one extra step (outside the timed region) under torch.profiler: device kernels
    that are PyTorch (at::native / c10) or vendor-library (hipBLASLt / MIOpen / CK)
    kernels.  Every rank runs it (collectives stay matched)."""
    import torch
    from torch.profiler import profile, ProfilerActivity
    from hetu_61a7_amd.utils import hipgraph
    torch.cuda.synchronize()
    hipgraph.FORCE_EAGER[0] += 1          # the kernels of the step, not one graph launch
    try:
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            step()
            torch.cuda.synchronize()
    finally:
        hipgraph.FORCE_EAGER[0] -= 1
    n = aten = vendor = 0
    names = {}
    for e in prof.events():
        if 'CUDA' not in str(e.device_type):
            continue
        n += 1
        if 'at::native' in e.name or 'c10::' in e.name:
            aten += 1
            names[e.name[:80]] = names.get(e.name[:80], 0) + 1
        elif any(v in e.name for v in _VENDOR_MARKS):
            vendor += 1
            names[e.name[:80]] = names.get(e.name[:80], 0) + 1
    return {'kernels_per_step': n, 'aten_kernels_per_step': aten, 'vendor_kernels_per_step': vendor,
            'non_native_kernels': names}


def main():
    args = parse()
    if args.comm_trace or int(os.environ.get('WORLD_SIZE', '1')) > 1:
        # multi-GPU runs always report the last step's bucket timeline (launch / done
        # relative to the end of the backward pass): the overlap is visible in the JSON
        args.comm_trace = True
        os.environ['HETU_COMM_TRACE'] = '1'
    os.environ['HETU_GRAD_WIRE'] = args.grad_wire
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1:
        import faulthandler
        # a rank silent for HETU_STALL_DUMP_S (240) s prints all its threads' stacks (then keeps running)
        faulthandler.dump_traceback_later(float(os.environ.get('HETU_STALL_DUMP_S', '240')), repeat=True,
                                          file=sys.stderr)
    local = int(os.environ.get('LOCAL_RANK', '0'))
    server = start_ps_server(world, local) if args.model == 'wdl' else None
    import torch
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.parallel import comm as C

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    assert world == args.gpus or world == 1, 'launch with --nproc-per-node == --gpus'
    if os.environ.get('HETU_DIST_BACKEND') == 'gloo':
        local = local % torch.cuda.device_count()     # multi-rank rehearsal on one GPU
    cpu_only = args.model == 'logreg' or args.rehearse_cpu
    if args.rehearse_cpu:
        args.dtype = 'fp32'
    if not cpu_only:
        torch.cuda.set_device(local)
    dev = torch.device('cpu') if cpu_only else torch.device('cuda', local)

    finish = None
    if args.model == 'resnet50':
        from hetu_61a7_amd.models import resnet50_imagenet
        B = args.batch or 256
        x = ht.Variable(name='x')
        y_ = ht.Variable(name='y_')
        loss, logits = resnet50_imagenet(x, y_, 1000)
        opt = ht.optim.MomentumOptimizer(learning_rate=0.1 / max(world, 1), momentum=0.9)
        train_op = opt.minimize(loss)
        kw = dict(mixed_precision=None if cpu_only else args.dtype, bucket_mb=args.bucket_mb, seed=1234,
                  zero=args.zero, timing='gpu' if args.op_profile else None)
        if world > 1:
            ex = ht.Executor({'train': [loss, train_op]}, dist_strategy=ht.dist.DataParallel('allreduce'), **kw)
        else:
            ex = ht.Executor({'train': [loss, train_op]}, ctx=ht.cpu(0) if cpu_only else ht.gpu(local), **kw)
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + rank)
        dt = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
        X = torch.randn((B, 3, 224, 224), generator=g, device=dev).to(dt)
        if not cpu_only:
            X = X.contiguous(memory_format=torch.channels_last)
        lab = torch.randint(0, 1000, (B,), generator=g, device=dev)
        Y = torch.nn.functional.one_hot(lab, 1000).to(dt)
        feed = {x: X, y_: Y}
        metric = 'samples/sec (whole node) ResNet-50 AllReduce'
        cfg = {'model': 'ResNet-50 (ImageNet-shaped, v1.5)', 'global_batch': B * world, 'seq_len': None,
               'image': '3x224x224', 'parallelism': 'dp%d' % world, 'optimizer': 'momentum-sgd',
               'per_gpu_batch': B}
        step = lambda: ex.run('train', feed_dict=feed)
        samples_per_step = B * world
    elif args.model == 'bert':
        from hetu_61a7_amd.models.bert import bert_bench
        step, samples_per_step, cfg, metric, finish = bert_bench(args, world, rank, local)
    elif args.model == 'logreg':
        from hetu_61a7_amd.models.cnn import logreg_bench
        step, samples_per_step, cfg, metric, finish = logreg_bench(args, world, rank, local)
    elif args.model == 'moe':
        from hetu_61a7_amd.models.moe import moe_top_bench
        step, samples_per_step, cfg, metric, finish = moe_top_bench(args, world, rank, local)
    else:
        from hetu_61a7_amd.models.ctr import wdl_criteo_bench
        step, samples_per_step, cfg, metric, finish = wdl_criteo_bench(args, world, rank, local)

    def barrier():
        if world > 1:
            C.world().barrier()

    _progress(rank, world, 'graph built, comm=%s' % (C.world().backend if C.world() is not None else 'none'))
    if world > 1 and not cpu_only and C.world() is not None and C.world().backend != 'hetu-rccl' and \
            os.environ.get('HETU_DIST_BACKEND') != 'gloo' and os.environ.get('HETU_COMM', 'native') != 'torch':
        # a multi-GPU number must come from the framework's own RCCL communicator: a silent
        # fallback to another backend would be measured and reported as if it were
        raise SystemExit('bench: %d ranks but the communicator is %r, not the native hetu-rccl (set '
                         'HETU_COMM=torch to measure torch.distributed on purpose)' % (world, C.world().backend))
    sync = (lambda: None) if cpu_only else torch.cuda.synchronize
    for i in range(args.warmup):
        step()
        _progress(rank, world, 'warmup step %d issued' % i)
    sync()
    _progress(rank, world, 'warmup done')
    from hetu_61a7_amd import kernels as K
    K.reset_dispatch_stats()     # vendor_calls / fallbacks below count the timed steps only
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier()
    sync()
    dt_s = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt_s], dtype=torch.float64, device=dev)
        C.world().all_reduce(t, 'max')
        dt_s = float(t.item())
    ms = dt_s * 1000.0 / args.steps
    if args.op_profile and args.model == 'resnet50' and rank == 0:
        s = ex.logOut(args.op_profile + '.node', log_level='node', clear=False, name='train')
        t = ex.logOut(args.op_profile, log_level='type', name='train')
        print('op-type ms/step:', sorted(t.items(), key=lambda kv: -kv[1])[:25], file=sys.stderr)
        from hetu_61a7_amd.ops.executor import layout_report
        print('non-channels-last 4D outputs:', layout_report(), file=sys.stderr)
    value = samples_per_step * args.steps / dt_s
    _progress(rank, world, 'timed steps done')
    cfg = dict(cfg)
    # hand-written-only accounting of the timed steps: library GEMM /
    # convolution calls and ops that left the native path, then a kernel census of one
    # more (untimed) step
    cfg['vendor_calls'] = dict(K.VENDOR_CALLS)
    if not cpu_only and args.model == 'resnet50':
        sub = ex.subexecutor['train']
        cfg['hipgraph'] = bool(sub.config.use_hipgraph and getattr(sub, 'graph', None) is not None
                               and getattr(sub.graph, 'graph', None) is not None)
    cfg['fallbacks'] = dict(K.FALLBACKS)
    if not cpu_only and os.environ.get('HETU_BENCH_CENSUS', '1') == '1':
        cfg.update(_kernel_census(step))
    if hasattr(step, 'extra'):
        ex_ = step.extra()
        cfg.update(ex_)
        if world > 1 and args.model == 'wdl':
            # every worker's HET cache hit rate and step breakdown (server wait = ps_wait)
            import torch.distributed as dist
            allx = [None] * world
            dist.all_gather_object(allx, {'cache_hit_rate': ex_.get('cache_hit_rate'),
                                          'step_breakdown_ms': ex_.get('step_breakdown_ms')})
            cfg['per_worker'] = allx
    if rank == 0 and os.environ.get('HETU_BENCH_PYPROF'):
        # host-side profile of extra (untimed) steady-state steps: where the Python time goes
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        n = int(os.environ.get('HETU_BENCH_PYPROF_STEPS', '50'))
        pr.enable()
        for _ in range(n):
            step()
        sync()
        pr.disable()
        buf = io.StringIO()
        st = pstats.Stats(pr, stream=buf)
        buf.write('%d steps\n' % n)
        st.sort_stats('tottime').print_stats(45)
        st.sort_stats('cumulative').print_stats(45)
        with open(os.environ['HETU_BENCH_PYPROF'], 'w') as f:
            f.write(buf.getvalue())
    if world > 1 or args.comm_trace:
        cfg = dict(cfg)
        cfg['comm'] = C.world().backend if C.world() is not None else 'none'
        cfg['comm_stats'] = C.stats()
        cfg['grad_wire'] = args.grad_wire
        if args.comm_trace and args.model == 'resnet50':
            tr = [op.comm_trace() for op in ex.optimizer_ops('train')] if hasattr(ex, 'optimizer_ops') else []
            cfg['comm_trace_last_step'] = tr[0] if tr else []
    # devices actually used: ranks of a gloo rehearsal share the node's GPUs (8 WDL workers on
    # one MI355X are 8 workers, 1 GPU)
    # (the CPU rehearsal of the driver's N-rank line keeps N)
    n_dev = 0 if args.model == 'logreg' else world
    if not cpu_only and os.environ.get('HETU_DIST_BACKEND') == 'gloo':
        n_dev = min(world, torch.cuda.device_count())
    if n_dev != world and args.model != 'logreg':
        cfg = dict(cfg)
        cfg['workers'] = world
    if rank == 0:
        out = {'metric': metric, 'value': round(value, 2), 'unit': 'tokens/s' if args.model == 'moe' else 'samples/s',
               'n_gpus': n_dev,
               'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3),
               'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
               'dtype': 'fp32' if cpu_only else args.dtype, 'data': 'synthetic (random-init weights)', 'config': cfg}
        print(json.dumps(out), flush=True)
    if rank == 0 and os.environ.get('HETU_AUTOTUNE_DUMP'):
        from hetu_61a7_amd.kernels import autotune
        autotune.dump(os.environ['HETU_AUTOTUNE_DUMP'])
    if rank == 0 and os.environ.get('HETU_AUTOTUNE_SAVE'):
        from hetu_61a7_amd.kernels import autotune
        autotune.save(os.environ['HETU_AUTOTUNE_SAVE'])
    if finish is not None:
        finish()
    if server is not None:
        server.wait(timeout=120)
    if world > 1:
        C.destroy()


if __name__ == '__main__':
    main()
