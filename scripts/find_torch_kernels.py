"""Which GPU kernels of one steady-state training step are not hand-written?

Runs a few steps of a bench model, profiles the last one with torch.profiler
(kineto/roctracer) and prints every device kernel that is neither a ``hetu::``
kernel nor a vendor GEMM/convolution library kernel, with the Python frame of
the graph op that launched it (the executor op's ``compute``).

    python scripts/find_torch_kernels.py --model resnet50 --batch 32
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VENDOR = ('Cijk', 'igemm', 'ck::', 'SubTensorOp', 'naive_conv', 'MIOpen', 'miopen', '__amd_rocclr', 'Custom_Cijk',
          'gridwise', 'kernel_batched_gemm', 'kernel_gemm')


def classify(name):
    if 'at::native' in name or 'c10::' in name:
        return 'torch'
    if any(v in name for v in VENDOR):
        return 'vendor'
    return 'hetu'   # hetu:: kernels and the library's file-local (anonymous-namespace) ones


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--model', default='resnet50', choices=['resnet50', 'bert', 'moe', 'wdl'])
    p.add_argument('--batch', type=int, default=None)
    p.add_argument('--steps', type=int, default=3)
    p.add_argument('--tiny', action='store_true', help='bert: the 2-layer config of tests/test_native_dispatch_gpu.py')
    a = p.parse_args()
    os.environ['HETU_PROFILE_OPS'] = '1'
    if a.model == 'wdl':
        # the PS server process, started before anything in this process touches the GPU
        import bench
        server = bench.start_ps_server(1, 0)
    import torch
    from torch.profiler import profile, ProfilerActivity
    sys.argv = ['bench.py', '--model', a.model, '--steps', '1', '--warmup', '0'] + \
        (['--batch', str(a.batch)] if a.batch else [])
    import bench
    args = bench.parse()
    if a.tiny:
        from hetu_61a7_amd.models.bert import BertConfig
        args.bert_config = BertConfig(vocab_size=8192, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                      intermediate_size=1024, max_position_embeddings=128)
        args.bert_config.seq_len = 128
        args.batch = 8
    import hetu_61a7_amd as ht  # noqa: F401
    step = _build(args)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    from hetu_61a7_amd.utils import hipgraph
    hipgraph.FORCE_EAGER[0] += 1      # an eager step: a graph replay would hide its kernels
    with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    hipgraph.FORCE_EAGER[0] -= 1
    counts = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    for e in prof.events():
        if e.device_type.name != 'CUDA' and getattr(e, 'device_type', None) is not None and \
                str(e.device_type) != 'DeviceType.CUDA':
            continue
        cls = classify(e.name)
        counts[cls] += 1
        if cls == 'torch':
            frames = []
            ev = e.cpu_parent if hasattr(e, 'cpu_parent') else None
            while ev is not None and len(frames) < 1:
                st = [s for s in (ev.stack or []) if 'hetu_61a7_amd' in s]
                if st:
                    frames.append(st[0])
                ev = ev.cpu_parent
            where[e.name[:110]][frames[0] if frames else '?'] += 1
    # attribute through the launching CPU op: aten ops whose device kernels are torch's
    for e in prof.events():
        ks = getattr(e, 'kernels', None) or []
        for k in ks:
            if classify(k.name) == 'torch':
                chain, ev = [], e
                while ev is not None:                  # aten op chain up to the graph op's range
                    chain.append(ev.name)
                    if ev.name.startswith('hetu_op:'):
                        break
                    ev = ev.cpu_parent
                where['%s <- %s' % (k.name[:70], e.name)][' < '.join(chain[::-1][:4])] += 1
    print('kernel classes in one step:', dict(counts))
    for name, fr in sorted(where.items(), key=lambda kv: -sum(kv[1].values())):
        print('%4d  %s' % (sum(fr.values()), name))
        for f, c in fr.most_common(3):
            print('        %4d  %s' % (c, f))
    if a.model == 'wdl':
        from hetu_61a7_amd.ps import worker
        worker.worker_finish()
        server.wait(timeout=60)
        for f, n in fr.most_common(4):
            print('        %3d  %s' % (n, f))


def _build(args):
    import torch
    import hetu_61a7_amd as ht
    if args.model == 'resnet50':
        from hetu_61a7_amd.models import resnet50_imagenet
        B = args.batch or 32
        x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
        loss, _ = resnet50_imagenet(x, y_, 1000)
        train = ht.optim.MomentumOptimizer(learning_rate=0.1, momentum=0.9).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=1)
        X = torch.randn((B, 3, 224, 224), device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
        Y = torch.nn.functional.one_hot(torch.randint(0, 1000, (B,), device='cuda'), 1000).bfloat16()
        return lambda: ex.run('train', feed_dict={x: X, y_: Y})
    if args.model == 'bert':
        from hetu_61a7_amd.models.bert import bert_bench
        return bert_bench(args, 1, 0, 0)[0]
    if args.model == 'moe':
        from hetu_61a7_amd.models.moe import moe_top_bench
        return moe_top_bench(args, 1, 0, 0)[0]
    from hetu_61a7_amd.models.ctr import wdl_criteo_bench
    return wdl_criteo_bench(args, 1, 0, 0)[0]


if __name__ == '__main__':
    main()
