"""Which graph ops of the Transformer example's training step launch PyTorch kernels?
Profiles one steady-state step with per-op record_function ranges (HETU_PROFILE_OPS=1)
and prints each at::native kernel with the hetu op range it ran under."""
import collections
import os
import sys

os.environ['HETU_PROFILE_OPS'] = '1'
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402

import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.transformer import Transformer, TransformerConfig, synthetic_batch  # noqa: E402


def main():
    hp = TransformerConfig(vocab_size=2048, d_model=256, d_ff=512, num_blocks=2, num_heads=4, maxlen1=100,
                           maxlen2=100, dropout_rate=0.1, batch_size=8)
    xs, xm, ys, ym, lab = (ht.Variable(name=n) for n in ('xs', 'xm', 'ys', 'ym', 'lab'))
    loss, _ = Transformer(hp).train(xs, xm, ys, ym, lab)
    train = ht.optim.AdamOptimizer(1e-4).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), mixed_precision='bf16', seed=1)
    b = synthetic_batch(hp)
    fd = {xs: b['xs'], xm: b['src_mask'], ys: b['ys'], ym: b['tgt_mask'], lab: b['labels']}
    for _ in range(3):
        ex.run('train', feed_dict=fd)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        ex.run('train', feed_dict=fd)
        torch.cuda.synchronize()
    ranges = [(e.time_range.start, e.time_range.end, e.name) for e in prof.events()
              if e.name.startswith('hetu_op:')]
    cpu_ops = [e for e in prof.events() if 'CUDA' not in str(e.device_type) and e.name.startswith('aten::')]
    found = collections.Counter()
    for e in prof.events():
        if 'CUDA' in str(e.device_type) and 'at::native' in e.name:
            # the launching aten op (CPU side) correlates by the kernel's parent
            par = getattr(e, 'cpu_parent', None)
            owner = '?'
            t = par.time_range.start if par is not None else None
            if t is not None:
                for s, en, nm in ranges:
                    if s <= t <= en:
                        owner = nm
            found[(owner, par.name if par is not None else '?', e.name[:70])] += 1
    for k, v in sorted(found.items(), key=lambda kv: -kv[1]):
        print(v, k)
    print('aten cpu ops:', collections.Counter(e.name for e in cpu_ops).most_common(30))


if __name__ == '__main__':
    main()
