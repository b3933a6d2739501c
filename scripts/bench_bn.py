"""BatchNorm kernel bandwidth over the ResNet-50 (bs 256, bf16, channels-last)
BN shapes, against a plain device copy of the same tensor, with a sweep of the
launch-shape tunables (hetu_bn_tune: partial-statistics block target, streaming
block cap, minimum row passes per thread).  GB/s counts the compulsory HBM bytes of each op:
  stats  = read x                      (col_sums: partial + merge)
  fwd    = read x (stats) + read x + write y   (bn_forward, ReLU)
  bwd    = read dy,x (partial) + read dy,x + write dx   (bn_backward, ReLU mode 2)

    python scripts/bench_bn.py [out.txt]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hetu_61a7_amd.kernels import norm as KN, fn, I32

CL = torch.channels_last
N = 256
SHAPES = [(64, 112), (64, 56), (256, 56), (128, 56), (128, 28), (512, 28), (256, 28), (256, 14),
          (1024, 14), (512, 14), (512, 7), (2048, 7)]
out_path = sys.argv[1] if len(sys.argv) > 1 else None
lines = []
tune = fn('hetu_bn_tune', [I32, I32, I32])


def emit(s):
    print(s, flush=True)
    lines.append(s)


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run(label):
    tot = {'copy': 0.0, 'stats': 0.0, 'fwd': 0.0, 'bwd': 0.0}
    emit('# %s' % label)
    for C, H in SHAPES:
        x = torch.randn(N, C, H, H, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn_like(x)
        sc = torch.rand(C, device='cuda') + 0.5
        bi = torch.randn(C, device='cuda') * 0.1
        rm, rv = torch.zeros(C, device='cuda'), torch.ones(C, device='cuda')
        y, mu, istd = KN.bn_forward(x, sc, bi, rm, rv, 0.1, 1e-5, True, relu=True)
        nb = x.numel() * 2
        dst = torch.empty_like(x)
        t = {'copy': timeit(lambda: dst.copy_(x)),
             'stats': timeit(lambda: KN.col_sums(x)),
             'fwd': timeit(lambda: KN.bn_forward(x, sc, bi, rm, rv, 0.1, 1e-5, True, relu=True)),
             'bwd': timeit(lambda: KN.bn_backward(dy, y, x, sc, mu, istd, relu=True, bias=bi))}
        passes = {'copy': 2, 'stats': 1, 'fwd': 3, 'bwd': 5}
        for k in t:
            tot[k] += t[k]
        emit('C %4d H %3d %6.1f MB | ' % (C, H, nb / 1e6) + ' | '.join(
            '%s %.3f ms %4.0f GB/s' % (k, t[k], passes[k] * nb / t[k] / 1e6) for k in t))
        del x, dy, y, dst
    emit('total ms (one BN per shape): ' + ' '.join('%s %.3f' % kv for kv in tot.items()))


run('defaults (chunk target 512, apply cap 2048, min passes 16)')
for ct, cap, mp in [(1024, 2048, 1), (1024, 2048, 8), (1024, 2048, 16), (1024, 2048, 32), (2048, 2048, 16)]:
    tune(ct, cap, mp)
    run('chunk target %d, apply cap %d, min passes %d' % (ct, cap, mp))
tune(512, 2048, 16)
if out_path:
    with open(out_path, 'w') as f:
        f.write('\n'.join(lines) + '\n')
