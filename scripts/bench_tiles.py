"""A/B of the MFMA GEMM tile configurations (gemm.hip: 0 = 128x128 / 4 waves,
1 = 256x256 / 8 waves phase-interleaved) against hipBLASLt / MIOpen on plain
GEMMs and on the ResNet-50 3x3 / strided convolutions (bs 256, bf16, NHWC).
Random operands (zero-filled data over-reports MFMA throughput).

    python scripts/bench_tiles.py [out.txt]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from hetu_61a7_amd.kernels import gemm_mfma as G, conv_igemm as CI

CL = torch.channels_last
out_path = sys.argv[1] if len(sys.argv) > 1 else None
lines = []


def emit(s):
    print(s, flush=True)
    lines.append(s)


def timeit(fn, reps=10):
    fn()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


emit('# GEMM (TF/s): tile0 = 128x128 2-stage, tile1 = 256x256 8-wave, tile2 = 128x128 3-stage, blas = hipBLASLt (torch.mm)')
for (M, N, K, ta, tb) in [(4096, 4096, 4096, 0, 0), (4096, 4096, 4096, 0, 1), (8192, 8192, 8192, 0, 1),
                          (8192, 3072, 768, 0, 0), (8192, 768, 3072, 0, 0), (768, 3072, 8192, 1, 0),
                          (50176, 1024, 256, 0, 1), (50176, 256, 1024, 0, 1), (200704, 512, 128, 0, 1),
                          (802816, 256, 64, 0, 1)]:
    a = torch.randn(K, M, device='cuda').bfloat16().t() if ta else torch.randn(M, K, device='cuda').bfloat16()
    b = torch.randn(N, K, device='cuda').bfloat16().t() if tb else torch.randn(K, N, device='cuda').bfloat16()
    fl = 2.0 * M * N * K
    ref = a.float() @ b.float()
    res = {}
    for t in G.TILES:
        y = G.gemm(a, b, tile=t)
        err = rel(y, ref)
        ms = timeit(lambda: G.gemm(a, b, tile=t))
        res['tile%d' % t] = (ms, err)
    ms = timeit(lambda: torch.mm(a, b))
    res['blas'] = (ms, 0.0)
    emit('M %6d N %5d K %5d %s%s  ' % (M, N, K, 'T' if ta else 'N', 'T' if tb else 'N') +
         '  '.join('%s %.3f ms %5.0f TF (err %.1e)' % (k, v[0], fl / v[0] / 1e9, v[1]) for k, v in res.items()))
    del a, b, ref

emit('# ResNet-50 convolutions, bs 256 (ms): tile0 / tile1 / tile2 / vendor (MIOpen)')
N = 256
for (ci, H, co, k, st, p) in [(64, 56, 64, 3, 1, 1), (128, 28, 128, 3, 1, 1), (128, 56, 128, 3, 2, 1),
                              (256, 14, 256, 3, 1, 1), (256, 28, 256, 3, 2, 1), (512, 7, 512, 3, 1, 1),
                              (512, 14, 512, 3, 2, 1), (256, 56, 512, 1, 2, 0), (1024, 14, 2048, 1, 2, 0),
                              (256, 56, 64, 1, 1, 0), (64, 56, 256, 1, 1, 0)]:
    x = torch.randn(N, ci, H, H, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(co, ci, k, k, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    y = F.conv2d(x, w, None, st, p)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    Ho = y.shape[2]
    fl = 2.0 * N * Ho * Ho * co * ci * k * k
    row = []
    for name, fns in [('fwd', {t: (lambda t=t: CI.try_forward(x, w, (st, st), (p, p), tile=t)) for t in G.TILES}),
                      ('dgrad', {t: (lambda t=t: CI.try_backward_data(g, w, x.shape, (st, st), (p, p), tile=t))
                                 for t in G.TILES}),
                      ('wgrad', {t: (lambda t=t: CI.try_backward_filter(g, x, w.shape, (st, st), (p, p),
                                                                         accumulate=False, tile=t))
                                 for t in G.TILES})]:
        outs = {t: f() for t, f in fns.items()}
        err = rel(outs[1], outs[0]) if outs[0] is not None and outs[1] is not None else float('nan')
        tms = {t: timeit(f) for t, f in fns.items()}
        if name == 'fwd':
            v = timeit(lambda: F.conv2d(x, w, None, st, p))
        elif name == 'dgrad':
            v = timeit(lambda: torch.ops.aten.convolution_backward(g, x, w, None, [st, st], [p, p], [1, 1], False,
                                                                   [0, 0], 1, [True, False, False]))
        else:
            v = timeit(lambda: torch.ops.aten.convolution_backward(g, x, w, None, [st, st], [p, p], [1, 1], False,
                                                                   [0, 0], 1, [False, True, False]))
        row.append('%s %s/%.3f (%4.0f TF best, t1-vs-t0 %.0e)' % (
            name, '/'.join('%.3f' % tms[t] for t in G.TILES), v, fl / min(tms.values()) / 1e9, err))
    emit('cin %4d H %3d cout %4d k%d s%d | ' % (ci, H, co, k, st) + ' | '.join(row))
    del x, w, y, g

if out_path:
    with open(out_path, 'w') as f:
        f.write('\n'.join(lines) + '\n')
