"""ResNet-50 stem (7x7 / stride 2 / pad 3, 3 -> 64 channels, bs 256, bf16 NHWC):
the direct convolution vs the space-to-depth rewrite (2x2 pixel blocks folded
into channels: a 4x4 / stride 1 convolution over 12 (padded 16) channels), forward
and weight gradient, MIOpen and the hand-written implicit GEMM.

    python scripts/bench_stem.py [out.txt]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from hetu_61a7_amd.kernels import conv as KC, conv_igemm as CI

CL = torch.channels_last
lines = []


def emit(s):
    print(s, flush=True)
    lines.append(s)


def timeit(f, reps=10):
    f()
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


def s2d_input(x, cpad):
    """[N,3,224,224] CL -> z [N, cpad, 115, 115] CL with z[.., (p,q,c), i, j] = xpad[2i+p, 2j+q, c]"""
    n, c, h, w = x.shape
    xp = F.pad(x, (3, 3, 3, 3))                          # 230 x 230
    z = xp.permute(0, 2, 3, 1).reshape(n, h // 2 + 3, 2, w // 2 + 3, 2, c)   # n, i, p, j, q, c
    z = z.permute(0, 1, 3, 2, 4, 5).reshape(n, h // 2 + 3, w // 2 + 3, 4 * c)
    if cpad > 4 * c:
        z = F.pad(z, (0, cpad - 4 * c))
    return z.permute(0, 3, 1, 2)                          # channels-last view


def s2d_weight(w, cpad):
    """[64,3,7,7] -> [64, cpad, 4, 4]: w'[o, (p,q,c), a, b] = w[o, c, 2a+p, 2b+q] (0 past 7)"""
    o, c, kh, kw = w.shape
    wp = F.pad(w, (0, 1, 0, 1))                          # 8 x 8
    w2 = wp.reshape(o, c, 4, 2, 4, 2).permute(0, 3, 5, 1, 2, 4).reshape(o, 4 * c, 4, 4)
    if cpad > 4 * c:
        w2 = F.pad(w2, (0, 0, 0, 0, 0, cpad - 4 * c))
    return w2.contiguous(memory_format=CL)


def s2d_weight_back(w2, c=3):
    """inverse of s2d_weight (for the weight gradient)"""
    o = w2.shape[0]
    w8 = w2[:, :4 * c].reshape(o, 2, 2, c, 4, 4).permute(0, 3, 4, 1, 5, 2).reshape(o, c, 8, 8)
    return w8[:, :, :7, :7]


N = 256
x = torch.randn(N, 3, 224, 224, device='cuda').bfloat16().contiguous(memory_format=CL)
w = (torch.randn(64, 3, 7, 7, device='cuda') * 0.1).bfloat16().contiguous(memory_format=CL)
ref = F.conv2d(x.float(), w.float(), None, 2, 3)
g = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
fl = 2.0 * N * 112 * 112 * 64 * 147
emit('# stem forward (ms, TF/s of the 147-tap convolution)')
t = timeit(lambda: F.conv2d(x, w, None, 2, 3))
emit('miopen 7x7 s2 C3         %.3f ms %5.0f TF  err %.1e' % (t, fl / t / 1e9, rel(F.conv2d(x, w, None, 2, 3), ref)))
t = timeit(lambda: KC.conv2d(x, w, None, (2, 2), (3, 3)))
emit('framework choice         %.3f ms %5.0f TF' % (t, fl / t / 1e9))
for cp in (12, 16):
    z = s2d_input(x, cp).contiguous(memory_format=CL)
    w2 = s2d_weight(w, cp)
    tz = timeit(lambda: s2d_input(x, cp).contiguous(memory_format=CL))
    y = F.conv2d(z, w2)
    t = timeit(lambda: F.conv2d(z, w2))
    emit('s2d C%-2d  transform %.3f | miopen 4x4 s1 %.3f ms (%5.0f TF) err %.1e' % (cp, tz, t, fl / t / 1e9, rel(y, ref)))
    if cp % 8 == 0:
        for tile in (0, 1):
            yh = CI.try_forward(z, w2, (1, 1), (0, 0), tile=tile)
            if yh is not None:
                t = timeit(lambda: CI.try_forward(z, w2, (1, 1), (0, 0), tile=tile))
                emit('         hip tile%d 4x4 s1 %.3f ms (%5.0f TF) err %.1e' % (tile, t, fl / t / 1e9, rel(yh, ref)))

emit('# stem weight gradient')
xf = x.float().requires_grad_(True)
wf = w.float().requires_grad_(True)
F.conv2d(xf, wf, None, 2, 3).backward(g.float())
dw_ref = wf.grad
vw = lambda: torch.ops.aten.convolution_backward(g, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                  [False, True, False])[1]
t = timeit(vw)
emit('miopen 7x7 s2 C3         %.3f ms %5.0f TF  err %.1e' % (t, fl / t / 1e9, rel(vw(), dw_ref)))
t = timeit(lambda: KC.conv2d_backward_filter(g, x, w.shape, (2, 2), (3, 3)))
emit('framework choice         %.3f ms %5.0f TF' % (t, fl / t / 1e9))
for cp in (12, 16):
    z = s2d_input(x, cp).contiguous(memory_format=CL)
    w2 = s2d_weight(w, cp)
    v2 = lambda: torch.ops.aten.convolution_backward(g, z, w2, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                      [False, True, False])[1]
    t = timeit(v2)
    emit('s2d C%-2d miopen 4x4 s1     %.3f ms (%5.0f TF) err %.1e' % (cp, t, fl / t / 1e9,
                                                                    rel(s2d_weight_back(v2().float()), dw_ref)))
    if cp % 8 == 0:
        for tile in (0, 1):
            d = CI.try_backward_filter(g, z, w2.shape, (1, 1), (0, 0), accumulate=False, tile=tile)
            if d is not None:
                t = timeit(lambda: CI.try_backward_filter(g, z, w2.shape, (1, 1), (0, 0), accumulate=False,
                                                          tile=tile))
                emit('        hip tile%d 4x4 s1   %.3f ms (%5.0f TF) err %.1e' % (tile, t, fl / t / 1e9,
                                                                          rel(s2d_weight_back(d), dw_ref)))
if len(sys.argv) > 1:
    with open(sys.argv[1], 'w') as f:
        f.write('\n'.join(lines) + '\n')
