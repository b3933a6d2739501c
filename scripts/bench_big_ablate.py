"""Ablations of the 256x256 MFMA GEMM kernel (gemm.hip g_big_variant) at 4096^3 / 8192^3
NT bf16: which part of the phase loop costs the time.  Timing-only (results of the
ablated variants are wrong by construction)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hetu_61a7_amd.kernels import gemm_mfma as G, fn, I32

setv = fn('hetu_gemm_big_variant', [I32], restype=I32)


def timeit(f, reps=10):
    f(); f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for n in (4096, 8192):
    a = torch.randn(n, n, device='cuda').bfloat16()
    b = torch.randn(n, n, device='cuda').bfloat16().t()
    fl = 2.0 * n ** 3
    for v, name in [(0, 'full'), (1, 'no stagger'), (4, 'no setprio'), (8, 'no DMA'), (16, 'no MFMA'),
                    (24, 'no DMA no MFMA'), (9, 'no DMA no stagger')]:
        setv(v)
        ms = timeit(lambda: G.gemm(a, b, tile=1))
        print('n %d  %-20s %.3f ms  %5.0f TF' % (n, name, ms, fl / ms / 1e9), flush=True)
    setv(0)
