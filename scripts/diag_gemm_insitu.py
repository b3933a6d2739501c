"""Why is the hand-written GEMM slower inside the BERT step than in the tile bench?
Times the BERT-base GEMM shapes (tokens = 8192) hot (back-to-back) and cold (a 1 GiB
buffer is rewritten between calls, evicting L2 and MALL), without and with the fused
bias / GELU epilogue, against hipBLASLt; prints the hipBLASLt kernel names (macro tile).

    python scripts/diag_gemm_insitu.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hetu_61a7_amd.kernels import gemm_mfma as G

flush = torch.empty(256 << 20, dtype=torch.float32, device='cuda')


def timeit(fn, cold, reps=8):
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(reps):
        if cold:
            flush.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    return tot / reps * 1e3


shapes = [('qkv', 8192, 2304, 768), ('attn_out', 8192, 768, 768), ('ffn1', 8192, 3072, 768),
          ('ffn2', 8192, 768, 3072), ('vocab', 8192, 30528, 768)]
print('%-9s %-9s %-5s %9s %9s %9s %9s' % ('shape', 'epi', 'tile', 'hot us', 'cold us', 'hot TF', 'cold TF'))
for name, M, N, K in shapes:
    a = torch.randn(M, K, device='cuda').bfloat16()
    b = (torch.randn(K, N, device='cuda') * 0.05).bfloat16()
    bias = torch.randn(N, device='cuda')
    fl = 2.0 * M * N * K
    for epi, kw in [('none', {}), ('bias', dict(bias=bias)), ('bias+gelu', dict(bias=bias, act='gelu'))]:
        for t in G.TILES:
            h = timeit(lambda: G.gemm(a, b, tile=t, **kw), False)
            c = timeit(lambda: G.gemm(a, b, tile=t, **kw), True)
            print('%-9s %-9s %-5s %9.1f %9.1f %9.0f %9.0f' % (name, epi, t, h, c, fl / h / 1e6, fl / c / 1e6),
                  flush=True)
        bb = bias.bfloat16()
        vfn = (lambda: torch.mm(a, b)) if epi == 'none' else (lambda: torch.addmm(bb, a, b))
        h, c = timeit(vfn, False), timeit(vfn, True)
        print('%-9s %-9s %-5s %9.1f %9.1f %9.0f %9.0f' % (name, epi, 'blas', h, c, fl / h / 1e6, fl / c / 1e6),
              flush=True)
    del a, b

# hipBLASLt kernel names for the same shapes
from torch.profiler import profile, ProfilerActivity
names = {}
for name, M, N, K in shapes:
    a = torch.randn(M, K, device='cuda').bfloat16()
    b = torch.randn(K, N, device='cuda').bfloat16()
    torch.mm(a, b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as p:
        torch.mm(a, b)
        torch.cuda.synchronize()
    ks = [e.name for e in p.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    print('%-9s blas kernels: %s' % (name, ' | '.join(k[:140] for k in ks)), flush=True)
