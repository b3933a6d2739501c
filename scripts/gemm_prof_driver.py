"""Runs a few MFMA GEMM shapes back to back (random bf16 operands) for rocprofv3
counter passes: python scripts/gemm_prof_driver.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hetu_61a7_amd.kernels import gemm_mfma as G

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
shapes = [(8192, 8192, 8192, 0, 1, 1), (8192, 3072, 768, 0, 0, 0), (50176, 256, 1024, 0, 1, 0),
          (802816, 256, 64, 0, 1, 0)]
for M, N, K, ta, tb, tile in shapes:
    a = torch.randn(K, M, device='cuda').bfloat16().t() if ta else torch.randn(M, K, device='cuda').bfloat16()
    b = torch.randn(N, K, device='cuda').bfloat16().t() if tb else torch.randn(K, N, device='cuda').bfloat16()
    for _ in range(reps):
        G.gemm(a, b, tile=tile)
    torch.cuda.synchronize()
    del a, b
print('done')
