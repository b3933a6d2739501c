"""BERT-base GEMM shapes (fwd / dgrad / wgrad, B*S = 8192): hand-written MFMA
kernel vs hipBLASLt (torch.matmul), TFLOP/s."""
import torch
from hetu_61a7_amd.kernels import gemm_mfma as G


def timeit(f, it=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


T = 8192
shapes = []
for (din, dout) in [(768, 2304), (768, 768), (768, 3072), (3072, 768)]:
    shapes += [('fwd', T, dout, din, False, False), ('dgrad', T, din, dout, False, True),
               ('wgrad', din, dout, T, True, False)]
shapes += [('mlm_fwd', T, 30522, 768, False, True), ('mlm_dgrad', T, 768, 30522, False, False),
           ('mlm_wgrad', 30522, 768, T, True, False)]
tot_h = tot_v = tot_b = 0.0
for name, M, N, K, ta, tb in shapes:
    a = torch.randn(K, M, device='cuda').bfloat16().t() if ta else torch.randn(M, K, device='cuda').bfloat16()
    b = torch.randn(N, K, device='cuda').bfloat16().t() if tb else torch.randn(K, N, device='cuda').bfloat16()
    out32 = torch.empty(M, N, device='cuda', dtype=torch.float32)
    th = timeit(lambda: G.gemm(a, b)) if G.gemm(a, b) is not None else float('nan')
    tv = timeit(lambda: a @ b)
    fl = 2 * M * N * K
    best = min(th, tv)
    tot_h += th
    tot_v += tv
    tot_b += best
    print('%-9s M=%5d N=%5d K=%5d ta=%d tb=%d  hip %6.1f us %6.0f TF | vendor %6.1f us %6.0f TF' %
          (name, M, N, K, ta, tb, th * 1e3, fl / th / 1e9, tv * 1e3, fl / tv / 1e9), flush=True)
print('sum per layer-set: hip %.3f ms  vendor %.3f ms  best %.3f ms' % (tot_h, tot_v, tot_b))
