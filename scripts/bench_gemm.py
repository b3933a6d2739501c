"""Hand-written MFMA GEMM / conv vs vendor (hipBLASLt / MIOpen via torch): TFLOP/s."""
import torch
import torch.nn.functional as F
from hetu_61a7_amd.kernels import gemm_mfma as G, conv_igemm as CI, conv as KC

CL = torch.channels_last


def timeit(f, it=20):
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


print('== GEMM (M,N,K,mode): hip vs torch TFLOP/s')
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072), (128, 2048, 2048)]:
    for ta, tb in [(False, False), (False, True), (True, False)]:
        a = torch.randn(K, M, device='cuda').bfloat16().t() if ta else torch.randn(M, K, device='cuda').bfloat16()
        b = torch.randn(N, K, device='cuda').bfloat16().t() if tb else torch.randn(K, N, device='cuda').bfloat16()
        th = timeit(lambda: G.gemm(a, b))
        tv = timeit(lambda: a @ b)
        fl = 2 * M * N * K
        print('%5d %5d %5d ta=%d tb=%d  hip %7.1f  vendor %7.1f' % (M, N, K, ta, tb, fl / th / 1e9, fl / tv / 1e9))

print('== ResNet-50 conv (N,C,H,K,k,s): us  hip vs MIOpen  (fwd / dgrad / wgrad)')
shapes = [(256, 64, 56, 64, 1, 1, 0), (256, 64, 56, 64, 3, 1, 1), (256, 64, 56, 256, 1, 1, 0),
          (256, 256, 56, 64, 1, 1, 0), (256, 128, 28, 128, 3, 1, 1), (256, 128, 56, 128, 3, 2, 1),
          (256, 256, 14, 256, 3, 1, 1), (256, 1024, 14, 256, 1, 1, 0), (256, 512, 7, 512, 3, 1, 1),
          (256, 2048, 7, 512, 1, 1, 0), (256, 256, 56, 512, 1, 2, 0)]
for (N, C, H, K, k, s, p) in shapes:
    x = torch.randn(N, C, H, H, device='cuda').bfloat16().contiguous(memory_format=CL)
    w = torch.randn(K, C, k, k, device='cuda').bfloat16().contiguous(memory_format=CL)
    y = F.conv2d(x, w, None, s, p)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    fl = 2 * N * K * C * k * k * y.shape[2] * y.shape[3]
    r = []
    for hip, vend in [(lambda: CI.try_forward(x, w, (s, s), (p, p)), lambda: F.conv2d(x, w, None, s, p)),
                      (lambda: CI.try_backward_data(g, w, x.shape, (s, s), (p, p)),
                       lambda: torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False])),
                      (lambda: CI.try_backward_filter(g, x, w.shape, (s, s), (p, p)),
                       lambda: torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]))]:
        th, tv = timeit(hip, 10), timeit(vend, 10)
        r.append('%6.0f/%6.0f (%4.0f/%4.0f TF)' % (th * 1e3, tv * 1e3, fl / th / 1e9, fl / tv / 1e9))
    print((N, C, H, K, k, s), ' | '.join(r))
