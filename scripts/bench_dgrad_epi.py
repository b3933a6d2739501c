"""Micro-benchmark of the output-bound 1x1 data-gradient epilogues of ResNet-50 (batch 256):
plain / + gradient join (Cin) / + BN-backward sums / + masked store, per tile, in us and
effective HBM TB/s.  Run on the GPU box: python scripts/bench_dgrad_epi.py"""
import sys
import torch

sys.path.insert(0, '.')
from hetu_61a7_amd.kernels import conv_igemm as CI  # noqa: E402

CL = torch.channels_last
DEV = 'cuda'
# (g [N, K, H, W], w [K, C, 1, 1]) -> dx [N, C, H, W]
SHAPES = [((256, 64, 56, 56), (64, 256, 1, 1)),
          ((256, 128, 28, 28), (128, 512, 1, 1)),
          ((256, 256, 14, 14), (256, 1024, 1, 1)),
          ((256, 256, 56, 56), (256, 64, 1, 1))]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def roofline():
    """HBM ceilings on the largest epilogue tensor (256x256x56x56 bf16): copy, read, write"""
    a = torch.randn(256 * 256 * 56 * 56, device=DEV).bfloat16()
    b = torch.empty_like(a)
    nb = a.numel() * 2
    us = timeit(lambda: b.copy_(a))
    print('%-20s %8.1f us %6.2f TB/s' % ('copy (r+w)', us, 2 * nb / us / 1e6))
    af = a.view(torch.float32)
    us = timeit(lambda: af.sum())
    print('%-20s %8.1f us %6.2f TB/s' % ('read (sum)', us, nb / us / 1e6))
    us = timeit(lambda: b.fill_(1.0))
    print('%-20s %8.1f us %6.2f TB/s' % ('write (fill)', us, nb / us / 1e6), flush=True)


def main():
    torch.manual_seed(0)
    roofline()
    if '--roofline' in sys.argv:
        return
    for gs, ws in SHAPES:
        N, K, H, W = gs
        C = ws[1]
        xs = (N, C, H, W)
        g = torch.randn(gs, device=DEV).bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(ws, device=DEV) * 0.05).bfloat16().contiguous(memory_format=CL)
        xb = torch.randn(xs, device=DEV).bfloat16().contiguous(memory_format=CL)
        acc = torch.randn(xs, device=DEV).bfloat16().contiguous(memory_format=CL)
        mask = torch.randint(0, 256, (xb.numel() // 8,), device=DEV, dtype=torch.int32).to(torch.uint8)
        sums = torch.zeros(2 * C, device=DEV)
        R = CI.bn_sum_replicas(N * H * W)
        sumsr = torch.zeros(R * 2 * C, device=DEV)
        gb, ob = g.numel() * 2, xb.numel() * 2
        for tile in (0, 2, 3):
            if tile == 2 and C % 64:
                continue
            variants = [('plain', None, None, gb + ob),
                        ('join', acc, None, gb + 2 * ob),
                        ('join+bn', acc, (sums, xb, mask), gb + 3 * ob + ob // 16),
                        ('join+bn+mstore', acc, (sums, xb, mask, True), gb + 3 * ob + ob // 16),
                        ('bn', None, (sums, xb, mask), gb + 2 * ob + ob // 16),
                        ('join+bn+ms r%d' % R, acc, (sumsr, xb, mask, True), gb + 3 * ob + ob // 16),
                        ('bn r%d' % R, None, (sumsr, xb, mask), gb + 2 * ob + ob // 16)]
            for name, a, bnb, byts in variants:
                f = lambda: CI.try_backward_data(g, w, xs, (1, 1), (0, 0), acc=a, tile=tile, bnb=bnb)  # noqa: E731
                if f() is None:
                    continue
                us = timeit(f)
                print('%-20s %-20s tile=%d %-16s %8.1f us %6.2f TB/s' % (gs, ws, tile, name, us, byts / us / 1e6),
                      flush=True)


if __name__ == '__main__':
    main()
