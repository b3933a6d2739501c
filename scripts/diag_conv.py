"""Which kernels does each conv pass launch (MIOpen via torch) for channels-last bf16
ResNet-50 shapes, and how long does each take.  Usage: python scripts/diag_conv.py"""
import torch
from torch.profiler import profile, ProfilerActivity
from hetu_61a7_amd.kernels import conv as KC

CL = torch.channels_last
shapes = [  # N, Cin, H, Cout, k, stride, pad
    (256, 256, 56, 64, 1, 1, 0), (256, 64, 56, 64, 3, 1, 1), (256, 64, 56, 256, 1, 1, 0),
    (256, 128, 28, 128, 3, 1, 1), (256, 512, 14, 256, 1, 1, 0)]
for (N, Ci, H, Co, k, s, p) in shapes:
    x = torch.randn(N, Ci, H, H, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = torch.randn(Co, Ci, k, k, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    y = KC.conv2d(x, w, None, (s, s), (p, p))
    g = torch.randn_like(y).contiguous(memory_format=CL)
    for _ in range(3):
        KC.conv2d(x, w, None, (s, s), (p, p)); KC.conv2d_backward_data(g, w, x.shape, (s, s), (p, p))
        KC.conv2d_backward_filter(g, x, w.shape, (s, s), (p, p))
    torch.cuda.synchronize()
    for name, f in [('fwd', lambda: KC.conv2d(x, w, None, (s, s), (p, p))),
                    ('dgrad', lambda: KC.conv2d_backward_data(g, w, x.shape, (s, s), (p, p))),
                    ('wgrad', lambda: KC.conv2d_backward_filter(g, x, w.shape, (s, s), (p, p)))]:
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            out = f(); torch.cuda.synchronize()
        ks = [(e.name[:70], e.device_time) for e in prof.events() if e.device_time > 0]
        fl = 2 * N * Co * Ci * k * k * (y.shape[2] * y.shape[3])
        tot = sum(t for _, t in ks)
        print('%s %-5s out_cl=%s total=%.1fus %.0f TFLOP/s' % ((N, Ci, H, Co, k, s), name,
              out.is_contiguous(memory_format=CL), tot, fl / tot / 1e6))
        for n, t in ks:
            print('      %8.1fus %s' % (t, n))
