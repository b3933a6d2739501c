"""Which kernels does each VENDOR conv pass launch (MIOpen via torch) for
channels-last bf16 ResNet-50 shapes, and how long each takes."""
import torch
import torch.nn.functional as F
from torch.profiler import profile, ProfilerActivity

CL = torch.channels_last
shapes = [(256, 64, 56, 64, 3, 1, 1), (256, 128, 28, 128, 3, 1, 1), (256, 256, 56, 64, 1, 1, 0)]
for (N, Ci, H, Co, k, s, p) in shapes:
    x = torch.randn(N, Ci, H, H, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = torch.randn(Co, Ci, k, k, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    y = F.conv2d(x, w, None, s, p)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    xs = torch.empty_like(x)
    cands = [('fwd', lambda: F.conv2d(x, w, None, s, p)),
             ('dgrad_cb', lambda: torch.ops.aten.convolution_backward(g, xs, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False])[0]),
             ('dgrad_ct', lambda: F.conv_transpose2d(g, w, None, s, p)),
             ('wgrad_cb', lambda: torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False])[1])]
    for _ in range(3):
        for _, f in cands:
            f()
    torch.cuda.synchronize()
    for name, f in cands:
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            out = f(); torch.cuda.synchronize()
        ks = [(e.name[:80], e.device_time) for e in prof.events() if e.device_time > 0]
        print('%s %-9s out_cl=%s total=%.1fus' % ((N, Ci, H, Co, k, s), name,
              out.is_contiguous(memory_format=CL), sum(t for _, t in ks)))
        for n, t in ks:
            print('      %8.1fus %s' % (t, n))
