"""Which kernels does torch's MIOpen convolution_backward (data / weight) launch for
channels-last bf16 operands (ResNet-50 layer1 3x3, bs 256)?"""
import torch
from torch.profiler import profile, ProfilerActivity

CL = torch.channels_last
for (n, c, h, k) in [(256, 64, 56, 64), (256, 256, 14, 256)]:
    x = torch.randn(n, c, h, h, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(k, c, 3, 3, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(n, k, h, h, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    for mask in ([True, False, False], [False, True, False]):
        for _ in range(3):
            torch.ops.aten.convolution_backward(g, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, mask)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            r = torch.ops.aten.convolution_backward(g, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, mask)
            torch.cuda.synchronize()
        out = r[0] if mask[0] else r[1]
        print('shape', (n, c, h, k), 'dgrad' if mask[0] else 'wgrad', 'out CL:', out.is_contiguous(memory_format=CL),
              'dtype', out.dtype)
        for e in prof.key_averages():
            if e.device_time_total > 0:
                print('   %-90s %8.1f us x%d' % (e.key[:90], e.device_time_total, e.count))
