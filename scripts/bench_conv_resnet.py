"""Per-shape timing of every ResNet-50 (bs 256, bf16, NHWC) convolution pass
through the framework's autotuned dispatch: every hand-written candidate (implicit-GEMM
MFMA tiles 'hip*', halo-tile 'hip33', stem 'hip_stem', channel-padded 'hip_pad' for the
3-channel stem) is timed (MIOpen references: scripts/vendor_ref.py), with
achieved TFLOP/s and HBM GB/s (compulsory bytes) of the chosen one.

    python scripts/bench_conv_resnet.py [batch] [out.txt]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collections import Counter
import torch
import torch.nn.functional as F
from hetu_61a7_amd.kernels import conv as KC, autotune

CL = torch.channels_last
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
out_path = sys.argv[2] if len(sys.argv) > 2 else None


def resnet50_convs():
    s = [(3, 224, 64, 7, 2, 3)]                        # (Cin, H, Cout, k, stride, pad)
    cin, H = 64, 56
    for si, (n, w) in enumerate(zip([3, 4, 6, 3], [64, 128, 256, 512])):
        for b in range(n):
            st = 2 if (b == 0 and si > 0) else 1
            s.append((cin, H, w, 1, 1, 0))
            s.append((w, H, w, 3, st, 1))
            Ho = H // st
            s.append((w, Ho, 4 * w, 1, 1, 0))
            if st != 1 or cin != 4 * w:
                s.append((cin, H, 4 * w, 1, st, 0))
            cin, H = 4 * w, Ho
    return Counter(s)


lines = []
tot = 0.0
# CONV_ONLY="ci,H,co,k,s;..." restricts the sweep to those shapes (e.g. "3,224,64,7,2;64,56,64,3,1")
only = [tuple(int(v) for v in t.split(',')) for t in os.environ.get('CONV_ONLY', '').split(';') if t]
for (ci, H, co, k, st, p), cnt in sorted(resnet50_convs().items()):
    if only and (ci, H, co, k, st) not in only:
        continue
    x = torch.randn(N, ci, H, H, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(co, ci, k, k, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    y = F.conv2d(x, w, None, st, p)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    dw = torch.empty(co, ci, k, k, device='cuda').contiguous(memory_format=CL)
    Ho = y.shape[2]
    flops = 2.0 * N * Ho * Ho * co * ci * k * k
    byts = x.numel() * 2 + y.numel() * 2
    before = set(autotune.report())
    ref = F.conv2d(x.float(), w.float(), None, st, p)
    yy = KC.conv2d(x, w, None, (st, st), (p, p))
    err = (yy.float() - ref).abs().max().item() / ref.abs().max().item()
    passes = ['fwd', 'wgrad']
    KC.conv2d_backward_filter(g, x, w.shape, (st, st), (p, p), out=dw)
    if ci != 3:
        KC.conv2d_backward_data(g, w, x.shape, (st, st), (p, p))
        passes.insert(1, 'dgrad')
    torch.cuda.synchronize()
    new = [kk for kk in autotune.report() if kk not in before]
    for kk in new:
        choice, times = autotune.report()[kk]
        best = times[choice]
        tot += cnt * best
        ln = '%-5s cin %4d H %3d cout %4d k%d s%d x%d  -> %-8s %7.3f ms %6.0f TF/s %5.0f GB/s | %s%s' % (
            kk[0], ci, H, co, k, st, cnt, choice, best, flops / best / 1e9, byts / best / 1e6,
            ' '.join('%s=%.3f' % (n_, t) for n_, t in sorted(times.items(), key=lambda kv: kv[1])),
            '  fwd rel.err %.1e' % err if kk[0] == 'fwd' else '')
        print(ln, flush=True)
        lines.append(ln)
summ = 'per-step total of the chosen kernels (x multiplicity): %.2f ms' % tot
print(summ)
lines.append(summ)
if out_path:
    open(out_path, 'w').write('\n'.join(lines) + '\n')
