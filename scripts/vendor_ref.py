"""Vendor-library references for A/B measurements (NOT part of the framework).

The package has no library path: every device GEMM / convolution runs on a hand-written
kernel or raises ``NoKernelError``.  The hipBLASLt / MIOpen calls that the round-1..5
runtime carried as an opt-in switch live here, for harnesses that time the hand-written
kernels against the libraries (``csrc/bench/gemm_bench.hip`` does the same for GEMMs
in C++):

    python scripts/vendor_ref.py gemm 4096 4096 4096     # hipBLASLt vs the autotuned MFMA tiles
    python scripts/vendor_ref.py conv 256 64 56 64 3 1   # MIOpen vs the hand-written conv
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch                      # noqa: E402
import torch.nn.functional as F   # noqa: E402

CL = torch.channels_last


def gemm(A, B, bias=None):
    """hipBLASLt (through torch): A @ B (+ bias in the library epilogue)"""
    return torch.addmm(bias, A, B) if bias is not None else torch.mm(A, B)


def gemm_f32_out(A, B, out):
    """bf16 x bf16 -> fp32 written directly (aten::mm.dtype) when available"""
    try:
        return torch.mm(A, B, out_dtype=torch.float32, out=out)
    except (RuntimeError, TypeError):
        out.copy_(torch.mm(A, B))
        return out


def gemm_splitk_f32(A, B, out, s=4):
    """K split into ``s`` batched library GEMMs + one reduction"""
    M, K = A.shape
    N = B.shape[1]
    kc = K // s
    Av = A.as_strided((s, M, kc), (kc * A.stride(1), A.stride(0), A.stride(1)))
    Bv = B.as_strided((s, kc, N), (kc * B.stride(0), B.stride(0), B.stride(1)))
    torch.sum(torch.bmm(Av, Bv, out_dtype=torch.float32), 0, out=out)
    return out


def conv_fwd(x, w, stride, padding):
    """MIOpen forward"""
    return F.conv2d(x, w, None, stride, padding)


def conv_dgrad(g, w, x_shape, stride, padding):
    """MIOpen data gradient (x only supplies shape and layout)"""
    xs = torch.empty(x_shape, dtype=g.dtype, device=g.device).contiguous(memory_format=CL)
    dx, _, _ = torch.ops.aten.convolution_backward(
        g, xs, w, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [True, False, False])
    return dx


def conv_wgrad(g, x, w_shape, stride, padding):
    """MIOpen weight gradient"""
    ws = torch.empty(w_shape, dtype=g.dtype, device=g.device).contiguous(memory_format=CL)
    _, dw, _ = torch.ops.aten.convolution_backward(
        g, x, ws, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, [False, True, False])
    return dw


def _time(f, reps=20):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main(argv):
    if argv[0] == 'gemm':
        from hetu_61a7_amd.kernels import gemm as KG
        M, N, K = (int(v) for v in argv[1:4])
        A = torch.randn(M, K, device='cuda').bfloat16()
        B = torch.randn(K, N, device='cuda').bfloat16()
        for name, f in (('hipblaslt', lambda: gemm(A, B)), ('hetu', lambda: KG.matmul(A, B))):
            ms = _time(f)
            print('%-10s %8.3f ms  %7.1f TF/s' % (name, ms, 2.0 * M * N * K / ms / 1e9))
    elif argv[0] == 'conv':
        from hetu_61a7_amd.kernels import conv as KC
        n, ci, h, co, k, s = (int(v) for v in argv[1:7])
        p = k // 2
        x = torch.randn(n, ci, h, h, device='cuda').bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(co, ci, k, k, device='cuda') * 0.05).bfloat16().contiguous(memory_format=CL)
        for name, f in (('miopen', lambda: conv_fwd(x, w, (s, s), (p, p))),
                        ('hetu', lambda: KC.conv2d(x, w, None, (s, s), (p, p)))):
            print('%-10s fwd %8.3f ms' % (name, _time(f)))


if __name__ == '__main__':
    main(sys.argv[1:])
