"""Attention kernel timing on one GPU: the fixed-length fused kernels (attention.hip,
S <= 128, D = 64) against the general flash kernels (flash_attn.hip) on BERT-base's
shape, plus the general kernels on the Transformer / BERT phase-2 shapes.

    python scripts/bench_attn.py        -> one line per (shape, kernel, direction): us, TF/s
"""
import contextlib
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hetu_61a7_amd.kernels import attention as KA  # noqa: E402


# A/B: ALT_FLASH_LIB names a library built from another revision of flash_attn.hip
# (same C ABI); its kernels are timed next to the in-tree ones
_ALT = ctypes.CDLL(os.environ['ALT_FLASH_LIB']) if os.environ.get('ALT_FLASH_LIB') else None


@contextlib.contextmanager
def _alt_flash():
    import hetu_61a7_amd.kernels as K
    saved = {n: K._cache.get(n) for n in ('hetu_flash_fwd', 'hetu_flash_bwd')}
    for n, f in saved.items():
        if f is None:
            raise RuntimeError('time the in-tree kernels first')
        g = getattr(_ALT, n)
        g.argtypes, g.restype = f.argtypes, f.restype
        K._cache[n] = g
    try:
        yield
    finally:
        K._cache.update(saved)


def timeit(f, reps=20, rounds=5):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            f()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best * 1e3   # us


def packed_case(B, S, NH, D, keep):
    H = NH * D
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    qkv = (torch.randn((B * S, 3 * H), device='cuda', generator=g) * 0.5).bfloat16()
    mask = torch.zeros((B, S), device='cuda')
    fl_f = 4.0 * B * NH * S * S * D
    out, lse = KA.attention_fwd(qkv, mask, B, S, NH, keep, 7)
    do = torch.randn(out.shape, device='cuda', generator=g).bfloat16()
    rows = []
    if KA.fused_ok(qkv, S, D):
        t = timeit(lambda: KA.attention_fwd(qkv, mask, B, S, NH, keep, 7))
        rows.append(('fused', 'fwd', t, fl_f / t * 1e-6))
        mode0 = KA._BWD_MODE
        for mode in ('split', 'fused', 'w8'):   # the backward's forms (kernels/attention.py)
            KA._BWD_MODE, KA._BWD_SPLIT = mode, mode == 'split'
            t = timeit(lambda: KA.attention_bwd(do, qkv, out, lse, mask, B, S, NH, keep, 7))
            rows.append(('fused', 'bwd-' + mode, t, 2.5 * fl_f / t * 1e-6))
        KA._BWD_MODE, KA._BWD_SPLIT = mode0, mode0 == 'split'
    q, k, v = KA.packed_heads(qkv, B, S, NH)
    m4 = mask.reshape(B, 1, 1, S)
    o4 = out.view(B, S, NH, D).permute(0, 2, 1, 3)
    t = timeit(lambda: KA.flash_fwd(q, k, v, m4, False, keep, 7, out=o4))
    rows.append(('flash', 'fwd', t, fl_f / t * 1e-6))
    g4 = do.view(B, S, NH, D).permute(0, 2, 1, 3)
    t = timeit(lambda: KA.flash_bwd(g4, q, k, v, o4, lse, m4, False, keep, 7))
    rows.append(('flash', 'bwd', t, 2.5 * fl_f / t * 1e-6))
    if _ALT is not None:
        with _alt_flash():
            t = timeit(lambda: KA.flash_fwd(q, k, v, m4, False, keep, 7, out=o4))
            rows.append(('alt', 'fwd', t, fl_f / t * 1e-6))
            t = timeit(lambda: KA.flash_bwd(g4, q, k, v, o4, lse, m4, False, keep, 7))
            rows.append(('alt', 'bwd', t, 2.5 * fl_f / t * 1e-6))
    for r in rows:
        print('B %3d S %4d NH %2d D %3d keep %.1f | %-5s %-9s %8.1f us %6.1f TF/s' % ((B, S, NH, D, keep) + r),
              flush=True)


def main():
    packed_case(64, 128, 12, 64, 0.9)      # BERT-base bench shape (dropout 0.1)
    packed_case(64, 128, 12, 64, 1.0)
    packed_case(16, 512, 12, 64, 1.0)      # BERT phase 2
    packed_case(32, 100, 8, 64, 1.0)       # Transformer encoder (maxlen 100)


if __name__ == '__main__':
    main()
