"""Bandwidth of BERT-base's memory-bound kernels at the bench shapes (batch 64 x seq 128
= 8192 rows, hidden 768, FFN 3072, bf16): fused LayerNorm forward (dropout + residual)
and backward (dropout mask + linear-bias column sums), the GELU-gradient column sum and
the flat Adam update over BERT-base's dense parameters.  Prints us / call and GB/s of
the bytes each kernel must move; an ATen device copy of a same-sized buffer is the
streaming reference.

    python scripts/bench_memops.py [--ln-blocks 256,512,1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch


def timed(fn, it=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ln-blocks', default='256,512,1024,2048')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    from hetu_61a7_amd.kernels import layernorm as KL, optim as KO
    dev = torch.device('cuda')
    R, N, F = 8192, 768, 3072
    bf = torch.bfloat16
    x = torch.randn(R, N, device=dev).to(bf)
    res = torch.randn(R, N, device=dev).to(bf)
    g = torch.rand(N, device=dev) + 0.5
    b = torch.randn(N, device=dev)
    rows = []

    def rep(name, us, nbytes, **kw):
        r = dict(kernel=name, us=round(us, 2), gbps=round(nbytes / us * 1e-3, 1), **kw)
        rows.append(r)
        print(json.dumps(r), flush=True)

    big = torch.empty(R * N * 4 // 2, dtype=torch.float32, device=dev)
    big2 = torch.empty_like(big)
    rep('aten_copy_ref', timed(lambda: big2.copy_(big)), 2 * big.numel() * 4)

    y, s, mean, rstd = KL.layer_norm_fused(x, res, g, b, 1e-12, keep=0.9, seed=7)
    rep('ln_fwd_res_drop', timed(lambda: KL.layer_norm_fused(x, res, g, b, 1e-12, keep=0.9, seed=7)),
        4 * R * N * 2)
    rep('ln_fwd_plain', timed(lambda: KL.layer_norm_fused(x, None, g, b, 1e-12)), 2 * R * N * 2)
    dy = torch.randn(R, N, device=dev).to(bf)
    for nb in [int(v) for v in args.ln_blocks.split(',')]:
        for wv in (4, 8):
            KL._LN_BWD_BLOCKS, KL._LN_BWD_WAVES = nb, wv
            fnb = lambda: KL.layer_norm_fused_backward(dy, s, g, mean, rstd, keep=0.9, seed=7, want_dlin=True)
            rep('ln_bwd_drop_dlin', timed(fnb), 4 * R * N * 2, blocks=nb, waves=wv)
    pre = torch.randn(R, F, device=dev).to(bf)
    dyf = torch.randn(R, F, device=dev).to(bf)
    rep('gelu_grad_colsum', timed(lambda: KL.gelu_grad_colsum(pre, dyf)), 3 * R * F * 2)
    n = 85_800_000           # BERT-base dense parameters (word embeddings update sparsely)
    p = torch.randn(n, device=dev)
    gr = torch.randn(n, device=dev) * 1e-3
    m1 = torch.zeros(n, device=dev)
    m2 = torch.zeros(n, device=dev)
    sh = torch.empty(n, dtype=bf, device=dev)
    rep('adam_flat_shadow', timed(lambda: KO.optimizer_flat('adam', p, gr, m1, m2, sh, lr=1e-4, beta1t=0.9,
                                                            beta2t=0.999)), n * 30)
    if args.out:
        with open(args.out, 'w') as f:
            for r in rows:
                f.write(json.dumps(r) + '\n')


if __name__ == '__main__':
    main()
