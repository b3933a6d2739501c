// Implicit-GEMM convolution (NHWC, bf16 operands, fp32 accumulate) on the MFMA
// kernels of gemm_core.h: forward, data gradient (split into stride classes) and
// weight gradient (split-K over output pixels).  1x1 / stride-1 convolutions are
// plain GEMMs and go through the buffer-descriptor loaders.
//
// Replaces cuDNN convolution (reference src/ops/CudnnConv2d.cu:54-245,
// CudnnConv2dAddBias.cu:93), SURVEY.md §2.7.
#include "gemm_core.h"

using namespace hetu;
using namespace hetu::gemm;

// y[N,OH,OW,K] (NHWC) = conv(x[N,H,W,C] NHWC, w[K,KH,KW,C]) (+bias[K]) -> act.  C % 8 == 0.
// colstats (optional, 2*K floats, zeroed by the caller) += per-channel sum and sum of
// squares of the stored y: the statistics a training-mode BatchNorm on y needs; csrep:
// colstats holds that many replicas ([csrep][2K], Epi::cs_rep).
HETU_API int hetu_conv_fwd_bf16(const void* x, const void* w, void* y, const float* bias, int N,
                                int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph,
                                int pw, int act, float* colstats, int tile, int csrep, hipStream_t st) {
  ConvGeom g = geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  int64_t M = (int64_t)N * g.OH * g.OW, Kt = (int64_t)KH * KW * C;
  Epi ep{y, nullptr, bias, K, 0, 0, 0, 1.f, 0.f, act, 0, 0, 0, 0, nullptr, 0, colstats};
  ep.cs_rep = colstats ? csrep : 0;
  if (KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && buf_ok(M * C * 2, (int64_t)K * C * 2))
    return C % BK == 0 ? launch_buf<true>((const bf16*)x, (const bf16*)w, 1, 1, C, C, 0, 0, ep, M, K, C, 1, 1, st, tile)
                       : launch_buf<false>((const bf16*)x, (const bf16*)w, 1, 1, C, C, 0, 0, ep, M, K, C, 1, 1, st, tile);
  ConvFwdA la{};
  la.x = (const bf16*)x;
  g.ctap = C % BK == 0;
  la.g = g;
  la.Ktot = Kt;
  la.rows = M;
  return launch(la, PlainK{(const bf16*)w, Kt, K, Kt, 0}, ep, M, K, Kt, 1, 1, st, tile);
}

// dx[N,H,W,C] = conv_transpose(dy[N,OH,OW,K], w[K,KH,KW,C]) (+ acc[N,H,W,C] when given:
// the gradient joined at the conv input, added in the epilogue).  K % 8 == 0, C % 8 == 0.
// bnsums (nullable, 2*C fp32 pre-zeroed) += sum(dx') and sum(dx' * bnx) per channel with
// dx' = dx masked by bnmask (the ReLU keep-bits of the BatchNorm whose output the conv
// reads; null = no ReLU) and bnx that BN's input [N,H,W,C]: the BN backward's reduction.
// bnstore: dx is stored masked (dx'), the form the BN backward and a residual branch use.
// bnrep: bnsums holds that many replicas ([bnrep][2C], see Epi::cs_rep).
const int kBnAlign = 15;
HETU_API int hetu_conv_dgrad_bf16(const void* dy, const void* w, void* dx, const void* acc,
                                  int acc_f32, int N, int H, int W, int C, int K, int KH, int KW,
                                  int sh, int sw, int ph, int pw, int tile, float* bnsums, const void* bnx,
                                  const uint8_t* bnmask, int bnstore, int acc_s2, int bnrep, hipStream_t st) {
  ConvGeom g = geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  if (bnsums && (!bnx || C % 8 || (((uintptr_t)bnx) & kBnAlign))) return (int)hipErrorInvalidValue;
  const bool plain1x1 = KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 &&
                        buf_ok((int64_t)N * H * W * K * 2, (int64_t)K * C * 2);
  // acc_s2: acc is [N, H/2, W/2, C], the gradient of a 1x1 stride-2 convolution of the same
  // input, added at the even positions (stride-1 1x1 data gradients only, even H and W)
  if (acc_s2 && (!acc || !plain1x1 || (H & 1) || (W & 1) || (int64_t)N * H * W >= (1ll << 31)))
    return (int)hipErrorInvalidValue;
  Epi ep{dx, acc, nullptr, C, C, 0, 0, 1.f, acc ? 1.f : 0.f, 0, 0, acc_f32, 0, 0, nullptr, 0, bnsums,
         bnsums ? (const bf16*)bnx : nullptr, bnsums ? bnmask : nullptr, (bnsums && bnmask && bnstore) ? 1 : 0,
         acc_s2 ? H : 0, acc_s2 ? W : 0, bnsums ? bnrep : 0};
  if (plain1x1) {
    int64_t M = (int64_t)N * H * W;
    return K % BK == 0 ? launch_buf<true>((const bf16*)dy, (const bf16*)w, 1, 0, K, C, 0, 0, ep, M, C, K, 1, 1, st, tile)
                       : launch_buf<false>((const bf16*)dy, (const bf16*)w, 1, 0, K, C, 0, 0, ep, M, C, K, 1, 1, st, tile);
  }
  // one launch over the sh*sw stride classes (blockIdx.y); grid sized for the
  // largest class, the others exit early per block
  int64_t Mmax = (int64_t)N * ((H + sh - 1) / sh) * ((W + sw - 1) / sw);
  int64_t Kmax = (int64_t)((KH + sh - 1) / sh) * ((KW + sw - 1) / sw) * K;
  g.ctap = K % BK == 0;
  ConvDgradA la{};
  la.dy = (const bf16*)dy;
  la.g = g;
  ConvDgradB lb{};
  lb.w = (const bf16*)w;
  lb.g = g;
  return launch(la, lb, ep, Mmax, C, Kmax, sh * sw, 1, st, tile);
}

// dw[K, KH*KW*C] fp32 (+)= sum over output pixels dy^T x_im2col.  Split-K over
// the pixel axis into fp32 slabs (ws: splitk*K*KH*KW*C floats) + one reduce; no atomics.
// tile 0-3: the gemm_core tiles with M = K, N = KH*KW*C; tile 4: roles swapped (K <= 64).
HETU_API int hetu_conv_wgrad_bf16(const void* dy, const void* x, float* dw, int N, int H, int W,
                                  int C, int K, int KH, int KW, int sh, int sw, int ph, int pw,
                                  int splitk, int accumulate, float* ws, int tile, hipStream_t st) {
  ConvGeom g = geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  int64_t P = (int64_t)N * g.OH * g.OW, Nc = (int64_t)KH * KW * C;
  if (tile == 4) {
    // roles swapped: M = KH*KW*C filter taps (im2col of x), N = K output channels on the
    // 128x64 tile, so a 64-channel filter bank fills the tile's N side instead of half
    // of a 128-row M side; the slabs are reduced transposed into dw[K][Nc]
    if (!ws || K > 64) return (int)hipErrorInvalidValue;
    ConvWgradB la{};
    la.x = (const bf16*)x;
    la.g = g;
    la.P = P;
    return launch_t_transposed<ConvWgradB, PlainMN, 2>(la, PlainMN{(const bf16*)dy, K, K, P, 0}, dw, Nc, accumulate,
                                                       ws, Nc, K, P, splitk, st);
  }
  Epi ep{dw, nullptr, nullptr, Nc, 0, 0, 0, 1.f, 0.f, 0, 1, 0, accumulate, 0, splitk > 1 ? ws : nullptr, 0};
  PlainMN la{(const bf16*)dy, K, K, P, 0};
  if (KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && buf_ok(P * K * 2, P * C * 2))
    return P % BK == 0 ? launch_buf<true>((const bf16*)dy, (const bf16*)x, 0, 0, K, C, 0, 0, ep, K, Nc, P, 1, splitk, st, tile)
                       : launch_buf<false>((const bf16*)dy, (const bf16*)x, 0, 0, K, C, 0, 0, ep, K, Nc, P, 1, splitk, st, tile);
  ConvWgradB lb{};
  lb.x = (const bf16*)x;
  lb.g = g;
  lb.P = P;
  return launch(la, lb, ep, K, Nc, P, 1, splitk, st, tile);
}

