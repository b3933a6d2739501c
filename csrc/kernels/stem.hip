// Direct convolution for the few-channel network stem (ResNet-50 conv1: Cin 3, 7x7,
// stride 2, 64 filters) -- reference CudnnConv2d.cu:54-70 serves it through cuDNN.
//
// The implicit-GEMM kernels need 8-channel (16-byte) reduction chunks, so a 3-channel
// input had to be zero-padded to 8 channels: 2.7x the MFMA work plus a padding copy.
// Here the reduction runs over (kh, kw, c) with each filter row's KW*C values padded
// to 24 (a multiple of the 8-element fragment), so a lane's 8 reduction values lie
// in ONE input row of the staged patch, contiguous in NHWC order:
//   patch element (kh, ow) + t  with  t = kw*C + c.
// Block = R output rows x the whole output width of one image:
//   1. the R*s + KH - s input rows it reads are staged in LDS (zero halo);
//   2. the packed filters [64][KP] (one small prep kernel) are held in registers as
//      MFMA fragments for the whole block (4 column blocks x KP/32 k-steps);
//   3. each wave walks 16-pixel blocks: per k-step one fragment of 4 ds_read_b32 and
//      4 mfma_f32_16x16x32_bf16 (one per 16-filter block), D = filters x pixels so a
//      lane holds 4 consecutive output channels of one pixel -> 8-byte NHWC stores;
//   4. optional BatchNorm statistics (per-channel sum / sum of squares of the stored
//      bf16 values) reduced in registers, across waves in LDS, one atomic per channel.
#include "common.h"

#include <algorithm>

using namespace hetu;

namespace {

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int SEG = 24;      // padded KW*C per filter row
constexpr int CO = 64;       // output channels
constexpr int R = 4;         // output rows per block
constexpr int MAXKS = 6;     // k-steps of 32 held in registers (KH <= 8)

// wp[co][k], k = kh*SEG + kw*C + c (zero where kw*C + c >= KW*C or kh >= KH)
__global__ void __launch_bounds__(256) stem_pack_w_k(const bf16* __restrict__ w, bf16* __restrict__ wp, int KH,
                                                     int KW, int C, int KP) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= CO * KP) return;
  const int co = i / KP, k = i % KP;
  const int kh = k / SEG, t = k % SEG;
  float v = 0.f;
  if (kh < KH && t < KW * C) v = to_f(w[((co * KH + kh) * KW) * C + t]);
  wp[i] = __float2bfloat16(v);
}

__global__ void __launch_bounds__(256) stem_fwd_k(const bf16* __restrict__ x, const bf16* __restrict__ wp,
                                                  bf16* __restrict__ y, float* __restrict__ colstats, int H, int W,
                                                  int C, int KH, int KW, int s, int p, int OH, int OW, int KS,
                                                  int RS) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* patch = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rows_per_img = (OH + R - 1) / R;
  const int n = blockIdx.x / rows_per_img, oh0 = (blockIdx.x % rows_per_img) * R;
  const int IR = (R - 1) * s + KH;

  // 1. input rows oh0*s - p ... into LDS; patch column j <-> input element j - p*C of the row
  const int64_t img = (int64_t)n * H * W * C;
  const int WC = W * C;
  for (int rr = 0; rr < IR; ++rr) {
    const int ih = oh0 * s - p + rr;
    const bool rok = ih >= 0 && ih < H;
    const bf16* src = x + img + (int64_t)ih * WC - p * C;
    for (int j = tid; j < RS; j += 256) {
      const int e = j - p * C;
      patch[rr * RS + j] = (rok && e >= 0 && e < WC) ? src[j] : __float2bfloat16(0.f);
    }
  }

  // 2. filter fragments: A operand of D[co][px], lane holds co = 16cb + (lane&15),
  //    k = 32ks + 8(lane>>4) + j
  const int KP = KS * 32;
  v8s bw[4][MAXKS];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int ks = 0; ks < MAXKS; ++ks)
      if (ks < KS)
        bw[cb][ks] = *reinterpret_cast<const v8s*>(wp + (cb * 16 + (lane & 15)) * KP + ks * 32 + 8 * (lane >> 4));
  __syncthreads();

  float cs[4][4], cq[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) { cs[cb][i] = 0.f; cq[cb][i] = 0.f; }

  const int npx = R * OW;
  const int nrb = (npx + 15) / 16;
  const int sC = s * C;
  for (int rb = wave; rb < nrb; rb += 4) {
    const int px = rb * 16 + (lane & 15);
    const bool pok = px < npx;
    const int r = pok ? px / OW : 0, ow = pok ? px % OW : 0;
    const bool ook = pok && oh0 + r < OH;
    v4f acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < MAXKS; ++ks) {
      if (ks < KS) {
        const int k = ks * 32 + 8 * (lane >> 4);
        int kh = k / SEG;
        const int t = k - kh * SEG;
        kh = kh < KH ? kh : KH - 1;   // virtual filter rows: zero weights, any finite data
        const uint32_t* a = reinterpret_cast<const uint32_t*>(patch + (r * s + kh) * RS + ow * sC + t);
        union { uint32_t u[4]; v8s v; } f;
#pragma unroll
        for (int q = 0; q < 4; ++q) f.u[q] = a[q];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[cb][ks], f.v, acc[cb], 0, 0, 0);
      }
    }
    if (ook) {
      bf16* dst = y + (((int64_t)n * OH + oh0 + r) * OW + ow) * CO;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int co = cb * 16 + 4 * (lane >> 4);
        unsigned short h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h[i] = f_to_bf16_bits(acc[cb][i]);
          const float sv = bf16_bits_to_f(h[i]);
          cs[cb][i] += sv;
          cq[cb][i] += sv * sv;
        }
        uint2 pk;
        pk.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
        pk.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
        *reinterpret_cast<uint2*>(dst + co) = pk;
      }
    }
  }

  if (colstats) {
    // lanes sharing lane>>4 hold the same 16 channels: fold the 16 pixels
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          cs[cb][i] += __shfl_xor(cs[cb][i], o, 64);
          cq[cb][i] += __shfl_xor(cq[cb][i], o, 64);
        }
    __syncthreads();   // the patch is no longer read
    float* red = reinterpret_cast<float*>(smem);   // [4 waves][2][64]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = cb * 16 + 4 * (lane >> 4) + i;
          red[(wave * 2) * CO + co] = cs[cb][i];
          red[(wave * 2 + 1) * CO + co] = cq[cb][i];
        }
    }
    __syncthreads();
    if (tid < 2 * CO) {
      const int which = tid / CO, co = tid % CO;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * CO + co];
      unsafeAtomicAdd(colstats + which * CO + co, v);
    }
  }
}

}  // namespace

// Packed filter bytes the forward needs: 64 x KP bf16, KP = 32 * ceil(KH*24/32).
HETU_API int64_t hetu_stem_wp_elems(int KH) { return (int64_t)CO * 32 * ((KH * SEG + 31) / 32); }

// x [N][H][W][C] bf16 (channels-last), w [64][KH][KW][C] bf16, y [N][OH][OW][64] bf16;
// colstats (nullable) [2*64] fp32, pre-zeroed.  Requires KW*C <= 24, s*C even (4-byte
// fragment reads), KH*24 <= 32*6.
HETU_API int hetu_stem_fwd(const void* x, const void* w, void* wp, void* y, float* colstats, int N, int H, int W,
                           int C, int KH, int KW, int s, int p, hipStream_t st) {
  if (KW * C > SEG || (s * C) % 2 || KH * SEG > 32 * MAXKS || N <= 0) return (int)hipErrorInvalidValue;
  const int OH = (H + 2 * p - KH) / s + 1, OW = (W + 2 * p - KW) / s + 1;
  const int KS = (KH * SEG + 31) / 32, KP = KS * 32;
  // patch row: (OW-1)*s + KW input columns, +SEG slack for the padded fragment tail, even
  int RS = ((OW - 1) * s + KW) * C + SEG;
  RS += RS & 1;
  const int IR = (R - 1) * s + KH;
  const size_t lds = std::max<size_t>((size_t)IR * RS * 2, 4 * 2 * CO * sizeof(float));
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_pack_w_k, dim3((CO * KP + 255) / 256), dim3(256), 0, st, (const bf16*)w, (bf16*)wp, KH,
                     KW, C, KP);
  const int blocks = N * ((OH + R - 1) / R);
  hipLaunchKernelGGL(stem_fwd_k, dim3(blocks), dim3(256), lds, st, (const bf16*)x, (const bf16*)wp, (bf16*)y,
                     colstats, H, W, C, KH, KW, s, p, OH, OW, KS, RS);
  return (int)hipGetLastError();
}
