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
                                                  bf16* __restrict__ y, float* __restrict__ colstats, int csrep,
                                                  int H, int W, int C, int KH, int KW, int s, int p, int OH, int OW,
                                                  int KS, int RS, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* patch = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rows_per_img = (OH + R - 1) / R;
  const int n = blockIdx.x / rows_per_img, oh0 = (blockIdx.x % rows_per_img) * R;
  const int IR = (R - 1) * s + KH;

  // 1. input rows oh0*s - p ... into LDS; patch column j <-> input element j - p*C of the row
  const int64_t img = (int64_t)n * H * W * C;
  const int WC = W * C;
  if (vec) {
    // rows as 16-byte pieces, four per thread in flight before their LDS writes (element
    // by element: the halo offset p*C is odd for C = 3); then the halo columns.  (The
    // element-wise loop below waits one memory latency per element it stages.)
    const int pC = p * C, nvr = WC / 8, tot = IR * nvr;
    unsigned short* pu = reinterpret_cast<unsigned short*>(patch);
    for (int b0 = 0; b0 < tot; b0 += 4 * 256) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = b0 + u * 256 + tid;
        v[u] = make_uint4(0u, 0u, 0u, 0u);
        if (i < tot) {
          const int rr = i / nvr, q = i - rr * nvr;
          const int ih = oh0 * s - p + rr;
          if (ih >= 0 && ih < H) v[u] = *reinterpret_cast<const uint4*>(x + img + (int64_t)ih * WC + q * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = b0 + u * 256 + tid;
        if (i < tot) {
          const int rr = i / nvr, q = i - rr * nvr;
          unsigned short* d = pu + rr * RS + pC + q * 8;
          const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            d[2 * t] = (unsigned short)(w4[t] & 0xffffu);
            d[2 * t + 1] = (unsigned short)(w4[t] >> 16);
          }
        }
      }
    }
    const int hz = RS - WC;   // zero columns per row: [0, pC) and [pC + WC, RS)
    for (int i = tid; i < IR * hz; i += 256) {
      const int rr = i / hz, c = i - rr * hz;
      pu[rr * RS + (c < pC ? c : c + WC)] = 0;
    }
  } else {
    for (int rr = 0; rr < IR; ++rr) {
      const int ih = oh0 * s - p + rr;
      const bool rok = ih >= 0 && ih < H;
      const bf16* src = x + img + (int64_t)ih * WC - p * C;
      for (int j = tid; j < RS; j += 256) {
        const int e = j - p * C;
        patch[rr * RS + j] = (rok && e >= 0 && e < WC) ? src[j] : __float2bfloat16(0.f);
      }
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
      unsafeAtomicAdd(colstats + (csrep > 1 ? (int)(blockIdx.x % csrep) * 2 * CO : 0) + which * CO + co, v);
    }
  }
}


// ---- weight gradient of the stem -----------------------------------------------------
// dW[co][kh][kw][c] = sum over output pixels of dy[px][co] * x[patch(px) + (kh, kw, c)].
// MIOpen's solver took 360 us at bs 256 and the 8-channel-padded implicit GEMM 870 us;
// the reduction over 3.2 M pixels is staged per block of WR output rows:
//   1. the WR*s + KH - s input rows the block reads go to LDS twice: as they are, and
//      shifted by 2 elements, so every 4-element run (kh, t..t+3) of any output pixel
//      starts 8-byte aligned in one of the two copies (s*C is even, so a pixel's run
//      starts at 0 or 2 mod 4);
//   2. the block's dy rows go to LDS as [px][64] (zero rows pad the width to 32 pixels);
//   3. both MFMA operands are gathered with the hardware transpose read (T10): lane
//      4q+p of a 16-lane group supplies the address of reduction row q (a pixel) and 4
//      contiguous columns, so each lane receives 4 pixels of its column -- D[k][co] over
//      (kh, t) = 11 blocks of 16 filter taps x 16 channels per wave, k = kh*24 + t;
//   4. each block accumulates its task rows in registers and stores one fp32 partial
//      [64][176] into a slab; stem_wgrad_reduce_k sums the slabs into dW.
constexpr int WR = 2;        // output rows per stage
constexpr int WKB = 11;      // 16-wide tap blocks: 7 filter rows x 24 padded taps = 168 -> 176

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

__device__ __forceinline__ v8s tr_pair(const bf16* a, const bf16* b) {
  v4s_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(a));
  v4s_t y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(b));
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

constexpr int WXL = 4;       // 16-byte input pieces per thread per task (IR * W*C / 8 <= 1024)
constexpr int WDL = 8;       // 16-byte dy pieces per thread per task (WR * OW * 8 <= 2048)

__global__ void __launch_bounds__(256, 2) stem_wgrad_k(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       float* __restrict__ slab, int N, int H, int W, int C, int KH,
                                                       int s, int p, int OH, int OW, int OWP, int RS, int IR) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* pe = reinterpret_cast<bf16*>(smem);        // IR x RS input rows (zero halo)
  bf16* po = pe + IR * RS;                          // the same shifted: po[j] = pe[j + 2]
  bf16* dl = po + IR * RS;                          // WR x OWP x 64 output gradients
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int rpi = (OH + WR - 1) / WR, ntask = N * rpi;
  const int WC = W * C, sC = s * C, pC = p * C;
  const int xv = WC / 8, nxv = IR * xv;             // 16-byte pieces of the staged input rows
  const int nvd = OW * 8;                           // 16-byte pieces of one dy row

  // halo columns and padded pixels stay zero for every task: clear once
  for (int i = tid; i < (2 * IR * RS + WR * OWP * CO) / 8; i += 256)
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);

  v4f acc[WKB];
#pragma unroll
  for (int kb = 0; kb < WKB; ++kb) acc[kb] = v4f{0.f, 0.f, 0.f, 0.f};

  // per-lane tap-run geometry of the 11 blocks: filter row and column offset of the
  // lane's 4-column run (rows past KH are clamped: their outputs are never stored)
  int roff[WKB], toff[WKB];
#pragma unroll
  for (int kb = 0; kb < WKB; ++kb) {
    const int k0 = kb * 16 + 4 * pp;
    int kh = k0 / SEG;
    toff[kb] = k0 - kh * SEG;
    roff[kb] = (kh < KH ? kh : KH - 1) * RS;
  }

  // the task's global reads are issued together into registers (and the next task's
  // right after the LDS writes, so they land during this task's MFMAs)
  uint4 xr[WXL], dr[WDL];
  auto load = [&](int task) {
    const int n = task / rpi, oh0 = (task - n * rpi) * WR;
    const bf16* img = x + (int64_t)n * H * WC;
#pragma unroll
    for (int u = 0; u < WXL; ++u) {
      const int v = tid + u * 256;
      xr[u] = make_uint4(0, 0, 0, 0);
      if (v < nxv) {
        const int rr = v / xv, ih = oh0 * s - p + rr;
        if (ih >= 0 && ih < H) xr[u] = *reinterpret_cast<const uint4*>(img + (int64_t)ih * WC + (v - rr * xv) * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < WDL; ++u) {
      const int v = tid + u * 256;
      dr[u] = make_uint4(0, 0, 0, 0);
      if (v < WR * nvd) {
        const int r = v / nvd;
        if (oh0 + r < OH)
          dr[u] = *reinterpret_cast<const uint4*>(dy + (((int64_t)n * OH + oh0 + r) * OW) * CO + (v - r * nvd) * 8);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < WXL; ++u) {
      const int v = tid + u * 256;
      if (v < nxv) {
        const int rr = v / xv, j = rr * RS + pC + (v - rr * xv) * 8;
        const uint32_t w4[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
        unsigned short* e = reinterpret_cast<unsigned short*>(pe);
        unsigned short* o = reinterpret_cast<unsigned short*>(po);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned short h = (unsigned short)(k & 1 ? w4[k >> 1] >> 16 : w4[k >> 1] & 0xffffu);
          e[j + k] = h;
          if (j + k - 2 >= rr * RS) o[j + k - 2] = h;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < WDL; ++u) {
      const int v = tid + u * 256;
      if (v < WR * nvd) {
        const int r = v / nvd, px8 = v - r * nvd;
        *reinterpret_cast<uint4*>(dl + (r * OWP) * CO + px8 * 8) = dr[u];
      }
    }
  };

  int task = blockIdx.x;
  if (task < ntask) load(task);
  for (; task < ntask; task += gridDim.x) {
    store();
    __syncthreads();
    if (task + (int)gridDim.x < ntask) load(task + gridDim.x);
    const int nsteps = OWP / 32;
    for (int r = 0; r < WR; ++r) {
      const int prow = r * s;
      for (int st = 0; st < nsteps; ++st) {
        const int px0 = st * 32 + 8 * g + q, px1 = px0 + 4;
        const v8s a = tr_pair(dl + (r * OWP + px0) * CO + 16 * wave + 4 * pp,
                              dl + (r * OWP + px1) * CO + 16 * wave + 4 * pp);
        const int ow0 = px0 < OW ? px0 : OW - 1, ow1 = px1 < OW ? px1 : OW - 1;
        const int b0 = prow * RS + ow0 * sC, b1 = prow * RS + ow1 * sC;
#pragma unroll
        for (int kb = 0; kb < WKB; ++kb) {
          const int e0 = b0 + roff[kb] + toff[kb], e1 = b1 + roff[kb] + toff[kb];
          const bf16* a0 = (e0 & 3) ? po + (e0 - 2) : pe + e0;
          const bf16* a1 = (e1 & 3) ? po + (e1 - 2) : pe + e1;
          acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_pair(a0, a1), a, acc[kb], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // 4. lane holds D[k = 16kb + 4g + i][co = 16*wave + (lane & 15)]
  float* S = slab + (int64_t)blockIdx.x * CO * (WKB * 16);
  const int co = 16 * wave + (lane & 15);
#pragma unroll
  for (int kb = 0; kb < WKB; ++kb)
    *reinterpret_cast<float4*>(S + co * (WKB * 16) + kb * 16 + 4 * g) =
        make_float4(acc[kb][0], acc[kb][1], acc[kb][2], acc[kb][3]);
}

// dW[co][kh][kw][c] (+)= sum over nb slabs of slab[b][co][kh*24 + kw*C + c]
__global__ void __launch_bounds__(256) stem_wgrad_reduce_k(const float* __restrict__ slab, int nb,
                                                           float* __restrict__ dw, int KH, int KW, int C,
                                                           int accumulate) {
  __shared__ float part[4][64];
  const int KT = KH * KW * C;
  const int o = blockIdx.x * 64 + (threadIdx.x & 63);   // output element (co, kh, kw, c)
  const int part_id = threadIdx.x >> 6;
  float v = 0.f;
  int co = 0, k = 0;
  if (o < CO * KT) {
    co = o / KT;
    const int r = o - co * KT, kh = r / (KW * C);
    k = kh * SEG + (r - kh * KW * C);
    const float* src = slab + co * (WKB * 16) + k;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int b = part_id;
    for (; b + 12 < nb; b += 16) {
      a0 += src[(int64_t)b * CO * (WKB * 16)];
      a1 += src[(int64_t)(b + 4) * CO * (WKB * 16)];
      a2 += src[(int64_t)(b + 8) * CO * (WKB * 16)];
      a3 += src[(int64_t)(b + 12) * CO * (WKB * 16)];
    }
    for (; b < nb; b += 4) a0 += src[(int64_t)b * CO * (WKB * 16)];
    v = (a0 + a1) + (a2 + a3);
  }
  part[part_id][threadIdx.x & 63] = v;
  __syncthreads();
  if (threadIdx.x < 64 && o < CO * KT) {
    const float t = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
    dw[o] = accumulate ? dw[o] + t : t;
  }
}
}  // namespace

// Packed filter bytes the forward needs: 64 x KP bf16, KP = 32 * ceil(KH*24/32).
HETU_API int64_t hetu_stem_wp_elems(int KH) { return (int64_t)CO * 32 * ((KH * SEG + 31) / 32); }

// x [N][H][W][C] bf16 (channels-last), w [64][KH][KW][C] bf16, y [N][OH][OW][64] bf16;
// colstats (nullable) [csrep][2*64] fp32, pre-zeroed (block b adds into replica b % csrep).
// Requires KW*C <= 24, s*C even (4-byte fragment reads), KH*24 <= 32*6.
HETU_API int hetu_stem_fwd(const void* x, const void* w, void* wp, void* y, float* colstats, int N, int H, int W,
                           int C, int KH, int KW, int s, int p, int csrep, hipStream_t st) {
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
  // 16-byte staging: whole rows of 16-byte pieces, each landing inside the patch row
  const int vec = (W * C) % 8 == 0 && ((uintptr_t)x & 15) == 0 && p * C + W * C <= RS && !getenv("HETU_STEM_SCALAR");
  hipLaunchKernelGGL(stem_fwd_k, dim3(blocks), dim3(256), lds, st, (const bf16*)x, (const bf16*)wp, (bf16*)y,
                     colstats, csrep, H, W, C, KH, KW, s, p, OH, OW, KS, RS, vec);
  return (int)hipGetLastError();
}

// slab floats hetu_stem_wgrad needs for `blocks` blocks
HETU_API int64_t hetu_stem_wgrad_ws(int blocks) { return (int64_t)blocks * CO * WKB * 16; }

// dw [64][KH][KW][C] fp32 (channels-last filter layout) (+)= weight gradient of the stem
// convolution; x [N][H][W][C] bf16, dy [N][OH][OW][64] bf16, ws: hetu_stem_wgrad_ws(blocks)
// floats.  Same geometry limits as hetu_stem_fwd.
HETU_API int hetu_stem_wgrad(const void* x, const void* dy, float* dw, float* ws, int blocks, int N, int H, int W,
                             int C, int KH, int KW, int s, int p, int accumulate, hipStream_t st) {
  if (KW * C > SEG || (s * C) % 2 || KH * SEG > WKB * 16 || N <= 0 || blocks < 1 || (W * C) % 8 ||
      ((uintptr_t)x & 15) || ((uintptr_t)dy & 15))
    return (int)hipErrorInvalidValue;
  const int OH = (H + 2 * p - KH) / s + 1, OW = (W + 2 * p - KW) / s + 1;
  const int OWP = (OW + 31) / 32 * 32;
  if ((int64_t)((WR - 1) * s + KH) * (W * C / 8) > 256 * WXL || (int64_t)WR * OW * 8 > 256 * WDL)
    return (int)hipErrorInvalidValue;
  // patch row: every run (ow, kh, t<24) of a padded pixel stays inside it; multiple of 4
  int RS = ((OWP - 1) * s + KW) * C + SEG + 4;
  RS = std::max(RS, p * C + W * C + 8);   // the staged row (p*C zero columns, then W*C values)
  RS = (RS + 7) / 8 * 8;
  const int IR = (WR - 1) * s + KH;
  const size_t lds = (size_t)2 * IR * RS * 2 + (size_t)WR * OWP * CO * 2;
  if (lds > 80 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_wgrad_k, dim3(blocks), dim3(256), lds, st, (const bf16*)x, (const bf16*)dy, ws, N, H, W, C,
                     KH, s, p, OH, OW, OWP, RS, IR);
  HETU_LAUNCH_CHECK();
  const int KT = KH * KW * C;
  hipLaunchKernelGGL(stem_wgrad_reduce_k, dim3((CO * KT + 63) / 64), dim3(256), 0, st, ws, blocks, dw, KH, KW, C,
                     accumulate);
  return (int)hipGetLastError();
}
