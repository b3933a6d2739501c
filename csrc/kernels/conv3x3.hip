// 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels (ResNet-50
// stage 1 at 56x56, and its data gradient), as a halo-tile MFMA kernel.
//
// The implicit-GEMM kernels (gemm_core.h) fetch each input pixel once per filter tap:
// nine K-tiles, nine passes of the activation through L2.  Here one block owns one image
// and walks it TH output rows at a time:
//   * the 64x9x64 filter bank stays in LDS for the block's lifetime (72 KiB, one
//     [co][64] K-major image per tap, 16-byte chunks XOR-swizzled by row);
//   * input rows live in a ring of NSLOT halo rows (64 positions x 128 B each, column 0
//     and W+1 the zero pad); the TH rows the next tile needs are DMA'd (global_load_lds,
//     swizzle applied on the source side) while the current tile computes, so every
//     input row crosses HBM/L2 once;
//   * a tap is just an LDS address offset: the pixel operand of tap (kh, kw) is the
//     ds_read_b128 of halo position (tx + kw) in ring row (ty + kh).
// Waves own two 16-pixel blocks x all 64 output channels (8 accumulator tiles of
// mfma_f32_16x16x32_bf16, D[co][px]), so a lane stores 4 consecutive channels of one
// pixel.  Optional epilogue: + Cin (the data-gradient join, bf16 or fp32) and the
// per-channel sum / sum of squares of the stored values (BatchNorm statistics).
//
// Replaces cuDNN/MIOpen for these shapes (reference src/ops/CudnnConv2d.cu:54-70).
#include "common.h"
#include "lds_tr.h"
#include <stdlib.h>

#include <algorithm>

using namespace hetu;

namespace {

// BatchNorm-backward statistics in a data-gradient epilogue (see gemm_core.h Epi::bnx):
// with x set, colstats receives sum(dx') and sum(dx' * x) of the stored dx, dx' masked by
// the forward ReLU keep-bits (one byte per 8 channels; null = no ReLU)
struct BnB {
  const bf16* x;
  const uint8_t* mask;
  int store;   // store the masked gradient dx' (mask applied before the store)
  int rep;     // colstats replicas ([rep][2 * channels]; see gemm_core.h Epi::cs_rep)
};

// mask bits of 4 channels at element offset e (co % 4 == 0), all-ones without a mask
__device__ __forceinline__ unsigned mask4(const BnB& bn, int64_t e) {
  return (bn.x && bn.mask) ? ((unsigned)bn.mask[e >> 3] >> (e & 7)) & 0xfu : 0xfu;
}

// BN operands of 4 channels at element offset e, requested before the tile's Cin load and
// store so the round trips overlap
struct Bn4 {
  uint2 x;
  unsigned mk;
};
__device__ __forceinline__ Bn4 bn_load4(const BnB& bn, int64_t e) {
  Bn4 r{make_uint2(0, 0), 0xfu};
  if (bn.x) {
    r.x = *reinterpret_cast<const uint2*>(bn.x + e);
    r.mk = mask4(bn, e);
  }
  return r;
}

// 4 stored channels into the running sums s[0..3], q[0..3]
__device__ __forceinline__ void stats4(const BnB& bn, const Bn4& b4, const unsigned short (&h)[4], float* s, float* q) {
  if (bn.x) {
    const float xv[4] = {bf16_bits_to_f((unsigned short)(b4.x.x & 0xffffu)), bf16_bits_to_f((unsigned short)(b4.x.x >> 16)),
                         bf16_bits_to_f((unsigned short)(b4.x.y & 0xffffu)), bf16_bits_to_f((unsigned short)(b4.x.y >> 16))};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float g = (b4.mk >> i) & 1u ? bf16_bits_to_f(h[i]) : 0.f;
      s[i] += g;
      q[i] += g * xv[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float sv = bf16_bits_to_f(h[i]);
      s[i] += sv;
      q[i] += sv * sv;
    }
  }
}

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int CH = 64;                 // input = output channels
constexpr int RP = 64;                 // halo positions per ring row (W + 2 <= 64)
constexpr int ROWB = RP * CH * 2;      // 8 KiB per ring row
constexpr int TAPB = CH * CH * 2;      // 8 KiB per filter tap image
constexpr int WBYTES = 9 * TAPB;       // 72 KiB

static __device__ __attribute__((aligned(64))) bf16 g_zero16[32];

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// byte offset of logical 16-byte chunk c of row r in a [rows][64 bf16] swizzled image
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

template <int WD, int TH>
struct Geo {
  static constexpr int PX = TH * WD;            // pixels per tile
  static constexpr int PB = (PX + 15) / 16;     // 16-pixel blocks
  static constexpr int NW = (PB + 1) / 2;       // waves: two blocks each
  static constexpr int NT = NW * 64;
  static constexpr int NSLOT = 2 * TH + 2;      // rows in use (TH + 2) + rows in flight (TH)
};

template <int WD, int TH>
__global__ __launch_bounds__((Geo<WD, TH>::NT), 1) void conv3x3_c64_k(const bf16* __restrict__ x,
                                                                      const bf16* __restrict__ w,
                                                                      bf16* __restrict__ y, const void* cin,
                                                                      int cin_f32, float* colstats, BnB bn,
                                                                      int H) {
  using G = Geo<WD, TH>;
  __shared__ __attribute__((aligned(16))) char smem[WBYTES + G::NSLOT * ROWB];
  char* wl = smem;
  char* ring = smem + WBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x;
  const bf16* img = x + (int64_t)n * H * WD * CH;

  // stage input row ih (may be out of range: zeros) into its ring slot; 8 wave
  // instructions of 1 KiB (8 halo positions x 8 chunks) per row, dealt to the waves
  auto stage_rows = [&](int r0, int nrows) {
    const int total = nrows * 8;
    for (int I = wave; I < total; I += G::NW) {
      const int rr = I >> 3, pos0 = (I & 7) * 8;
      const int ih = r0 + rr;
      const int slot = (ih + 1 + G::NSLOT) % G::NSLOT;
      const int pos = pos0 + (lane >> 3);
      const int c = (lane & 7) ^ (pos & 7);
      const int iw = pos - 1;
      const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < WD;
      const void* src = ok ? (const void*)(img + ((int64_t)ih * WD + iw) * CH + c * 8) : (const void*)g_zero16;
      dma16(src, ring + slot * ROWB + pos0 * 128);
    }
  };

  // filter bank: tap image t, row co, chunk c <- w[co][t][c*8 .. +8]
  for (int J = wave; J < 72; J += G::NW) {
    const int tap = J >> 3, co = (J & 7) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (co & 7);
    dma16(w + ((int64_t)co * 9 + tap) * CH + c * 8, wl + tap * TAPB + (J & 7) * 1024);
  }
  stage_rows(-1, TH + 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // this lane's two pixel blocks: tile-relative row / column of pixel (lane & 15)
  int ty[2], tx[2];
  bool pv[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int px = (2 * wave + p) * 16 + (lane & 15);
    pv[p] = px < G::PX;
    const int pc = pv[p] ? px : 0;
    ty[p] = pc / WD;
    tx[p] = pc - ty[p] * WD;
  }
  const int q4 = lane >> 4;    // k-chunk within a 32-wide k-step / 4-channel group of D

  float cs[16], cq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { cs[i] = 0.f; cq[i] = 0.f; }

  const int ntiles = (H + TH - 1) / TH;
  for (int t = 0; t < ntiles; ++t) {
    const int oh0 = t * TH;
    // rows oh0+TH+1 .. oh0+2TH for the next tile land while this one computes
    if (t + 1 < ntiles) stage_rows(oh0 + TH + 1, TH);

    v4f acc[2][4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[p][q] = v4f{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      int rb[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) rb[p] = ((oh0 + ty[p] + kh) % G::NSLOT) * ROWB;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const char* wt = wl + (kh * 3 + kw) * TAPB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + q4;
          v8s wf[4], pf[2];
#pragma unroll
          for (int q = 0; q < 4; ++q) wf[q] = *reinterpret_cast<const v8s*>(wt + swz(q * 16 + (lane & 15), c));
#pragma unroll
          for (int p = 0; p < 2; ++p)
            pf[p] = *reinterpret_cast<const v8s*>(ring + rb[p] + swz(tx[p] + kw, c));
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[q], pf[p], acc[p][q], 0, 0, 0);
        }
      }
    }

    // epilogue: lane holds channels q*16 + 4*q4 + i of pixel (ty, tx)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int oh = oh0 + ty[p];
      if (!pv[p] || oh >= H) continue;
      const int64_t pix = ((int64_t)n * H + oh) * WD + tx[p];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = q * 16 + 4 * q4;
        float v[4] = {acc[p][q][0], acc[p][q][1], acc[p][q][2], acc[p][q][3]};
        const Bn4 b4 = colstats ? bn_load4(bn, pix * CH + co) : Bn4{make_uint2(0, 0), 0xfu};
        if (cin) {
          if (cin_f32) {
            const float4 a = *reinterpret_cast<const float4*>((const float*)cin + pix * CH + co);
            v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
          } else {
            const uint2 a = *reinterpret_cast<const uint2*>((const bf16*)cin + pix * CH + co);
            v[0] += bf16_bits_to_f((unsigned short)(a.x & 0xffffu));
            v[1] += bf16_bits_to_f((unsigned short)(a.x >> 16));
            v[2] += bf16_bits_to_f((unsigned short)(a.y & 0xffffu));
            v[3] += bf16_bits_to_f((unsigned short)(a.y >> 16));
          }
        }
        if (bn.store) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (b4.mk >> i) & 1u ? v[i] : 0.f;
        }
        unsigned short h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = f_to_bf16_bits(v[i]);
        if (colstats) stats4(bn, b4, h, cs + q * 4, cq + q * 4);
        uint2 pk;
        pk.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
        pk.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
        *reinterpret_cast<uint2*>(y + pix * CH + co) = pk;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if (colstats) {
    // lanes of one 16-lane group hold the same 16 channels: fold their pixels, then the
    // waves through LDS (the ring is free now), one atomic per channel and statistic
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        cs[i] += __shfl_xor(cs[i], o, 64);
        cq[i] += __shfl_xor(cq[i], o, 64);
      }
    float* red = reinterpret_cast<float*>(ring);   // [NW][2][64]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = q * 16 + 4 * q4 + i;
          red[(wave * 2) * CH + co] = cs[q * 4 + i];
          red[(wave * 2 + 1) * CH + co] = cq[q * 4 + i];
        }
    }
    __syncthreads();
    if (tid < 2 * CH) {
      const int which = tid / CH, co = tid % CH;
      float v = 0.f;
      for (int ww = 0; ww < G::NW; ++ww) v += red[(ww * 2 + which) * CH + co];
      unsafeAtomicAdd(colstats + (bn.rep > 1 ? (n % bn.rep) * 2 * CH : 0) + which * CH + co, v);
    }
  }
}

// w'[ci][kh][kw][co] = w[co][2-kh][2-kw][ci]: the data gradient of a 3x3 / pad-1 /
// stride-1 convolution is the same convolution of dy with this bank
__global__ void __launch_bounds__(256) flip_bank_k(const bf16* __restrict__ w, bf16* __restrict__ wt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= CH * 9 * CH) return;
  const int ci = i / (9 * CH), r = i - ci * 9 * CH, tap = r / CH, co = r - tap * CH;
  wt[i] = w[((int64_t)co * 9 + (8 - tap)) * CH + ci];
}

template <int WD, int TH>
int launch_c64(const bf16* x, const bf16* w, bf16* y, const void* cin, int cin_f32, float* colstats, BnB bn, int N,
               int H, hipStream_t st) {
  using G = Geo<WD, TH>;
  hipLaunchKernelGGL((conv3x3_c64_k<WD, TH>), dim3(N), dim3(G::NT), 0, st, x, w, y, cin, cin_f32, colstats, bn, H);
  return (int)hipGetLastError();
}

int dispatch_c64(const bf16* x, const bf16* w, bf16* y, const void* cin, int cin_f32, float* colstats, BnB bn, int N,
                 int H, int W, hipStream_t st) {
  // tiles of 224 pixels: 4 rows of 56 (the only width 64-channel 3x3 layers have in ResNet-50)
  if (W == 56) return launch_c64<56, 4>(x, w, y, cin, cin_f32, colstats, bn, N, H, st);
  return (int)hipErrorInvalidValue;
}


// ---- weight gradient ---------------------------------------------------------------------
// dW[co][kh][kw][ci] = sum over pixels dy[px][co] * x[px + (kh-1, kw-1)][ci].  Same walk as
// the forward (one block per image, TH-row tiles, DMA ring of halo rows, prefetch of the
// next tile), plus the tile's dy rows as a [px][64] swizzled image (double buffered).  The
// reduction over pixels needs pixel-contiguous MFMA operands: both are gathered with the
// hardware transpose read (T10) -- lane 4q+p of a 16-lane group supplies the address of
// pixel row q and 4 contiguous channels, so each lane receives 4 pixels of its channel.
// Wave w owns output channel block (w & 3) x input channel blocks 2(w>>2), 2(w>>2)+1 for all
// 9 taps: 18 accumulator tiles D[ci][co] (4 consecutive ci per lane -> float4 stores).  The
// block's partial goes to a slab; wgrad_reduce_k sums the slabs into dW.
constexpr int WG_NW = 8;
constexpr int WG_PX = 224;                       // pixels per tile (4 rows of 56)

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

__device__ __forceinline__ v8s tr_pair(const char* a, const char* b) {
  v4s_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(a));
  v4s_t y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(b));
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}
// asm form (lds_tr.h) for a K loop with the next tile's DMA in flight: the intrinsic would
// wait for that DMA; consumers call frag_wait() before the MFMAs
__device__ __forceinline__ v8s tr_pair_asm(const char* a, const char* b) {
  v4s_t x = ds_tr16(a);
  v4s_t y = ds_tr16(b);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ASMTR: fragment reads as asm (the next tile's DMA stays in flight: all 19 fragments of
// a k-step, one wait, 18 MFMAs) or the intrinsic (the compiler waits for that DMA before the
// first read, then interleaves reads and MFMAs); HETU_C64_WGRAD_ASM picks (default 1)
template <int WD, int TH, bool ASMTR = true>
__global__ __launch_bounds__(WG_NW * 64, 1) void conv3x3_c64_wgrad_k(const bf16* __restrict__ x,
                                                                   const bf16* __restrict__ dy,
                                                                   float* __restrict__ slab, int H) {
  constexpr int NSLOT = 2 * TH + 2;
  constexpr int PX = TH * WD;
  constexpr int DYB = PX * 128;                   // one dy tile image
  static_assert(PX % 32 == 0, "pixel tile must be whole 32-pixel k-steps");
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * ROWB + 2 * DYB];
  char* ring = smem;
  char* dyl = smem + NSLOT * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x;
  const bf16* img = x + (int64_t)n * H * WD * CH;
  const bf16* gimg = dy + (int64_t)n * H * WD * CH;

  auto stage_rows = [&](int r0, int nrows) {
    for (int I = wave; I < nrows * 8; I += WG_NW) {
      const int rr = I >> 3, pos0 = (I & 7) * 8;
      const int ih = r0 + rr;
      const int slot = (ih + 1 + NSLOT) % NSLOT;
      const int pos = pos0 + (lane >> 3);
      const int c = (lane & 7) ^ (pos & 7);
      const int iw = pos - 1;
      const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < WD;
      const void* src = ok ? (const void*)(img + ((int64_t)ih * WD + iw) * CH + c * 8) : (const void*)g_zero16;
      dma16(src, ring + slot * ROWB + pos0 * 128);
    }
  };
  // dy rows oh0 .. oh0+TH-1 into dy buffer b: PX/8 instructions of 8 pixels
  auto stage_dy = [&](int oh0, int b) {
    for (int I = wave; I < PX / 8; I += WG_NW) {
      const int px = I * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (px & 7);
      const int ty = px / WD, tx = px - ty * WD;
      const bool ok = oh0 + ty < H;
      const void* src = ok ? (const void*)(gimg + ((int64_t)(oh0 + ty) * WD + tx) * CH + c * 8) : (const void*)g_zero16;
      dma16(src, dyl + b * DYB + I * 1024);
    }
  };

  stage_rows(-1, TH + 2);
  stage_dy(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int cb = wave & 3, cib0 = 2 * (wave >> 2);
  v4f acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[t][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int ntiles = (H + TH - 1) / TH;
  for (int t = 0; t < ntiles; ++t) {
    const int oh0 = t * TH, cur = t & 1;
    if (t + 1 < ntiles) {
      stage_rows(oh0 + TH + 1, TH);
      stage_dy(oh0 + TH, cur ^ 1);
    }
    const char* dyb = dyl + cur * DYB;
#pragma unroll 1
    for (int st = 0; st < PX / 32; ++st) {
      const int px0 = st * 32 + 8 * g + q, px1 = px0 + 4;
      // dy operand: pixels px0 / px1, channels 16cb + 4p .. +3
      const int dch = 2 * cb + (p >> 1), dof = (p & 1) * 8;
      const v8s bf = (ASMTR ? tr_pair_asm : tr_pair)(dyb + px0 * 128 + ((dch ^ (px0 & 7)) << 4) + dof,
                             dyb + px1 * 128 + ((dch ^ (px1 & 7)) << 4) + dof);
      const int ty0 = px0 / WD, tx0 = px0 - ty0 * WD, ty1 = px1 / WD, tx1 = px1 - ty1 * WD;
      // all 18 x fragments of the k-step first (asm reads: the next tile's DMA stays in
      // flight), one wait, then the MFMAs
      v8s af[9][2];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* r0 = ring + ((oh0 + ty0 + kh) % NSLOT) * ROWB;
        const char* r1 = ring + ((oh0 + ty1 + kh) % NSLOT) * ROWB;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int pos0 = tx0 + kw, pos1 = tx1 + kw;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int xch = 2 * (cib0 + j) + (p >> 1);
            af[kh * 3 + kw][j] = (ASMTR ? tr_pair_asm : tr_pair)(r0 + pos0 * 128 + ((xch ^ (pos0 & 7)) << 4) + dof,
                                         r1 + pos1 * 128 + ((xch ^ (pos1 & 7)) << 4) + dof);
          }
        }
      }
      if constexpr (ASMTR) frag_wait();
#pragma unroll
      for (int tp = 0; tp < 9; ++tp)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[tp][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tp][j], bf, acc[tp][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // lane holds D[ci = 16*cib + 4g + i][co = 16cb + (lane & 15)] of every tap
  float* S = slab + (int64_t)n * 9 * CH * CH;
  const int co = 16 * cb + (lane & 15);
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      *reinterpret_cast<float4*>(S + ((int64_t)co * 9 + tp) * CH + 16 * (cib0 + j) + 4 * g) =
          make_float4(acc[tp][j][0], acc[tp][j][1], acc[tp][j][2], acc[tp][j][3]);
}

// dw[i] (+)= sum over nb slabs of slab[b][i], i over 64*9*64 fp32 (float4 per thread)
// first pass of the two-pass slab sum: group blockIdx.y adds slabs [g*per, (g+1)*per) (eight
// loads in flight per thread) and writes the total over its own first slab (each thread reads
// its element of every slab of the group before it writes that element).  One pass over all
// N = 256 per-image slabs left 36 blocks each walking 256 slabs two at a time (35 us).
__global__ void __launch_bounds__(256) wgrad_slab_group_k(float4* __restrict__ slab, int nb, int per, int n4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int k0 = blockIdx.y * per, k1 = min(nb, k0 + per);
  float4 a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = k0;
  for (; k + 7 < k1; k += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(k + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) { a[u].x += v[u].x; a[u].y += v[u].y; a[u].z += v[u].z; a[u].w += v[u].w; }
  }
  for (; k < k1; ++k) {
    const float4 v = slab[(int64_t)k * n4 + i];
    a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
  }
#pragma unroll
  for (int u = 1; u < 8; ++u) { a[0].x += a[u].x; a[0].y += a[u].y; a[0].z += a[u].z; a[0].w += a[u].w; }
  if (k0 < k1) slab[(int64_t)k0 * n4 + i] = a[0];
}

// second pass: dw (+)= the group totals (slabs 0, per, 2 per, ...)
__global__ void __launch_bounds__(256) wgrad_slab_final_k(const float4* __restrict__ slab, int nb, int per,
                                                          float4* __restrict__ dw, int n4, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < nb; k += per) {
    const float4 v = slab[(int64_t)k * n4 + i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (accumulate) {
    const float4 o = dw[i];
    a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
  }
  dw[i] = a;
}

__global__ void __launch_bounds__(256) wgrad_slab_reduce_k(const float4* __restrict__ slab, int nb,
                                                           float4* __restrict__ dw, int n4, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int k = 0;
  for (; k + 1 < nb; k += 2) {
    const float4 u = slab[(int64_t)k * n4 + i], v = slab[(int64_t)(k + 1) * n4 + i];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (k < nb) {
    const float4 u = slab[(int64_t)k * n4 + i];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  if (accumulate) {
    const float4 o = dw[i];
    a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
  }
  dw[i] = a;
}

// ---- wide layers: C, K multiples of 64 / 128 ---------------------------------------------
// ResNet-50 stages 2-4 (128 ch @ 28x28, 256 @ 14x14, 512 @ 7x7): the filter bank no longer
// fits in LDS, so a block owns a pixel tile (TH full rows of IMG images, padded to 7
// 16-pixel blocks) x 128 output channels and walks K = (64-channel chunk, tap):
//   * per chunk the tile's halo [IMG][TH+2][W+2][64] is DMA'd once and serves all 9 taps
//     (the implicit-GEMM loaders fetch it 9 times);
//   * per (chunk, tap) the 128 x 64 filter slice is DMA'd (16 KiB, L2-resident: every
//     pixel tile of a channel block reads the same slices);
//   * single LDS stage (39 KiB) and <= 128 registers: 4 blocks per CU hide each other's
//     DMA waits (the short-K regime, cf. the gemm_core tile 3).
// Waves own two 16-channel blocks x all 7 pixel blocks (14 accumulator tiles D[co][px]).
constexpr int WPB = 7;                 // pixel blocks per tile
constexpr int WBN = 128;               // output channels per block
constexpr int WSL = WBN * 128;         // one filter slice image [128 co][64 ci], 16 KiB

template <int WD, int TH, int IMG>
struct WGeo {
  static constexpr int HP = TH + 2, WP = WD + 2;
  static constexpr int POS = IMG * HP * WP;                  // halo positions
  static constexpr int POS8 = (POS + 7) / 8 * 8;
  static constexpr int PXT = IMG * TH * WD;                  // real pixels per tile
  static_assert(PXT <= WPB * 16, "tile exceeds 7 pixel blocks");
};

template <int WD, int TH, int IMG>
__global__ __launch_bounds__(256, 4) void conv3x3_wide_k(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                         bf16* __restrict__ y, const void* cin, int cin_f32,
                                                         float* colstats, BnB bn, int N, int H, int C, int K) {
  using G = WGeo<WD, TH, IMG>;
  __shared__ __attribute__((aligned(16))) char smem[G::POS8 * 128 + WSL];
  char* halo = smem;
  char* wl = smem + G::POS8 * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kblocks = K / WBN;
  const int cob = blockIdx.x % kblocks, tile = blockIdx.x / kblocks;
  const int tpi = (H + TH - 1) / TH;                         // row tiles per image (IMG == 1)
  const int n0 = IMG == 1 ? tile / tpi : tile * IMG;
  const int r0 = IMG == 1 ? (tile - n0 * tpi) * TH : 0;

  // this lane's pixel slots: halo base position (tap (0,0)) and output pixel of each block
  int hb[WPB];
  int64_t opx[WPB];
#pragma unroll
  for (int b = 0; b < WPB; ++b) {
    const int sidx = b * 16 + (lane & 15);
    const bool v = sidx < G::PXT;
    const int sc = v ? sidx : 0;
    const int il = sc / (TH * WD), rem = sc - il * (TH * WD), ty = rem / WD, tx = rem - ty * WD;
    hb[b] = (il * G::HP + ty) * G::WP + tx;
    const int oh = r0 + ty, n = n0 + il;
    opx[b] = (v && oh < H && n < N) ? ((int64_t)n * H + oh) * WD + tx : -1;
  }
  const int q4 = lane >> 4;

  float cs[8], cq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { cs[i] = 0.f; cq[i] = 0.f; }
  v4f acc[WPB][2];
#pragma unroll
  for (int b = 0; b < WPB; ++b)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[b][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nch = C / 64;
  for (int ch = 0; ch < nch; ++ch) {
    for (int tap = 0; tap < 9; ++tap) {
      if (tap == 0) {
        // halo of chunk ch: POS8/8 wave instructions of 8 positions x 8 chunks
        for (int I = wave; I < G::POS8 / 8; I += 4) {
          const int pos = I * 8 + (lane >> 3);
          const int c = (lane & 7) ^ (pos & 7);
          const int il = pos / (G::HP * G::WP), rr = pos - il * (G::HP * G::WP);
          const int hy = rr / G::WP, hx = rr - hy * G::WP;
          const int ih = r0 + hy - 1, iw = hx - 1, n = n0 + il;
          const bool ok = pos < G::POS && n < N && ih >= 0 && ih < H && iw >= 0 && iw < WD;
          const void* src = ok ? (const void*)(x + (((int64_t)n * H + ih) * WD + iw) * C + ch * 64 + c * 8)
                               : (const void*)g_zero16;
          dma16(src, halo + I * 1024);
        }
      }
      // filter slice: rows co (128), chunks of ci ch*64 .. +64 of tap `tap`
      for (int I = wave; I < WBN / 8; I += 4) {
        const int co = I * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (co & 7);
        dma16(w + (((int64_t)(cob * WBN + co)) * 9 + tap) * C + ch * 64 + c * 8, wl + I * 1024);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int kh = tap / 3, kw = tap - kh * 3, toff = kh * G::WP + kw;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + q4;
        v8s wf[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) wf[j] = *reinterpret_cast<const v8s*>(wl + swz((2 * wave + j) * 16 + (lane & 15), c));
#pragma unroll
        for (int b = 0; b < WPB; ++b) {
          const v8s pf = *reinterpret_cast<const v8s*>(halo + swz(hb[b] + toff, c));
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], pf, acc[b][j], 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }

  // epilogue: lane holds channels cob*128 + (2*wave + j)*16 + 4*q4 + i of its pixels
#pragma unroll
  for (int b = 0; b < WPB; ++b) {
    if (opx[b] < 0) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = cob * WBN + (2 * wave + j) * 16 + 4 * q4;
      float v[4] = {acc[b][j][0], acc[b][j][1], acc[b][j][2], acc[b][j][3]};
      const Bn4 b4 = colstats ? bn_load4(bn, opx[b] * K + co) : Bn4{make_uint2(0, 0), 0xfu};
      if (cin) {
        if (cin_f32) {
          const float4 a = *reinterpret_cast<const float4*>((const float*)cin + opx[b] * K + co);
          v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        } else {
          const uint2 a = *reinterpret_cast<const uint2*>((const bf16*)cin + opx[b] * K + co);
          v[0] += bf16_bits_to_f((unsigned short)(a.x & 0xffffu));
          v[1] += bf16_bits_to_f((unsigned short)(a.x >> 16));
          v[2] += bf16_bits_to_f((unsigned short)(a.y & 0xffffu));
          v[3] += bf16_bits_to_f((unsigned short)(a.y >> 16));
        }
      }
      if (bn.store) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (b4.mk >> i) & 1u ? v[i] : 0.f;
      }
      unsigned short h[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) h[i] = f_to_bf16_bits(v[i]);
      if (colstats) stats4(bn, b4, h, cs + j * 4, cq + j * 4);
      uint2 pk;
      pk.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      pk.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
      *reinterpret_cast<uint2*>(y + opx[b] * K + co) = pk;
    }
  }
  if (colstats) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        cs[i] += __shfl_xor(cs[i], o, 64);
        cq[i] += __shfl_xor(cq[i], o, 64);
      }
    float* cst = colstats + (bn.rep > 1 ? (int64_t)(tile % bn.rep) * 2 * K : 0);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = cob * WBN + (2 * wave + j) * 16 + 4 * q4 + i;
          unsafeAtomicAdd(cst + co, cs[j * 4 + i]);
          unsafeAtomicAdd(cst + K + co, cq[j * 4 + i]);
        }
    }
  }
}

// w'[ci][tap][co] = w[co][8 - tap][ci] for any C, K
__global__ void __launch_bounds__(256) flip_bank_any_k(const bf16* __restrict__ w, bf16* __restrict__ wt, int C,
                                                       int K) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)C * 9 * K) return;
  const int ci = (int)(i / (9 * K)), r = (int)(i - (int64_t)ci * 9 * K), tap = r / K, co = r - tap * K;
  wt[i] = w[((int64_t)co * 9 + (8 - tap)) * C + ci];
}

template <int WD, int TH, int IMG>
int launch_wide(const bf16* x, const bf16* w, bf16* y, const void* cin, int cin_f32, float* colstats, BnB bn, int N,
                int H, int C, int K, hipStream_t st) {
  const int tiles = IMG == 1 ? N * ((H + TH - 1) / TH) : (N + IMG - 1) / IMG;
  hipLaunchKernelGGL((conv3x3_wide_k<WD, TH, IMG>), dim3(tiles * (K / WBN)), dim3(256), 0, st, x, w, y, cin,
                     cin_f32, colstats, bn, N, H, C, K);
  return (int)hipGetLastError();
}

int dispatch_wide(const bf16* x, const bf16* w, bf16* y, const void* cin, int cin_f32, float* colstats, BnB bn, int N,
                  int H, int W, int C, int K, hipStream_t st) {
  if (W == 56 && H % 2 == 0) return launch_wide<56, 2, 1>(x, w, y, cin, cin_f32, colstats, bn, N, H, C, K, st);
  if (W == 28 && H % 4 == 0) return launch_wide<28, 4, 1>(x, w, y, cin, cin_f32, colstats, bn, N, H, C, K, st);
  if (W == 14 && H % 7 == 0) return launch_wide<14, 7, 1>(x, w, y, cin, cin_f32, colstats, bn, N, H, C, K, st);
  if (W == 7 && H == 7) return launch_wide<7, 7, 2>(x, w, y, cin, cin_f32, colstats, bn, N, H, C, K, st);
  return (int)hipErrorInvalidValue;
}

bool wide_ok(int C, int K, int H, int W) {
  return C % 64 == 0 && K % WBN == 0 && ((W == 56 && H % 2 == 0) || (W == 28 && H % 4 == 0) ||
                                         (W == 14 && H % 7 == 0) || (W == 7 && H == 7));
}

// ---- weight gradient of the wide layers --------------------------------------------------
// Block = (64 output channels, 64 input channels) x a group of pixel tiles (the tiles of
// conv3x3_wide_k, padded to whole 32-pixel k-steps with zero dy rows); per tile the input
// channel chunk's halo and the tile's dy columns are DMA'd into LDS and the 8 waves run the
// conv3x3_c64_wgrad_k reduction (transpose-read operands, 18 accumulator tiles per wave, all
// 9 taps).  Each block stores its fp32 partial [64 co][9][64 ci] into a slab; a reduce sums
// the pixel groups of each channel pair into dW[K][3][3][C].
template <int WD, int TH, int IMG>
__global__ __launch_bounds__(WG_NW * 64, 2) void conv3x3_wide_wgrad_k(const bf16* __restrict__ x,
                                                                     const bf16* __restrict__ dy,
                                                                     float* __restrict__ slab, int N, int H, int C,
                                                                     int K, int groups) {
  using G = WGeo<WD, TH, IMG>;
  constexpr int PXP = (G::PXT + 31) / 32 * 32;
  __shared__ __attribute__((aligned(16))) char smem[G::POS8 * 128 + PXP * 128];
  char* halo = smem;
  char* dyl = smem + G::POS8 * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kb = K / 64, pairs = kb * (C / 64);
  const int pair = blockIdx.x % pairs, grp = blockIdx.x / pairs;
  const int cob = pair % kb, cich = pair / kb;
  const int tpi = (H + TH - 1) / TH;
  const int ntiles = IMG == 1 ? N * tpi : (N + IMG - 1) / IMG;

  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int cb = wave & 3, cib0 = 2 * (wave >> 2);
  const int dof = (p & 1) * 8;
  // halo base positions of the lane's two pixel rows in each of the PXP/32 k-steps are
  // recomputed per step (cheap: compile-time divisors)
  auto hbase = [&](int px) {
    const int pc = px < G::PXT ? px : 0;
    const int il = pc / (TH * WD), rem = pc - il * (TH * WD), ty = rem / WD, tx = rem - ty * WD;
    return (il * G::HP + ty) * G::WP + tx;
  };

  v4f acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[t][j] = v4f{0.f, 0.f, 0.f, 0.f};

  for (int tile = grp; tile < ntiles; tile += groups) {
    const int n0 = IMG == 1 ? tile / tpi : tile * IMG;
    const int r0 = IMG == 1 ? (tile - n0 * tpi) * TH : 0;
    for (int I = wave; I < G::POS8 / 8; I += WG_NW) {
      const int pos = I * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (pos & 7);
      const int il = pos / (G::HP * G::WP), rr = pos - il * (G::HP * G::WP);
      const int hy = rr / G::WP, hx = rr - hy * G::WP;
      const int ih = r0 + hy - 1, iw = hx - 1, n = n0 + il;
      const bool ok = pos < G::POS && n < N && ih >= 0 && ih < H && iw >= 0 && iw < WD;
      const void* src = ok ? (const void*)(x + (((int64_t)n * H + ih) * WD + iw) * C + cich * 64 + c * 8)
                           : (const void*)g_zero16;
      dma16(src, halo + I * 1024);
    }
    for (int I = wave; I < PXP / 8; I += WG_NW) {
      const int px = I * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (px & 7);
      const int il = px / (TH * WD), rem = px - il * (TH * WD), ty = rem / WD, tx = rem - ty * WD;
      const int n = n0 + il, oh = r0 + ty;
      const bool ok = px < G::PXT && n < N && oh < H;
      const void* src = ok ? (const void*)(dy + (((int64_t)n * H + oh) * WD + tx) * K + cob * 64 + c * 8)
                           : (const void*)g_zero16;
      dma16(src, dyl + I * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int st = 0; st < PXP / 32; ++st) {
      const int px0 = st * 32 + 8 * g + q, px1 = px0 + 4;
      const int dch = 2 * cb + (p >> 1);
      const v8s bf = tr_pair(dyl + px0 * 128 + ((dch ^ (px0 & 7)) << 4) + dof,
                             dyl + px1 * 128 + ((dch ^ (px1 & 7)) << 4) + dof);
      const int h0 = hbase(px0), h1 = hbase(px1);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int pos0 = h0 + kh * G::WP + kw, pos1 = h1 + kh * G::WP + kw;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int xch = 2 * (cib0 + j) + (p >> 1);
            const v8s af = tr_pair(halo + pos0 * 128 + ((xch ^ (pos0 & 7)) << 4) + dof,
                                   halo + pos1 * 128 + ((xch ^ (pos1 & 7)) << 4) + dof);
            acc[kh * 3 + kw][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[kh * 3 + kw][j], 0, 0, 0);
          }
        }
    }
    __syncthreads();
  }
  // slab[block][co 64][tap][ci 64]
  float* S = slab + (int64_t)blockIdx.x * 9 * 64 * 64;
  const int co = 16 * cb + (lane & 15);
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      *reinterpret_cast<float4*>(S + ((int64_t)co * 9 + tp) * 64 + 16 * (cib0 + j) + 4 * g) =
          make_float4(acc[tp][j][0], acc[tp][j][1], acc[tp][j][2], acc[tp][j][3]);
}

// dw[co][tap][ci] (+)= sum over the pixel groups of slab[grp*pairs + pair][co%64][tap][ci%64]
__global__ void __launch_bounds__(256) wide_wgrad_reduce_k(const float4* __restrict__ slab, int groups, int pairs,
                                                           int kb, float4* __restrict__ dw, int C, int K,
                                                           int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;       // float4 of dw
  const int64_t n4 = (int64_t)K * 9 * C / 4;
  if (i >= n4) return;
  const int64_t e = i * 4;
  const int co = (int)(e / (9 * C)), r = (int)(e - (int64_t)co * 9 * C), tap = r / C, ci = r - tap * C;
  const int pair = (ci / 64) * kb + co / 64;
  const int64_t off = ((int64_t)(co % 64) * 9 + tap) * 64 + (ci % 64);   // floats within a block slab
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int gi = 0; gi < groups; ++gi) {
    const float4 u = slab[(((int64_t)gi * pairs + pair) * 9 * 64 * 64 + off) / 4];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  if (accumulate) {
    const float4 o = dw[i];
    a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
  }
  dw[i] = a;
}

template <int WD, int TH, int IMG>
int launch_wide_wgrad(const bf16* x, const bf16* dy, float* dw, float* ws, int64_t ws_floats, int accumulate, int N,
                      int H, int C, int K, hipStream_t st) {
  const int pairs = (K / 64) * (C / 64);
  const int ntiles = IMG == 1 ? N * ((H + TH - 1) / TH) : (N + IMG - 1) / IMG;
  int groups = std::max(1, std::min(ntiles, 512 / pairs));
  while ((int64_t)groups * pairs * 9 * 64 * 64 > ws_floats && groups > 1) --groups;
  if ((int64_t)groups * pairs * 9 * 64 * 64 > ws_floats) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((conv3x3_wide_wgrad_k<WD, TH, IMG>), dim3(groups * pairs), dim3(WG_NW * 64), 0, st, x, dy, ws,
                     N, H, C, K, groups);
  HETU_LAUNCH_CHECK();
  const int64_t n4 = (int64_t)K * 9 * C / 4;
  hipLaunchKernelGGL(wide_wgrad_reduce_k, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, (const float4*)ws,
                     groups, pairs, K / 64, (float4*)dw, C, K, accumulate);
  return (int)hipGetLastError();
}

bool wide_wgrad_ok(int C, int K, int H, int W) {
  return C % 64 == 0 && K % 64 == 0 && ((W == 28 && H % 4 == 0) || (W == 14 && H % 7 == 0) || (W == 7 && H == 7));
}
}  // namespace

HETU_API int hetu_conv3x3_c64_supported(int C, int K, int W) { return C == CH && K == CH && W == 56; }

// y[N,H,W,64] = conv3x3(x[N,H,W,64], w[64][3][3][64]), stride 1, pad 1 (NHWC bf16);
// colstats (nullable, csrep x 128 fp32 pre-zeroed) += per-channel sum / sum of squares of y
// (image n into replica n % csrep)
HETU_API int hetu_conv3x3_c64_fwd(const void* x, const void* w, void* y, float* colstats, int N, int H, int W,
                                  int csrep, hipStream_t st) {
  if ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)y)) & 15) return (int)hipErrorInvalidValue;
  return dispatch_c64((const bf16*)x, (const bf16*)w, (bf16*)y, nullptr, 0, colstats, BnB{nullptr, nullptr, 0, csrep},
                      N, H, W, st);
}

// dx[N,H,W,64] = conv3x3^T(dy, w) (+ acc: bf16 or fp32 [N,H,W,64]); wt: 64*9*64 bf16 scratch.
// bnsums (nullable, 128 fp32 pre-zeroed) += sum(dx') / sum(dx' * bnx) per channel, dx' = dx
// masked by bnmask (see BnB): the reduction of the backward of the BN that produced x;
// bnstore: dx is stored masked; bnrep: bnsums holds that many replicas ([bnrep][128], block
// of image n adds into replica n % bnrep)
HETU_API int hetu_conv3x3_c64_dgrad(const void* dy, const void* w, void* wt, void* dx, const void* acc, int acc_f32,
                                    int N, int H, int W, float* bnsums, const void* bnx, const uint8_t* bnmask,
                                    int bnstore, int bnrep, hipStream_t st) {
  if ((((uintptr_t)dy) | ((uintptr_t)wt) | ((uintptr_t)dx) | ((uintptr_t)acc) | ((uintptr_t)bnx)) & 15)
    return (int)hipErrorInvalidValue;
  if (bnsums && !bnx) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(flip_bank_k, dim3((CH * 9 * CH + 255) / 256), dim3(256), 0, st, (const bf16*)w, (bf16*)wt);
  HETU_LAUNCH_CHECK();
  return dispatch_c64((const bf16*)dy, (const bf16*)wt, (bf16*)dx, acc, acc_f32, bnsums,
                      BnB{bnsums ? (const bf16*)bnx : nullptr, bnsums ? bnmask : nullptr,
                          (bnsums && bnmask && bnstore) ? 1 : 0, bnsums ? bnrep : 0},
                      N, H, W, st);
}

// slab floats hetu_conv3x3_c64_wgrad needs for a batch of N images
HETU_API int64_t hetu_conv3x3_c64_wgrad_ws(int N) { return (int64_t)N * 9 * CH * CH; }

// dw[64][3][3][64] fp32 (+)= weight gradient of the 3x3/s1/p1 64->64 convolution;
// x, dy [N,H,W,64] bf16; ws: hetu_conv3x3_c64_wgrad_ws(N) floats
HETU_API int hetu_conv3x3_c64_wgrad(const void* x, const void* dy, float* dw, float* ws, int accumulate, int N,
                                    int H, int W, hipStream_t st) {
  if ((((uintptr_t)x) | ((uintptr_t)dy) | ((uintptr_t)dw) | ((uintptr_t)ws)) & 15) return (int)hipErrorInvalidValue;
  if (W != 56) return (int)hipErrorInvalidValue;
  static const bool asm_tr = [] {
    const char* e = getenv("HETU_C64_WGRAD_ASM");
    return e == nullptr || e[0] != '0';
  }();
  if (asm_tr)
    hipLaunchKernelGGL((conv3x3_c64_wgrad_k<56, 4, true>), dim3(N), dim3(WG_NW * 64), 0, st, (const bf16*)x,
                       (const bf16*)dy, ws, H);
  else
    hipLaunchKernelGGL((conv3x3_c64_wgrad_k<56, 4, false>), dim3(N), dim3(WG_NW * 64), 0, st, (const bf16*)x,
                       (const bf16*)dy, ws, H);
  HETU_LAUNCH_CHECK();
  const int n4 = 9 * CH * CH / 4;
  if (N >= 64 && !getenv("HETU_SLAB_ONEPASS")) {
    const int G = 16, per = (N + G - 1) / G;
    hipLaunchKernelGGL(wgrad_slab_group_k, dim3((n4 + 255) / 256, (N + per - 1) / per), dim3(256), 0, st,
                       (float4*)ws, N, per, n4);
    hipLaunchKernelGGL(wgrad_slab_final_k, dim3((n4 + 255) / 256), dim3(256), 0, st, (const float4*)ws, N, per,
                       (float4*)dw, n4, accumulate);
  } else {
    hipLaunchKernelGGL(wgrad_slab_reduce_k, dim3((n4 + 255) / 256), dim3(256), 0, st, (const float4*)ws, N,
                       (float4*)dw, n4, accumulate);
  }
  return (int)hipGetLastError();
}

HETU_API int hetu_conv3x3_wide_supported(int C, int K, int H, int W) { return wide_ok(C, K, H, W); }

// y[N,H,W,K] = conv3x3(x[N,H,W,C], w[K][3][3][C]) (stride 1, pad 1), C % 64 == 0, K % 128 == 0
// (colstats: csrep replicas of [2K], pixel tile t into replica t % csrep)
HETU_API int hetu_conv3x3_wide_fwd(const void* x, const void* w, void* y, float* colstats, int N, int H, int W, int C,
                                   int K, int csrep, hipStream_t st) {
  if (!wide_ok(C, K, H, W) || ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)y)) & 15))
    return (int)hipErrorInvalidValue;
  return dispatch_wide((const bf16*)x, (const bf16*)w, (bf16*)y, nullptr, 0, colstats, BnB{nullptr, nullptr, 0, csrep},
                       N, H, W, C, K, st);
}

// dx[N,H,W,C] = conv3x3^T(dy[N,H,W,K], w) (+ acc), K % 64 == 0, C % 128 == 0; wt: C*9*K bf16;
// bnsums / bnx / bnmask / bnstore / bnrep as hetu_conv3x3_c64_dgrad (bnrep * 2*C floats)
HETU_API int hetu_conv3x3_wide_dgrad(const void* dy, const void* w, void* wt, void* dx, const void* acc, int acc_f32,
                                     int N, int H, int W, int C, int K, float* bnsums, const void* bnx,
                                     const uint8_t* bnmask, int bnstore, int bnrep, hipStream_t st) {
  if (!wide_ok(K, C, H, W) ||
      ((((uintptr_t)dy) | ((uintptr_t)wt) | ((uintptr_t)dx) | ((uintptr_t)acc) | ((uintptr_t)bnx)) & 15))
    return (int)hipErrorInvalidValue;
  if (bnsums && !bnx) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)C * 9 * K;
  hipLaunchKernelGGL(flip_bank_any_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const bf16*)w, (bf16*)wt,
                     C, K);
  HETU_LAUNCH_CHECK();
  return dispatch_wide((const bf16*)dy, (const bf16*)wt, (bf16*)dx, acc, acc_f32, bnsums,
                       BnB{bnsums ? (const bf16*)bnx : nullptr, bnsums ? bnmask : nullptr,
                           (bnsums && bnmask && bnstore) ? 1 : 0, bnsums ? bnrep : 0},
                       N, H, W, K, C, st);
}

HETU_API int hetu_conv3x3_wide_wgrad_supported(int C, int K, int H, int W) { return wide_wgrad_ok(C, K, H, W); }

// slab floats the wide weight gradient needs at most (<= 512 blocks of 64x9x64 partials)
HETU_API int64_t hetu_conv3x3_wide_wgrad_ws(int C, int K) {
  const int pairs = (K / 64) * (C / 64);
  return (int64_t)std::max(pairs, 512 / std::max(pairs, 1) * pairs) * 9 * 64 * 64;
}

// dw[K][3][3][C] fp32 (+)= weight gradient of the 3x3/s1/p1 convolution x[N,H,W,C] -> dy[N,H,W,K]
HETU_API int hetu_conv3x3_wide_wgrad(const void* x, const void* dy, float* dw, float* ws, int64_t ws_floats,
                                     int accumulate, int N, int H, int W, int C, int K, hipStream_t st) {
  if (!wide_wgrad_ok(C, K, H, W) || ((((uintptr_t)x) | ((uintptr_t)dy) | ((uintptr_t)dw) | ((uintptr_t)ws)) & 15))
    return (int)hipErrorInvalidValue;
  const bf16 *xb = (const bf16*)x, *gb = (const bf16*)dy;
  if (W == 28) return launch_wide_wgrad<28, 4, 1>(xb, gb, dw, ws, ws_floats, accumulate, N, H, C, K, st);
  if (W == 14) return launch_wide_wgrad<14, 7, 1>(xb, gb, dw, ws, ws_floats, accumulate, N, H, C, K, st);
  return launch_wide_wgrad<7, 7, 2>(xb, gb, dw, ws, ws_floats, accumulate, N, H, C, K, st);
}
