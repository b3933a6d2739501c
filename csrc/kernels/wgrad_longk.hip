// Weight gradients with a small output and a very long reduction: dW[M][N] = sum_p
// A[p][m] * B[p][n] with both operands pixel-major ([P][M], [P][N], channels contiguous)
// -- the 1x1 convolutions of ResNet-50 stage 1 (64 x 64 outputs over 802,816 pixels).
// The 128x128 MFMA tiles spend 3/4 of their MFMAs and half their staging on zero rows
// here (103 us vs MIOpen's 53-61 us).  This kernel tiles the output in 64x64 blocks and
// splits the pixels over ~1024 workgroups:
//   * per 64-pixel K-step both 64-channel operand slices are DMA'd into LDS
//     ([64 px][64 ch], 16-byte chunks XOR-swizzled by pixel), double buffered;
//   * the MFMA operands need 8 consecutive pixels per lane: both come from the hardware
//     transpose read (T10), lane 4q+p of a 16-lane group addressing pixel row q and
//     channels 4p..4p+3;
//   * 4 waves own a 32x32 quadrant each (2x2 mfma_f32_16x16x32_bf16 tiles);
//   * each workgroup stores its fp32 partial tile into a slab; a vectorised reduce sums
//     the slabs into dW (overwrite or accumulate).
#include "common.h"
#include "lds_tr.h"

using namespace hetu;

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

static __device__ __attribute__((aligned(64))) bf16 g_zero_lk[32];

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// asm transposing reads (lds_tr.h): the next K-step's DMA stays in flight; frag_wait()
// before the MFMAs
__device__ __forceinline__ v8s tr_pair(const char* a, const char* b) {
  v4s x = ds_tr16(a);
  v4s y = ds_tr16(b);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

constexpr int KS = 64;              // pixels per K-step
constexpr int SL = KS * 128;        // one [64 px][64 ch] slice, 8 KiB

// grid: (M/64) * (N/64) output tiles x splits; block z-major: tile = blockIdx.x % tiles
__global__ void __launch_bounds__(256, 2) wgrad_longk_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        float* __restrict__ slab, int64_t P, int M, int N, int lda,
                                                        int ldb, int kps) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * SL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tn = N / 64, tiles = (M / 64) * tn;
  const int tile = blockIdx.x % tiles, split = blockIdx.x / tiles;
  const int m0 = (tile / tn) * 64, n0 = (tile % tn) * 64;
  const int64_t nks = (P + KS - 1) / KS;
  const int64_t ks0 = (int64_t)split * kps, ks1 = ks0 + kps < nks ? ks0 + kps : nks;

  // stage K-step ks into buffer b: 8 instructions per operand (8 pixels x 8 chunks each),
  // two per wave per operand
  auto stage = [&](int64_t ks, int b) {
    char* As = smem + b * 2 * SL;
    char* Bs = As + SL;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int I = wave * 2 + u;
      const int px = I * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (px & 7);
      const int64_t p = ks * KS + px;
      const bool ok = p < P;
      dma16(ok ? (const void*)(A + p * lda + m0 + c * 8) : (const void*)g_zero_lk, As + I * 1024);
      dma16(ok ? (const void*)(B + p * ldb + n0 + c * 8) : (const void*)g_zero_lk, Bs + I * 1024);
    }
  };

  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int wm = wave & 1, wn = wave >> 1;
  const int dof = (pp & 1) * 8;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  if (ks0 < ks1) stage(ks0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t ks = ks0; ks < ks1; ++ks) {
    const int cur = (int)((ks - ks0) & 1);
    if (ks + 1 < ks1) stage(ks + 1, cur ^ 1);
    const char* As = smem + cur * 2 * SL;
    const char* Bs = As + SL;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int px0 = s2 * 32 + 8 * g + q, px1 = px0 + 4;
      v8s af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ch = 2 * (wm * 2 + i) + (pp >> 1);     // 16-byte chunk of channels 16*blk + 4pp
        af[i] = tr_pair(As + px0 * 128 + ((ch ^ (px0 & 7)) << 4) + dof, As + px1 * 128 + ((ch ^ (px1 & 7)) << 4) + dof);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ch = 2 * (wn * 2 + j) + (pp >> 1);
        bfr[j] = tr_pair(Bs + px0 * 128 + ((ch ^ (px0 & 7)) << 4) + dof, Bs + px1 * 128 + ((ch ^ (px1 & 7)) << 4) + dof);
      }
      frag_wait();
      // D[n][m]: lane holds 4 consecutive n (columns of dW) for one m -> float4 stores
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // partial tile: slab[block][64][64], row m (local), 4 columns n per lane
  float* S = slab + (int64_t)blockIdx.x * 64 * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = (wm * 2 + i) * 16 + (lane & 15);
      const int n = (wn * 2 + j) * 16 + 4 * g;
      *reinterpret_cast<float4*>(S + m * 64 + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
}

// dw[m][n] (ldd) (+)= sum over splits of slab[split*tiles + tile][m%64][n%64]
__global__ void __launch_bounds__(256) wgrad_longk_reduce_k(const float4* __restrict__ slab, int splits, int tiles,
                                                            int tn, float* __restrict__ dw, int M, int N, int64_t ldd,
                                                            int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // float4 index over M*N
  if (i >= (int64_t)M * N / 4) return;
  const int m = (int)(i * 4 / N), n = (int)(i * 4 - (int64_t)m * N);
  const int tile = (m / 64) * tn + n / 64;
  const int64_t off = ((int64_t)(m % 64) * 64 + (n % 64)) / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int s = 0;
  for (; s + 1 < splits; s += 2) {
    const float4 u = slab[((int64_t)s * tiles + tile) * 1024 + off];
    const float4 v = slab[((int64_t)(s + 1) * tiles + tile) * 1024 + off];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (s < splits) {
    const float4 u = slab[((int64_t)s * tiles + tile) * 1024 + off];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  float4* d = reinterpret_cast<float4*>(dw + m * ldd + n);
  if (accumulate) {
    const float4 o = *d;
    a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
  }
  *d = a;
}

}  // namespace

// slab floats for `splits` pixel splits of an M x N product
HETU_API int64_t hetu_wgrad_longk_ws(int M, int N, int splits) { return (int64_t)splits * M * N; }

// dw[M][N] fp32 (ldd, 16-byte aligned rows) (+)= A[P][M]^T (lda) @ B[P][N] (ldb), bf16,
// M, N multiples of 64, lda / ldb multiples of 8, 16-byte aligned bases; ws >= splits*M*N
HETU_API int hetu_wgrad_longk(const void* A, const void* B, float* dw, float* ws, int64_t P, int M, int N, int lda,
                              int ldb, int64_t ldd, int splits, int accumulate, hipStream_t st) {
  if (M % 64 || N % 64 || lda % 8 || ldb % 8 || ldd % 4 || splits < 1 ||
      ((((uintptr_t)A) | ((uintptr_t)B) | ((uintptr_t)dw) | ((uintptr_t)ws)) & 15))
    return (int)hipErrorInvalidValue;
  const int tiles = (M / 64) * (N / 64);
  const int64_t nks = (P + KS - 1) / KS;
  int kps = (int)((nks + splits - 1) / splits);
  splits = (int)((nks + kps - 1) / kps);
  hipLaunchKernelGGL(wgrad_longk_k, dim3((unsigned)(tiles * splits)), dim3(256), 0, st, (const bf16*)A,
                     (const bf16*)B, ws, P, M, N, lda, ldb, kps);
  HETU_LAUNCH_CHECK();
  const int64_t n4 = (int64_t)M * N / 4;
  hipLaunchKernelGGL(wgrad_longk_reduce_k, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, (const float4*)ws,
                     splits, tiles, N / 64, dw, M, N, ldd, accumulate);
  return (int)hipGetLastError();
}
