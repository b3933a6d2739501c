// Small / skinny GEMMs that the MFMA tiles cannot take: an operand extent or leading
// dimension that is not a multiple of 8 (BERT's 2-way NSP head, N = 2), or too few
// outputs to fill even one 128x128 tile with useful work (the 64-row pooler).  One wave
// per output element: the lanes split K (strided fp32 FMAs), a wave64 reduction, then
// the same epilogue as the MFMA kernels (alpha, beta * Cin, bias on N or M, ReLU / GELU).
// hipBLASLt took ~20 us per such call (launch-heuristic bound); these take a few us.
#include "common.h"

using namespace hetu;

namespace {

template <typename T>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
  return to_f(reinterpret_cast<const T*>(p)[i]);
}

__device__ __forceinline__ float erf_approx(float x) { return erff(x); }

template <typename TA, typename TB>
__global__ void __launch_bounds__(256) gemm_small_k(const void* __restrict__ A, const void* __restrict__ B,
                                                    void* __restrict__ C, const void* __restrict__ Cin,
                                                    const float* __restrict__ bias, int64_t M, int64_t N, int64_t K,
                                                    int64_t sam, int64_t sak, int64_t sbk, int64_t sbn, int64_t ldc,
                                                    int64_t ldcin, float alpha, float beta, int act, int out_f32,
                                                    int cin_f32, int bias_on_m) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t o = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); o < M * N; o += waves) {
    const int64_t m = o / N, n = o - m * N;
    float a0 = 0.f, a1 = 0.f;
    int64_t k = lane;
    for (; k + 64 < K; k += 128) {
      a0 += ld<TA>(A, m * sam + k * sak) * ld<TB>(B, k * sbk + n * sbn);
      a1 += ld<TA>(A, m * sam + (k + 64) * sak) * ld<TB>(B, (k + 64) * sbk + n * sbn);
    }
    if (k < K) a0 += ld<TA>(A, m * sam + k * sak) * ld<TB>(B, k * sbk + n * sbn);
    float v = wave_sum(a0 + a1) * alpha;
    if (lane == 0) {
      if (Cin && beta != 0.f)
        v += beta * (cin_f32 ? ((const float*)Cin)[m * ldcin + n] : to_f(((const bf16*)Cin)[m * ldcin + n]));
      if (bias) v += bias[bias_on_m ? m : n];
      if (act == 1) v = v > 0.f ? v : 0.f;
      else if (act == 2) v = 0.5f * v * (1.f + erf_approx(v * 0.70710678118f));
      if (out_f32) ((float*)C)[m * ldc + n] = v;
      else ((bf16*)C)[m * ldc + n] = __float2bfloat16(v);
    }
  }
}

}  // namespace

// C[m][n] (ldc) = act(alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] + beta * Cin + bias)
// a_f32 / b_f32: operand dtypes (else bf16); any strides, M*N outputs in a grid-stride loop
HETU_API int hetu_gemm_small(const void* A, const void* B, void* C, const void* Cin, const float* bias, int64_t M,
                             int64_t N, int64_t K, int64_t sam, int64_t sak, int64_t sbk, int64_t sbn, int64_t ldc,
                             int64_t ldcin, int a_f32, int b_f32, float alpha, float beta, int act, int out_f32,
                             int cin_f32, int bias_on_m, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  int64_t blocks = (M * N + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  const dim3 g((unsigned)blocks), b(256);
#define GS(TA, TB)                                                                                                    \
  hipLaunchKernelGGL((gemm_small_k<TA, TB>), g, b, 0, st, A, B, C, Cin, bias, M, N, K, sam, sak, sbk, sbn, ldc,      \
                     ldcin, alpha, beta, act, out_f32, cin_f32, bias_on_m)
  if (a_f32 && b_f32) GS(float, float);
  else if (a_f32) GS(float, bf16);
  else if (b_f32) GS(bf16, float);
  else GS(bf16, bf16);
#undef GS
  return (int)hipGetLastError();
}
