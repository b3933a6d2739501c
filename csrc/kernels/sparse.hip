// CSR sparse x dense products for gfx950 (reference src/ops/CuSparseCsrmm.cu,
// CuSparseCsrmv.cu; SURVEY §2.5 / §2.7 "cuSPARSE -> CSR SpMV/SpMM kernel").
//
//   csrmm : C[m, :] (+)= sum_{j in row m, c0 <= col[j] < c1} val[j] * B[col[j] - c0, :]
//           one wave per sparse row, lanes across the dense columns (4 per lane,
//           coalesced B-row reads); the [c0, c1) column window is the DistGCN-1.5D
//           stage slice (reference CuSparseCsrmm.cu spmm_kernel start/end).  No
//           atomics: the transposed product is served by an explicitly transposed
//           CSR (built once per matrix on the host), so results are deterministic.
//   csrmv : y[m] = sum_j val[j] * x[col[j]]   one wave per row, lanes over the
//           row's nonzeros, wave64 reduction.
#include "common.h"

namespace hetu {

template <typename T>
__global__ void __launch_bounds__(256) csrmm_k(const int* __restrict__ rp, const int* __restrict__ ci,
                                                const float* __restrict__ val, const T* __restrict__ B,
                                                T* __restrict__ C, int M, int N, int64_t ldb,
                                                int64_t ldc, int c0, int c1, float alpha,
                                                int accumulate) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int j0 = rp[row], j1 = rp[row + 1];
  for (int nb = 0; nb < N; nb += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = j0; j < j1; ++j) {
      const int col = ci[j];
      if (col < c0 || col >= c1) continue;
      const float v = val[j];
      const T* b = B + (int64_t)(col - c0) * ldb;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nb + lane + 64 * q;
        if (n < N) acc[q] += v * to_f(b[n]);
      }
    }
    T* c = C + (int64_t)row * ldc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nb + lane + 64 * q;
      if (n < N) {
        float r = alpha * acc[q];
        if (accumulate) r += to_f(c[n]);
        c[n] = from_f<T>(r);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) csrmv_k(const int* __restrict__ rp, const int* __restrict__ ci,
                                                const float* __restrict__ val, const T* __restrict__ x,
                                                T* __restrict__ y, int M) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float s = 0.f;
  for (int j = rp[row] + lane; j < rp[row + 1]; j += 64) s += val[j] * to_f(x[ci[j]]);
  s = wave_sum(s);
  if (lane == 0) y[row] = from_f<T>(s);
}

}  // namespace hetu

using namespace hetu;

HETU_API int hetu_csrmm(const int* rp, const int* ci, const float* val, const void* B, void* C, int M,
                        int N, int64_t ldb, int64_t ldc, int c0, int c1, float alpha, int accumulate,
                        int is_bf16, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  dim3 grid((M + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL(csrmm_k<bf16>, grid, dim3(256), 0, st, rp, ci, val, (const bf16*)B, (bf16*)C, M,
                       N, ldb, ldc, c0, c1, alpha, accumulate);
  else
    hipLaunchKernelGGL(csrmm_k<float>, grid, dim3(256), 0, st, rp, ci, val, (const float*)B, (float*)C,
                       M, N, ldb, ldc, c0, c1, alpha, accumulate);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_csrmv(const int* rp, const int* ci, const float* val, const void* x, void* y, int M,
                        int is_bf16, hipStream_t st) {
  if (M <= 0) return 0;
  dim3 grid((M + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL(csrmv_k<bf16>, grid, dim3(256), 0, st, rp, ci, val, (const bf16*)x, (bf16*)y, M);
  else
    hipLaunchKernelGGL(csrmv_k<float>, grid, dim3(256), 0, st, rp, ci, val, (const float*)x, (float*)y, M);
  HETU_LAUNCH_CHECK();
  return 0;
}
