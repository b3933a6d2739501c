// LayerNorm over the last dimension + Philox dropout, gfx950.
//
// LayerNorm replaces src/ops/LayerNorm.cu (forward: block per row with
// E[x^2]-E[x]^2 variance; backward: 3 elementwise kernels + 4 cuDNN reductions +
// chunk workspaces).  Here: one wave per row, two-pass mean/variance in fp32,
// and a backward that writes dx in the same row pass while each wave keeps its
// own dgamma/dbeta partial slab (wave-exclusive, no atomics), folded by a
// second column-sum kernel.
#include "common.h"

namespace hetu {

template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_k(const T* __restrict__ x, const float* __restrict__ g,
                                                 const float* __restrict__ b, T* __restrict__ y,
                                                 float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                 int64_t R, int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  float s = 0.f;
  for (int j = lane; j < N; j += 64) s += to_f(xr[j]);
  const float mean = wave_sum(s) / (float)N;
  float q = 0.f;
  for (int j = lane; j < N; j += 64) {
    float d = to_f(xr[j]) - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)N + eps);
  T* yr = y + row * N;
  for (int j = lane; j < N; j += 64) yr[j] = from_f<T>((to_f(xr[j]) - mean) * rstd * g[j] + b[j]);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                 const float* __restrict__ g, const float* __restrict__ mean,
                                                 const float* __restrict__ rstd, T* __restrict__ dx,
                                                 float* __restrict__ ws_g, float* __restrict__ ws_b,
                                                 int64_t R, int N, int nwaves) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nwaves) return;
  float* pg = ws_g + (int64_t)w * N;
  float* pb = ws_b + (int64_t)w * N;
  for (int j = lane; j < N; j += 64) { pg[j] = 0.f; pb[j] = 0.f; }
  for (int64_t row = w; row < R; row += nwaves) {
    const T* xr = x + row * N;
    const T* gr = dy + row * N;
    const float mu = mean[row], rs = rstd[row];
    float a = 0.f, c = 0.f;
    for (int j = lane; j < N; j += 64) {
      float xh = (to_f(xr[j]) - mu) * rs;
      float gy = to_f(gr[j]);
      float gg = gy * g[j];
      a += gg;
      c += gg * xh;
      pg[j] += gy * xh;
      pb[j] += gy;
    }
    a = wave_sum(a) / (float)N;
    c = wave_sum(c) / (float)N;
    T* dr = dx + row * N;
    for (int j = lane; j < N; j += 64) {
      float xh = (to_f(xr[j]) - mu) * rs;
      float gg = to_f(gr[j]) * g[j];
      dr[j] = from_f<T>(rs * (gg - a - xh * c));
    }
  }
}

__global__ void col_sum2_k(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ oa,
                           float* __restrict__ ob, int rows, int N) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  float sa = 0.f, sb = 0.f;
  for (int r = 0; r < rows; ++r) {
    sa += a[(int64_t)r * N + j];
    sb += b[(int64_t)r * N + j];
  }
  oa[j] = sa;
  ob[j] = sb;
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_k(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                  float keep, uint64_t seed) {
  const float inv = 1.f / keep;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    uint4 r = Philox::gen(seed, (uint64_t)(i >> 2));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i + k < n) {
        float u = Philox::u01(rr[k]);
        y[i + k] = from_f<T>(u < keep ? to_f(x[i + k]) * inv : 0.f);
      }
    }
  }
}

}  // namespace hetu

using namespace hetu;

HETU_API int hetu_layernorm_fwd(const void* x, const float* g, const float* b, void* y, float* mean,
                                float* rstd, int64_t R, int N, float eps, int is_bf16,
                                hipStream_t st) {
  dim3 grid((unsigned)((R + 3) / 4));
  if (is_bf16) hipLaunchKernelGGL(ln_fwd_k<bf16>, grid, dim3(256), 0, st, (const bf16*)x, g, b, (bf16*)y, mean, rstd, R, N, eps);
  else hipLaunchKernelGGL(ln_fwd_k<float>, grid, dim3(256), 0, st, (const float*)x, g, b, (float*)y, mean, rstd, R, N, eps);
  HETU_LAUNCH_CHECK();
  return 0;
}

// ws: 2 * nwaves * N floats
HETU_API int hetu_layernorm_bwd(const void* dy, const void* x, const float* g, const float* mean,
                                const float* rstd, void* dx, float* dg, float* db, float* ws,
                                int64_t R, int N, int nwaves, int is_bf16, hipStream_t st) {
  dim3 grid((unsigned)((nwaves + 3) / 4));
  float* wg = ws;
  float* wb = ws + (int64_t)nwaves * N;
  if (is_bf16) hipLaunchKernelGGL(ln_bwd_k<bf16>, grid, dim3(256), 0, st, (const bf16*)dy, (const bf16*)x, g, mean, rstd, (bf16*)dx, wg, wb, R, N, nwaves);
  else hipLaunchKernelGGL(ln_bwd_k<float>, grid, dim3(256), 0, st, (const float*)dy, (const float*)x, g, mean, rstd, (float*)dx, wg, wb, R, N, nwaves);
  hipLaunchKernelGGL(col_sum2_k, dim3((N + 255) / 256), dim3(256), 0, st, wg, wb, dg, db, nwaves, N);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_dropout(const void* x, void* y, int64_t n, float keep, int64_t seed, int is_bf16,
                          hipStream_t st) {
  int grid = stream_grid((n + 3) / 4, 256, 1);
  if (is_bf16) hipLaunchKernelGGL(dropout_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n, keep, (uint64_t)seed);
  else hipLaunchKernelGGL(dropout_k<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, n, keep, (uint64_t)seed);
  HETU_LAUNCH_CHECK();
  return 0;
}
