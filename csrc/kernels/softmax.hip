// Row softmax, log-softmax and fused softmax-cross-entropy for gfx950.
//
// Replaces src/ops/Softmax.cu (1 block x 1024 threads, one thread per row),
// CudnnSoftmax.cu, SoftmaxCrossEntropy.cu, SoftmaxCrossEntropySparse.cu and
// CudnnSoftmaxEntropy.cu of the reference: one 64-lane wave per row, online
// max/sum in registers, wave64 shuffle reductions, loss and gradient in a single
// pass each.
#include "common.h"

namespace hetu {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i) { return to_f(p[i]); }

// one wave per row, online (max, sum) merge
template <typename T>
__device__ __forceinline__ void row_max_sum(const T* x, int N, int lane, float& m, float& s) {
  m = -INFINITY;
  s = 0.f;
  for (int j = lane; j < N; j += 64) {
    float v = ld(x, j);
    float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    float a = (m == -INFINITY) ? 0.f : s * __expf(m - nm);
    float b = (om == -INFINITY) ? 0.f : os * __expf(om - nm);
    m = nm;
    s = a + b;
  }
}

template <typename T, bool LOG>
__global__ void __launch_bounds__(256) softmax_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                      int64_t R, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  T* yr = y + row * N;
  float m, s;
  row_max_sum(xr, N, lane, m, s);
  const float ls = __logf(s);
  const float inv = 1.f / s;
  for (int j = lane; j < N; j += 64) {
    float v = ld(xr, j) - m;
    yr[j] = from_f<T>(LOG ? v - ls : __expf(v) * inv);
  }
}

// dx = y * (dy - sum(dy*y))
template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_k(const T* __restrict__ y, const T* __restrict__ dy,
                                                      T* __restrict__ dx, int64_t R, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T *yr = y + row * N, *gr = dy + row * N;
  float d = 0.f;
  for (int j = lane; j < N; j += 64) d += ld(yr, j) * ld(gr, j);
  d = wave_sum(d);
  for (int j = lane; j < N; j += 64) dx[row * N + j] = from_f<T>(ld(yr, j) * (ld(gr, j) - d));
}

// loss[r] = sum_j y_j * (lse - x_j)   (dense / one-hot labels)
template <typename T, typename L>
__global__ void __launch_bounds__(256) sce_fwd_k(const T* __restrict__ x, const L* __restrict__ lab,
                                                  float* __restrict__ loss, float* __restrict__ lse_out,
                                                  int64_t R, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  const L* lr = lab + row * N;
  float m, s;
  row_max_sum(xr, N, lane, m, s);
  const float lse = m + __logf(s);
  float acc = 0.f;
  for (int j = lane; j < N; j += 64) {
    float yv = ld(lr, j);
    acc += yv * (lse - ld(xr, j));
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    loss[row] = acc;
    if (lse_out) lse_out[row] = lse;
  }
}

// dx = g[r] * (softmax(x) * sum(y) - y)
template <typename T, typename L>
__global__ void __launch_bounds__(256) sce_bwd_k(const T* __restrict__ x, const L* __restrict__ lab,
                                                  const float* __restrict__ g, int g_scalar,
                                                  const float* __restrict__ lse_in, T* __restrict__ dx,
                                                  int64_t R, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  const L* lr = lab + row * N;
  float lse;
  if (lse_in) {
    lse = lse_in[row];
  } else {
    float m, s;
    row_max_sum(xr, N, lane, m, s);
    lse = m + __logf(s);
  }
  float ys = 0.f;
  for (int j = lane; j < N; j += 64) ys += ld(lr, j);
  ys = wave_sum(ys);
  const float gr = g_scalar ? g[0] : g[row];
  for (int j = lane; j < N; j += 64)
    dx[row * N + j] = from_f<T>(gr * (__expf(ld(xr, j) - lse) * ys - ld(lr, j)));
}

// sparse labels (int64 class ids); ignored rows produce 0 loss and 0 grad
template <typename T>
__global__ void __launch_bounds__(256) sce_sparse_fwd_k(const T* __restrict__ x,
                                                         const int64_t* __restrict__ lab,
                                                         float* __restrict__ loss,
                                                         float* __restrict__ lse_out, int64_t R,
                                                         int N, int64_t ignored) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  float m, s;
  row_max_sum(xr, N, lane, m, s);
  const float lse = m + __logf(s);
  if (lane == 0) {
    const int64_t c = lab[row];
    loss[row] = (c == ignored || c < 0 || c >= N) ? 0.f : lse - ld(xr, c);
    if (lse_out) lse_out[row] = lse;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) sce_sparse_bwd_k(const T* __restrict__ x,
                                                         const int64_t* __restrict__ lab,
                                                         const float* __restrict__ g, int g_scalar,
                                                         const float* __restrict__ lse_in,
                                                         T* __restrict__ dx, int64_t R, int N,
                                                         int64_t ignored) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * N;
  const int64_t c = lab[row];
  const bool ign = (c == ignored || c < 0 || c >= N);
  float lse;
  if (lse_in) {
    lse = lse_in[row];
  } else {
    float m, s;
    row_max_sum(xr, N, lane, m, s);
    lse = m + __logf(s);
  }
  const float gr = ign ? 0.f : (g_scalar ? g[0] : g[row]);
  for (int j = lane; j < N; j += 64)
    dx[row * N + j] = from_f<T>(gr * (__expf(ld(xr, j) - lse) - (j == c ? 1.f : 0.f)));
}

}  // namespace hetu

using namespace hetu;

static inline dim3 rows_grid(int64_t R) { return dim3((unsigned)((R + 3) / 4)); }

HETU_API int hetu_softmax_fwd(const void* x, void* y, int64_t R, int N, int is_bf16, int log,
                              hipStream_t st) {
  if (is_bf16) {
    if (log) hipLaunchKernelGGL((softmax_fwd_k<bf16, true>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (bf16*)y, R, N);
    else hipLaunchKernelGGL((softmax_fwd_k<bf16, false>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (bf16*)y, R, N);
  } else {
    if (log) hipLaunchKernelGGL((softmax_fwd_k<float, true>), rows_grid(R), dim3(256), 0, st, (const float*)x, (float*)y, R, N);
    else hipLaunchKernelGGL((softmax_fwd_k<float, false>), rows_grid(R), dim3(256), 0, st, (const float*)x, (float*)y, R, N);
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_softmax_bwd(const void* y, const void* dy, void* dx, int64_t R, int N, int is_bf16,
                              hipStream_t st) {
  if (is_bf16) hipLaunchKernelGGL(softmax_bwd_k<bf16>, rows_grid(R), dim3(256), 0, st, (const bf16*)y, (const bf16*)dy, (bf16*)dx, R, N);
  else hipLaunchKernelGGL(softmax_bwd_k<float>, rows_grid(R), dim3(256), 0, st, (const float*)y, (const float*)dy, (float*)dx, R, N);
  HETU_LAUNCH_CHECK();
  return 0;
}

// dtype codes: 0 fp32, 1 bf16
HETU_API int hetu_softmax_ce_fwd(const void* x, const void* lab, float* loss, float* lse, int64_t R,
                                 int N, int x_bf16, int lab_bf16, hipStream_t st) {
  if (x_bf16 && lab_bf16) hipLaunchKernelGGL((sce_fwd_k<bf16, bf16>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (const bf16*)lab, loss, lse, R, N);
  else if (x_bf16) hipLaunchKernelGGL((sce_fwd_k<bf16, float>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (const float*)lab, loss, lse, R, N);
  else if (lab_bf16) hipLaunchKernelGGL((sce_fwd_k<float, bf16>), rows_grid(R), dim3(256), 0, st, (const float*)x, (const bf16*)lab, loss, lse, R, N);
  else hipLaunchKernelGGL((sce_fwd_k<float, float>), rows_grid(R), dim3(256), 0, st, (const float*)x, (const float*)lab, loss, lse, R, N);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_softmax_ce_bwd(const void* x, const void* lab, const float* g, int g_scalar,
                                 const float* lse, void* dx, int64_t R, int N, int x_bf16,
                                 int lab_bf16, hipStream_t st) {
  if (x_bf16 && lab_bf16) hipLaunchKernelGGL((sce_bwd_k<bf16, bf16>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (const bf16*)lab, g, g_scalar, lse, (bf16*)dx, R, N);
  else if (x_bf16) hipLaunchKernelGGL((sce_bwd_k<bf16, float>), rows_grid(R), dim3(256), 0, st, (const bf16*)x, (const float*)lab, g, g_scalar, lse, (bf16*)dx, R, N);
  else if (lab_bf16) hipLaunchKernelGGL((sce_bwd_k<float, bf16>), rows_grid(R), dim3(256), 0, st, (const float*)x, (const bf16*)lab, g, g_scalar, lse, (float*)dx, R, N);
  else hipLaunchKernelGGL((sce_bwd_k<float, float>), rows_grid(R), dim3(256), 0, st, (const float*)x, (const float*)lab, g, g_scalar, lse, (float*)dx, R, N);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_softmax_ce_sparse_fwd(const void* x, const int64_t* lab, float* loss, float* lse,
                                        int64_t R, int N, int x_bf16, int64_t ignored,
                                        hipStream_t st) {
  if (x_bf16) hipLaunchKernelGGL(sce_sparse_fwd_k<bf16>, rows_grid(R), dim3(256), 0, st, (const bf16*)x, lab, loss, lse, R, N, ignored);
  else hipLaunchKernelGGL(sce_sparse_fwd_k<float>, rows_grid(R), dim3(256), 0, st, (const float*)x, lab, loss, lse, R, N, ignored);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_softmax_ce_sparse_bwd(const void* x, const int64_t* lab, const float* g,
                                        int g_scalar, const float* lse, void* dx, int64_t R, int N,
                                        int x_bf16, int64_t ignored, hipStream_t st) {
  if (x_bf16) hipLaunchKernelGGL(sce_sparse_bwd_k<bf16>, rows_grid(R), dim3(256), 0, st, (const bf16*)x, lab, g, g_scalar, lse, (bf16*)dx, R, N, ignored);
  else hipLaunchKernelGGL(sce_sparse_bwd_k<float>, rows_grid(R), dim3(256), 0, st, (const float*)x, lab, g, g_scalar, lse, (float*)dx, R, N, ignored);
  HETU_LAUNCH_CHECK();
  return 0;
}
