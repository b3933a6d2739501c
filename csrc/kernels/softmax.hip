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

// Long rows (the MLM vocabulary, N ~ 30k) split into an unaligned scalar head,
// a 16-byte vector body (8 bf16 / 4 fp32 per lane: one max + one rescale per
// vector) and a scalar tail; the row start is only element-aligned in general.
template <typename T>
__device__ __forceinline__ int row_head(const T* x, int N) {
  const int h = (int)(((16 - ((uintptr_t)x & 15)) & 15) / sizeof(T));
  return h < N ? h : N;
}

template <typename T>
__device__ __forceinline__ void online_merge(float& m, float& s, float v) {
  const float nm = fmaxf(m, v);
  s = s * __expf(m - nm) + __expf(v - nm);
  m = nm;
}

template <typename T>
__device__ __forceinline__ void row_max_sum_vec(const T* x, int N, int lane, float& m, float& s) {
  constexpr int V = Vec<T>::N;
  m = -INFINITY;
  s = 0.f;
  const int h = row_head(x, N);
  if (lane < h) online_merge<T>(m, s, to_f(x[lane]));
  const int nv = (N - h) / V;
  const T* xb = x + h;
  int j = lane;
  for (; j + 64 < nv; j += 128) {          // two vectors in flight
    float v[V], w[V];
    load_vec<T>(xb + (int64_t)j * V, v);
    load_vec<T>(xb + (int64_t)(j + 64) * V, w);
    float vm = v[0];
#pragma unroll
    for (int k = 1; k < V; ++k) vm = fmaxf(vm, v[k]);
#pragma unroll
    for (int k = 0; k < V; ++k) vm = fmaxf(vm, w[k]);
    const float nm = fmaxf(m, vm);
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) t += __expf(v[k] - nm) + __expf(w[k] - nm);
    s = s * __expf(m - nm) + t;
    m = nm;
  }
  for (; j < nv; j += 64) {
    float v[V];
    load_vec<T>(xb + (int64_t)j * V, v);
    float vm = v[0];
#pragma unroll
    for (int k = 1; k < V; ++k) vm = fmaxf(vm, v[k]);
    const float nm = fmaxf(m, vm);
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) t += __expf(v[k] - nm);
    s = s * __expf(m - nm) + t;
    m = nm;
  }
  for (int t = h + nv * V + lane; t < N; t += 64) online_merge<T>(m, s, to_f(x[t]));
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
  const int64_t c = lab[row];
  if (c == ignored || c < 0 || c >= N) {
    // an ignored row's loss is 0 and its gradient 0 whatever its logits are (the BERT MLM
    // head ignores ~85 % of its rows): the row is not read; its lse is not computed (0)
    if (lane == 0) {
      loss[row] = 0.f;
      if (lse_out) lse_out[row] = 0.f;
    }
    return;
  }
  float m, s;
  row_max_sum_vec(xr, N, lane, m, s);
  const float lse = m + __logf(s);
  if (lane == 0) {
    loss[row] = lse - ld(xr, c);
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
  T* dr = dx + row * N;
  // (an ignored row is written as g = 0 times the softmax below, not by a zero-fill path
  // that skips the logits: the write-only rows measured slower, 216 vs 188 us per BERT step)
  float lse;
  if (ign) {
    // the forward does not compute an ignored row's lse: +inf makes every exp(x - lse) 0,
    // so the row is exactly 0 * (0 - 0) (a finite stand-in could overflow exp into 0 * inf)
    lse = __builtin_inff();
  } else if (lse_in) {
    lse = lse_in[row];
  } else {
    float m, s;
    row_max_sum_vec(xr, N, lane, m, s);
    lse = m + __logf(s);
  }
  const float gr = ign ? 0.f : (g_scalar ? g[0] : g[row]);
  constexpr int V = Vec<T>::N;
  // x and dx share the row pitch; vector body only when their rows align alike
  const int h = row_head(xr, N);
  const bool vec = ((uintptr_t)xr & 15) == ((uintptr_t)dr & 15);
  if (!vec) {
    for (int j = lane; j < N; j += 64)
      dr[j] = from_f<T>(gr * (__expf(ld(xr, j) - lse) - (j == c ? 1.f : 0.f)));
    return;
  }
  if (lane < h) dr[lane] = from_f<T>(gr * (__expf(ld(xr, lane) - lse) - (lane == c ? 1.f : 0.f)));
  const int nv = (N - h) / V;
  for (int j = lane; j < nv; j += 64) {
    const int64_t e0 = h + (int64_t)j * V;
    float v[V];
    load_vec<T>(xr + e0, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = gr * (__expf(v[k] - lse) - (e0 + k == c ? 1.f : 0.f));
    store_vec<T>(dr + e0, v);
  }
  for (int t = h + nv * V + lane; t < N; t += 64)
    dr[t] = from_f<T>(gr * (__expf(ld(xr, t) - lse) - (t == c ? 1.f : 0.f)));
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
