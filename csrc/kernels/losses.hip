// Loss kernels of the reference op library that are not the fused softmax-CE
// (softmax.hip): probability cross-entropy (dense and sparse labels, with an
// ignored index), binary cross-entropy and the NLL loss, forward and backward.
// Reference: src/ops/CrossEntropy.cu (cuDNN ReduceTensor for the row sum),
// CrossEntropySparse.cu, BinaryCrossEntropy.cu, NllLoss.cu (atomicAdd into one scalar).
// Rows are reduced by one wave each (wave64 shuffles); the NLL mean by a block sum
// per workgroup and one fp32 atomic per workgroup.
#include "common.h"

using namespace hetu;

namespace {

// out[r] = -sum_c lab[r,c] * log(y[r,c])
template <typename T>
__global__ void __launch_bounds__(256) ce_dense_k(const T* __restrict__ y, const T* __restrict__ lab,
                                                  float* __restrict__ out, int64_t rows, int64_t cols) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float s = 0.f;
  for (int64_t c = lane; c < cols; c += 64) {
    const float l = to_f(lab[r * cols + c]);
    if (l != 0.f) s -= l * logf(to_f(y[r * cols + c]));
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}

// dy = -g[r] * lab / y   (g broadcast: scalar when g_scalar)
template <typename T>
__global__ void __launch_bounds__(256) ce_dense_grad_k(const float* __restrict__ g, const T* __restrict__ y,
                                                       const T* __restrict__ lab, T* __restrict__ dy, int64_t rows,
                                                       int64_t cols, int g_scalar) {
  const int64_t total = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float gg = g[g_scalar ? 0 : i / cols];
    dy[i] = from_f<T>(-gg * to_f(lab[i]) / to_f(y[i]));
  }
}

// out[r] = lab[r] == ignore ? 0 : -log(y[r, lab[r]])
template <typename T>
__global__ void __launch_bounds__(256) ce_sparse_k(const T* __restrict__ y, const int64_t* __restrict__ lab,
                                                   float* __restrict__ out, int64_t rows, int64_t cols,
                                                   int64_t ignore) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = lab[r];
    out[r] = (l == ignore || l < 0 || l >= cols) ? 0.f : -logf(to_f(y[r * cols + l]));
  }
}

// dy[r, c] = c == lab[r] ? -g[r] / y[r, c] : 0
template <typename T>
__global__ void __launch_bounds__(256) ce_sparse_grad_k(const float* __restrict__ g, const T* __restrict__ y,
                                                        const int64_t* __restrict__ lab, T* __restrict__ dy,
                                                        int64_t rows, int64_t cols, int64_t ignore, int g_scalar) {
  const int64_t total = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols, c = i - r * cols, l = lab[r];
    float v = 0.f;
    if (c == l && l != ignore) v = -g[g_scalar ? 0 : r] / to_f(y[i]);
    dy[i] = from_f<T>(v);
  }
}

__device__ __forceinline__ float clampp(float y) { return fminf(fmaxf(y, 1e-12f), 1.f - 1e-7f); }

// elementwise: out = -l log(y) - (1 - l) log(1 - y)
template <typename T>
__global__ void __launch_bounds__(256) bce_k(const T* __restrict__ y, const T* __restrict__ lab,
                                             float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float p = clampp(to_f(y[i])), l = to_f(lab[i]);
    out[i] = -l * logf(p) - (1.f - l) * logf(1.f - p);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bce_grad_k(const T* __restrict__ y, const T* __restrict__ lab,
                                                  const float* __restrict__ g, T* __restrict__ dy, int64_t n,
                                                  int g_scalar) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float p = clampp(to_f(y[i])), l = to_f(lab[i]);
    dy[i] = from_f<T>(g[g_scalar ? 0 : i] * (-l / p + (1.f - l) / (1.f - p)));
  }
}

// class index of a label held as int64, int32 or a float (the data loaders' label tensors
// reach the loss in whatever dtype they were fed: no conversion kernel in front of it)
template <typename L>
__device__ __forceinline__ int64_t lab_idx(const L* t, int64_t r) { return (int64_t)t[r]; }

// out[0] += -sum_r x[r, t[r]] / rows  (out zeroed by the caller)
template <typename T, typename L>
__global__ void __launch_bounds__(256) nll_k(const T* __restrict__ x, const L* __restrict__ t,
                                             float* __restrict__ out, int64_t rows, int64_t cols) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = lab_idx(t, r);
    if (c >= 0 && c < cols) s += to_f(x[r * cols + c]);
  }
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) unsafeAtomicAdd(out, -s / (float)rows);
}

// dx[r, c] = c == t[r] ? -g / rows : 0
template <typename L>
__global__ void __launch_bounds__(256) nll_grad_k(const float* __restrict__ g, const L* __restrict__ t,
                                                  float* __restrict__ dx, int64_t rows, int64_t cols) {
  const int64_t total = rows * cols;
  const float v = -g[0] / (float)rows;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols;
    dx[i] = (i - r * cols) == lab_idx(t, r) ? v : 0.f;
  }
}

}  // namespace


HETU_API int hetu_ce_dense(const void* y, const void* lab, float* out, int64_t rows, int64_t cols, int bf,
                           hipStream_t st) {
  if (rows == 0) return 0;
  const dim3 g((unsigned)((rows + 3) / 4));
  if (bf) hipLaunchKernelGGL(ce_dense_k<bf16>, g, dim3(256), 0, st, (const bf16*)y, (const bf16*)lab, out, rows, cols);
  else hipLaunchKernelGGL(ce_dense_k<float>, g, dim3(256), 0, st, (const float*)y, (const float*)lab, out, rows, cols);
  return (int)hipGetLastError();
}

HETU_API int hetu_ce_dense_grad(const float* g, const void* y, const void* lab, void* dy, int64_t rows, int64_t cols,
                                int g_scalar, int bf, hipStream_t st) {
  if (rows * cols == 0) return 0;
  const dim3 gr(stream_grid(rows * cols, 256, 2));
  if (bf) hipLaunchKernelGGL(ce_dense_grad_k<bf16>, gr, dim3(256), 0, st, g, (const bf16*)y, (const bf16*)lab, (bf16*)dy, rows, cols, g_scalar);
  else hipLaunchKernelGGL(ce_dense_grad_k<float>, gr, dim3(256), 0, st, g, (const float*)y, (const float*)lab, (float*)dy, rows, cols, g_scalar);
  return (int)hipGetLastError();
}

HETU_API int hetu_ce_sparse(const void* y, const int64_t* lab, float* out, int64_t rows, int64_t cols, int64_t ignore,
                            int bf, hipStream_t st) {
  if (rows == 0) return 0;
  const dim3 g(stream_grid(rows, 256));
  if (bf) hipLaunchKernelGGL(ce_sparse_k<bf16>, g, dim3(256), 0, st, (const bf16*)y, lab, out, rows, cols, ignore);
  else hipLaunchKernelGGL(ce_sparse_k<float>, g, dim3(256), 0, st, (const float*)y, lab, out, rows, cols, ignore);
  return (int)hipGetLastError();
}

HETU_API int hetu_ce_sparse_grad(const float* g, const void* y, const int64_t* lab, void* dy, int64_t rows,
                                 int64_t cols, int64_t ignore, int g_scalar, int bf, hipStream_t st) {
  if (rows * cols == 0) return 0;
  const dim3 gr(stream_grid(rows * cols, 256, 2));
  if (bf) hipLaunchKernelGGL(ce_sparse_grad_k<bf16>, gr, dim3(256), 0, st, g, (const bf16*)y, lab, (bf16*)dy, rows, cols, ignore, g_scalar);
  else hipLaunchKernelGGL(ce_sparse_grad_k<float>, gr, dim3(256), 0, st, g, (const float*)y, lab, (float*)dy, rows, cols, ignore, g_scalar);
  return (int)hipGetLastError();
}

HETU_API int hetu_bce(const void* y, const void* lab, float* out, int64_t n, int bf, hipStream_t st) {
  if (n == 0) return 0;
  const dim3 g(stream_grid(n, 256, 2));
  if (bf) hipLaunchKernelGGL(bce_k<bf16>, g, dim3(256), 0, st, (const bf16*)y, (const bf16*)lab, out, n);
  else hipLaunchKernelGGL(bce_k<float>, g, dim3(256), 0, st, (const float*)y, (const float*)lab, out, n);
  return (int)hipGetLastError();
}

HETU_API int hetu_bce_grad(const void* y, const void* lab, const float* g, void* dy, int64_t n, int g_scalar, int bf,
                           hipStream_t st) {
  if (n == 0) return 0;
  const dim3 gr(stream_grid(n, 256, 2));
  if (bf) hipLaunchKernelGGL(bce_grad_k<bf16>, gr, dim3(256), 0, st, (const bf16*)y, (const bf16*)lab, g, (bf16*)dy, n, g_scalar);
  else hipLaunchKernelGGL(bce_grad_k<float>, gr, dim3(256), 0, st, (const float*)y, (const float*)lab, g, (float*)dy, n, g_scalar);
  return (int)hipGetLastError();
}

// out: one fp32, zeroed by the caller; tkind: label dtype 0 = int64, 1 = int32, 2 = fp32
template <typename T, typename L>
static void nll_launch(const void* x, const void* t, float* out, int64_t rows, int64_t cols, int nb, hipStream_t st) {
  hipLaunchKernelGGL((nll_k<T, L>), dim3(nb), dim3(256), 0, st, (const T*)x, (const L*)t, out, rows, cols);
}

HETU_API int hetu_nll(const void* x, const void* t, int tkind, float* out, int64_t rows, int64_t cols, int bf,
                      hipStream_t st) {
  if (rows == 0) return 0;
  if (tkind < 0 || tkind > 2) return (int)hipErrorInvalidValue;
  int nb = (int)((rows + 255) / 256);
  if (nb > 256) nb = 256;
  if (bf) {
    if (tkind == 0) nll_launch<bf16, int64_t>(x, t, out, rows, cols, nb, st);
    else if (tkind == 1) nll_launch<bf16, int32_t>(x, t, out, rows, cols, nb, st);
    else nll_launch<bf16, float>(x, t, out, rows, cols, nb, st);
  } else {
    if (tkind == 0) nll_launch<float, int64_t>(x, t, out, rows, cols, nb, st);
    else if (tkind == 1) nll_launch<float, int32_t>(x, t, out, rows, cols, nb, st);
    else nll_launch<float, float>(x, t, out, rows, cols, nb, st);
  }
  return (int)hipGetLastError();
}

HETU_API int hetu_nll_grad(const float* g, const void* t, int tkind, float* dx, int64_t rows, int64_t cols,
                           hipStream_t st) {
  if (rows * cols == 0) return 0;
  if (tkind < 0 || tkind > 2) return (int)hipErrorInvalidValue;
  const dim3 gr(stream_grid(rows * cols, 256, 2));
  if (tkind == 0) hipLaunchKernelGGL(nll_grad_k<int64_t>, gr, dim3(256), 0, st, g, (const int64_t*)t, dx, rows, cols);
  else if (tkind == 1) hipLaunchKernelGGL(nll_grad_k<int32_t>, gr, dim3(256), 0, st, g, (const int32_t*)t, dx, rows, cols);
  else hipLaunchKernelGGL(nll_grad_k<float>, gr, dim3(256), 0, st, g, (const float*)t, dx, rows, cols);
  return (int)hipGetLastError();
}
