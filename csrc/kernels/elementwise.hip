// Vectorised elementwise kernel family (unary / binary / broadcast / scalar).
//
// Replaces ~25 one-kernel files of the reference (Relu.cu, Gelu.cu, Sigmoid.cu,
// Tanh.cu, Exp.cu, Log.cu, Sqrt.cu, AddElewise.cu, MultiplyElewise.cu, ...),
// all of which use the "E1" 1-thread-per-element, 1024-thread launch, with one
// templated family: 16-byte vector loads, grid-stride over at most 2048 blocks,
// fp32 math on bf16/fp32 storage.
#include "common.h"
#include <algorithm>

namespace hetu {

enum UnaryOp {
  U_RELU = 0, U_SIGMOID, U_TANH, U_EXP, U_LOG, U_SQRT, U_RSQRT, U_ABS, U_NEG, U_GELU,
  U_LEAKY_RELU, U_FLOOR, U_SIN, U_COS, U_ADD_C, U_MUL_C, U_RSUB_C /* c - x */, U_RDIV_C /* c / x */,
  U_POW_C /* x^c */, U_CPOW /* c^x */, U_CLAMP, U_SIGN, U_BOOL_GT /* x > c */, U_RECIP, U_SQUARE,
  U_GELU_TANH
};

enum BinaryOp {
  B_ADD = 0, B_SUB, B_MUL, B_DIV, B_MAX, B_MIN,
  B_RELU_GRAD /* a=x b=g */, B_GELU_GRAD, B_TANH_GRAD /* a=y */, B_SIGMOID_GRAD /* a=y */,
  B_LEAKY_RELU_GRAD, B_ABS_GRAD, B_POW /* a^b */, B_ADD_RELU, B_LOG_GRAD /* a=x b=g: g/x */,
  B_SQRT_GRAD /* a=y b=g: g/(2y) */, B_GELU_TANH_GRAD,
  B_RELU_GRAD_C /* a=y b=g: y > 0 ? c g : 0 (ReLU + dropout backward from the output) */
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.70710678118f));
  float pdf = 0.3989422804f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k = 0.7978845608f;
  return 0.5f * x * (1.f + tanhf(k * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k = 0.7978845608f;
  float u = k * (x + 0.044715f * x * x * x);
  float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
}

template <int OP>
__device__ __forceinline__ float un(float x, float c, float c2) {
  switch (OP) {
    case U_RELU: return fmaxf(x, 0.f);
    case U_SIGMOID: return 1.f / (1.f + __expf(-x));
    case U_TANH: return tanhf(x);
    case U_EXP: return __expf(x);
    case U_LOG: return __logf(x);
    case U_SQRT: return sqrtf(x);
    case U_RSQRT: return rsqrtf(x);
    case U_ABS: return fabsf(x);
    case U_NEG: return -x;
    case U_GELU: return gelu_erf(x);
    case U_LEAKY_RELU: return x > 0.f ? x : c * x;
    case U_FLOOR: return floorf(x);
    case U_SIN: return __sinf(x);
    case U_COS: return __cosf(x);
    case U_ADD_C: return x + c;
    case U_MUL_C: return x * c;
    case U_RSUB_C: return c - x;
    case U_RDIV_C: return c / x;
    case U_POW_C: return powf(x, c);
    case U_CPOW: return powf(c, x);
    case U_CLAMP: return fminf(fmaxf(x, c), c2);
    case U_SIGN: return (float)((x > 0.f) - (x < 0.f));
    case U_BOOL_GT: return x > c ? 1.f : 0.f;
    case U_RECIP: return 1.f / x;
    case U_SQUARE: return x * x;
    case U_GELU_TANH: return gelu_tanh(x);
  }
  return x;
}

template <int OP>
__device__ __forceinline__ float bi(float a, float b, float c) {
  switch (OP) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_MAX: return fmaxf(a, b);
    case B_MIN: return fminf(a, b);
    case B_RELU_GRAD: return a > 0.f ? b : 0.f;
    case B_GELU_GRAD: return b * gelu_erf_grad(a);
    case B_TANH_GRAD: return b * (1.f - a * a);
    case B_SIGMOID_GRAD: return b * a * (1.f - a);
    case B_LEAKY_RELU_GRAD: return a > 0.f ? b : c * b;
    case B_ABS_GRAD: return a > 0.f ? b : (a < 0.f ? -b : 0.f);
    case B_POW: return powf(a, b);
    case B_ADD_RELU: return fmaxf(a + b, 0.f);
    case B_LOG_GRAD: return b / a;
    case B_SQRT_GRAD: return b * 0.5f / a;
    case B_GELU_TANH_GRAD: return b * gelu_tanh_grad(a);
    case B_RELU_GRAD_C: return a > 0.f ? b * c : 0.f;
  }
  return a;
}

template <typename T, int OP>
__global__ void __launch_bounds__(256) unary_k(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                float c, float c2) {
  constexpr int V = Vec<T>::N;
  // 16-byte vectors only on 16-byte aligned bases (offset views go scalar)
  const int64_t nv = (((uintptr_t)x | (uintptr_t)y) % 16 == 0) ? n / V : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float v[V];
    load_vec<T>(x + i * V, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = un<OP>(v[k], c, c2);
    store_vec<T>(y + i * V, v);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = from_f<T>(un<OP>(to_f(x[i]), c, c2));
}

// b_mode: 0 same shape; 1 b broadcast along rows (b has `inner` elements,
// a is [n/inner, inner]); 2 b is a scalar tensor; 3 b constant along the trailing
// `inner` elements and periodic with `bnum` values ([T,1] x [T,d] row scales, [1,C,1,1]
// per-channel NCHW operands): b[(i / inner) % bnum]
template <typename TB>
__device__ __forceinline__ float b_at(const TB* __restrict__ b, int b_mode, int64_t i, int64_t inner, int64_t bnum) {
  if (b_mode == 0) return to_f(b[i]);
  if (b_mode == 1) return to_f(b[i % inner]);
  if (b_mode == 2) return to_f(b[0]);
  return to_f(b[(i / inner) % bnum]);
}

template <typename T, typename TB, int OP>
__global__ void __launch_bounds__(256) binary_k(const T* __restrict__ a, const TB* __restrict__ b,
                                                 T* __restrict__ y, int64_t n, int b_mode,
                                                 int64_t inner, int64_t bnum, float c) {
  constexpr int V = Vec<T>::N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // 16-byte vector path only on 16-byte aligned bases (views with an element offset
  // take the scalar path)
  const uintptr_t al = (uintptr_t)a | (uintptr_t)y | (b_mode == 0 ? (uintptr_t)b : (uintptr_t)0);
  const bool vec_ok = (al % 16 == 0) &&
                      ((b_mode == 0 && sizeof(T) == sizeof(TB)) || (b_mode == 1 && inner % V == 0) ||
                       b_mode == 2 || (b_mode == 3 && inner % V == 0));
  if (vec_ok) {
    const int64_t nv = n / V;
    const float bs = b_mode == 2 ? to_f(b[0]) : 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
      float va[V], vb[V];
      load_vec<T>(a + i * V, va);
      if (b_mode == 0) {
        load_vec<T>((const T*)b + i * V, vb);
      } else if (b_mode == 1) {
        const int64_t c0 = (i * V) % inner;
#pragma unroll
        for (int k = 0; k < V; ++k) vb[k] = to_f(b[c0 + k]);
      } else if (b_mode == 3) {   // the whole vector lies in one inner block
        const float bv = to_f(b[((i * V) / inner) % bnum]);
#pragma unroll
        for (int k = 0; k < V; ++k) vb[k] = bv;
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) vb[k] = bs;
      }
#pragma unroll
      for (int k = 0; k < V; ++k) va[k] = bi<OP>(va[k], vb[k], c);
      store_vec<T>(y + i * V, va);
    }
    for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
      y[i] = from_f<T>(bi<OP>(to_f(a[i]), b_at(b, b_mode, i, inner, bnum), c));
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
      y[i] = from_f<T>(bi<OP>(to_f(a[i]), b_at(b, b_mode, i, inner, bnum), c));
  }
}

// General broadcast / strided binary op (the long tail the fast path above does not
// take: middle-dim broadcasts, non-contiguous views): the output is contiguous in
// `shape` (up to 8 dims); a and b are read through element strides (0 on broadcast dims).
struct NdGeom {
  int nd;
  int64_t shape[8], as[8], bs[8];
};

// IT: index type -- 32-bit when every offset fits (the host collapses mergeable dims
// first, so most calls carry 2-3 dims of 32-bit divisions per element)
template <typename T, typename TB, int OP, typename IT>
__global__ void __launch_bounds__(256) binary_nd_k(const T* __restrict__ a, const TB* __restrict__ b,
                                                    T* __restrict__ y, int64_t n, NdGeom g, float c) {
  IT shape[8], as[8], bs[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) { shape[d] = (IT)g.shape[d]; as[d] = (IT)g.as[d]; bs[d] = (IT)g.bs[d]; }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    IT r = (IT)i, oa = 0, ob = 0;
#pragma unroll
    for (int d = 7; d >= 0; --d) {
      if (d < g.nd) {
        const IT q = r / shape[d], k = r - q * shape[d];
        oa += k * as[d];
        ob += k * bs[d];
        r = q;
      }
    }
    y[i] = from_f<T>(bi<OP>(to_f(a[oa]), to_f(b[ob]), c));
  }
}

template <typename TI, typename TO>
__global__ void cast_k(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = from_f<TO>(to_f(x[i]));
}

}  // namespace hetu

using namespace hetu;

#define UCASE(OPV)                                                                             \
  case OPV:                                                                                    \
    if (is_bf16)                                                                               \
      hipLaunchKernelGGL((unary_k<bf16, OPV>), dim3(grid), dim3(256), 0, st, (const bf16*)x,   \
                         (bf16*)y, n, c, c2);                                                  \
    else                                                                                       \
      hipLaunchKernelGGL((unary_k<float, OPV>), dim3(grid), dim3(256), 0, st, (const float*)x, \
                         (float*)y, n, c, c2);                                                 \
    break;

HETU_API int hetu_unary(int op, const void* x, void* y, int64_t n, int is_bf16, float c, float c2,
                        hipStream_t st) {
  if (n <= 0) return 0;
  int grid = stream_grid(n, 256, is_bf16 ? 8 : 4);
  switch (op) {
    UCASE(U_RELU) UCASE(U_SIGMOID) UCASE(U_TANH) UCASE(U_EXP) UCASE(U_LOG) UCASE(U_SQRT)
    UCASE(U_RSQRT) UCASE(U_ABS) UCASE(U_NEG) UCASE(U_GELU) UCASE(U_LEAKY_RELU) UCASE(U_FLOOR)
    UCASE(U_SIN) UCASE(U_COS) UCASE(U_ADD_C) UCASE(U_MUL_C) UCASE(U_RSUB_C) UCASE(U_RDIV_C)
    UCASE(U_POW_C) UCASE(U_CPOW) UCASE(U_CLAMP) UCASE(U_SIGN) UCASE(U_BOOL_GT) UCASE(U_RECIP)
    UCASE(U_SQUARE) UCASE(U_GELU_TANH)
    default: return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

#define BCASE(OPV)                                                                              \
  case OPV:                                                                                     \
    if (is_bf16 && b_bf16)                                                                      \
      hipLaunchKernelGGL((binary_k<bf16, bf16, OPV>), dim3(grid), dim3(256), 0, st,             \
                         (const bf16*)a, (const bf16*)b, (bf16*)y, n, b_mode, inner, bnum, c);        \
    else if (is_bf16)                                                                           \
      hipLaunchKernelGGL((binary_k<bf16, float, OPV>), dim3(grid), dim3(256), 0, st,            \
                         (const bf16*)a, (const float*)b, (bf16*)y, n, b_mode, inner, bnum, c);       \
    else if (b_bf16)                                                                            \
      hipLaunchKernelGGL((binary_k<float, bf16, OPV>), dim3(grid), dim3(256), 0, st,            \
                         (const float*)a, (const bf16*)b, (float*)y, n, b_mode, inner, bnum, c);      \
    else                                                                                        \
      hipLaunchKernelGGL((binary_k<float, float, OPV>), dim3(grid), dim3(256), 0, st,           \
                         (const float*)a, (const float*)b, (float*)y, n, b_mode, inner, bnum, c);     \
    break;

HETU_API int hetu_binary3(int op, const void* a, const void* b, void* y, int64_t n, int is_bf16,
                          int b_bf16, int b_mode, int64_t inner, int64_t bnum, float c, hipStream_t st) {
  if (n <= 0) return 0;
  if (bnum < 1) bnum = 1;
  int grid = stream_grid(n, 256, is_bf16 ? 8 : 4);
  switch (op) {
    BCASE(B_ADD) BCASE(B_SUB) BCASE(B_MUL) BCASE(B_DIV) BCASE(B_MAX) BCASE(B_MIN)
    BCASE(B_RELU_GRAD) BCASE(B_GELU_GRAD) BCASE(B_TANH_GRAD) BCASE(B_SIGMOID_GRAD)
    BCASE(B_LEAKY_RELU_GRAD) BCASE(B_ABS_GRAD) BCASE(B_POW) BCASE(B_ADD_RELU) BCASE(B_LOG_GRAD)
    BCASE(B_SQRT_GRAD) BCASE(B_GELU_TANH_GRAD) BCASE(B_RELU_GRAD_C)
    default: return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_binary(int op, const void* a, const void* b, void* y, int64_t n, int is_bf16,
                         int b_bf16, int b_mode, int64_t inner, float c, hipStream_t st) {
  return hetu_binary3(op, a, b, y, n, is_bf16, b_bf16, b_mode, inner, 1, c, st);
}

#define BND_LAUNCH(OPV, IT)                                                                     \
    if (is_bf16 && b_bf16)                                                                      \
      hipLaunchKernelGGL((binary_nd_k<bf16, bf16, OPV, IT>), dim3(grid), dim3(256), 0, st,      \
                         (const bf16*)a, (const bf16*)b, (bf16*)y, n, g, c);                    \
    else if (is_bf16)                                                                           \
      hipLaunchKernelGGL((binary_nd_k<bf16, float, OPV, IT>), dim3(grid), dim3(256), 0, st,     \
                         (const bf16*)a, (const float*)b, (bf16*)y, n, g, c);                   \
    else if (b_bf16)                                                                            \
      hipLaunchKernelGGL((binary_nd_k<float, bf16, OPV, IT>), dim3(grid), dim3(256), 0, st,     \
                         (const float*)a, (const bf16*)b, (float*)y, n, g, c);                  \
    else                                                                                        \
      hipLaunchKernelGGL((binary_nd_k<float, float, OPV, IT>), dim3(grid), dim3(256), 0, st,    \
                         (const float*)a, (const float*)b, (float*)y, n, g, c);
#define BNDCASE(OPV)                                                                            \
  case OPV:                                                                                     \
    if (small) { BND_LAUNCH(OPV, int32_t) } else { BND_LAUNCH(OPV, int64_t) }                   \
    break;

// y (contiguous, shape[0..nd)) = op(a, b) with a / b read through element strides
HETU_API int hetu_binary_nd(int op, const void* a, const void* b, void* y, int nd, const int64_t* shape,
                            const int64_t* astride, const int64_t* bstride, int is_bf16, int b_bf16, float c,
                            hipStream_t st) {
  if (nd < 1 || nd > 8) return (int)hipErrorInvalidValue;
  NdGeom g;
  g.nd = nd;
  int64_t n = 1;
  for (int d = 0; d < 8; ++d) {
    g.shape[d] = d < nd ? shape[d] : 1;
    g.as[d] = d < nd ? astride[d] : 0;
    g.bs[d] = d < nd ? bstride[d] : 0;
    if (d < nd) n *= shape[d];
  }
  if (n <= 0) return 0;
  int64_t ea = 0, eb = 0;   // largest element offset each operand is read at
  for (int d = 0; d < nd; ++d) {
    ea += (shape[d] - 1) * astride[d];
    eb += (shape[d] - 1) * bstride[d];
  }
  const int64_t reach = std::max(n, std::max(ea, eb) + 1);
  const bool small = reach < (1ll << 31);
  int grid = stream_grid(n, 256, 1);
  switch (op) {
    BNDCASE(B_ADD) BNDCASE(B_SUB) BNDCASE(B_MUL) BNDCASE(B_DIV) BNDCASE(B_MAX) BNDCASE(B_MIN)
    BNDCASE(B_RELU_GRAD) BNDCASE(B_GELU_GRAD) BNDCASE(B_TANH_GRAD) BNDCASE(B_SIGMOID_GRAD)
    BNDCASE(B_LEAKY_RELU_GRAD) BNDCASE(B_ABS_GRAD) BNDCASE(B_POW) BNDCASE(B_ADD_RELU) BNDCASE(B_LOG_GRAD)
    BNDCASE(B_SQRT_GRAD) BNDCASE(B_GELU_TANH_GRAD) BNDCASE(B_RELU_GRAD_C)
    default: return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

// dtype codes 0 fp32 1 bf16
HETU_API int hetu_cast(const void* x, int xt, void* y, int yt, int64_t n, hipStream_t st) {
  int grid = stream_grid(n, 256, 1);
  if (xt == 0 && yt == 1) hipLaunchKernelGGL((cast_k<float, bf16>), dim3(grid), dim3(256), 0, st, (const float*)x, (bf16*)y, n);
  else if (xt == 1 && yt == 0) hipLaunchKernelGGL((cast_k<bf16, float>), dim3(grid), dim3(256), 0, st, (const bf16*)x, (float*)y, n);
  else return (int)hipErrorInvalidValue;
  HETU_LAUNCH_CHECK();
  return 0;
}

static thread_local char g_err[256];
HETU_API const char* HetuGetLastError() {
  hipError_t e = hipGetLastError();
  snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e));
  return g_err;
}
