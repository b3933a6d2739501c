// Layout / indexing / scan / sort / per-row reduction kernels for gfx950: the long
// tail of the reference's op library.
//
//   nd_copy       strided N-D copy with per-dim roll / modulo: concat and split
//                 (copy into / out of a strided view), pad and its gradient, roll,
//                 repeat, slice -- reference Concat.cu, Concatenate.cu, Pad.cu,
//                 Roll.cu, Repeat.cu, Slice.cu (those pass shape metadata through a
//                 per-call cudaMalloc + H2D copy; here it is a by-value kernel arg)
//   gather_dim /  torch.gather along a dim and its scatter-add gradient
//   scatter_add_dim (reference Gather.cu; fp32 atomics on the memory side)
//   scan_dim      inclusive prefix sum + bias along a dim (reference CumSum.cu, which
//                 runs one serial thread per line): wave64 scan for contiguous rows
//   argmax_dim    wave64 arg-reduce (reference Argmax.cu, warp-32 block reduce)
//   argsort_rows  bitonic sort of (key, index) pairs in LDS, one workgroup per row
//                 (reference Argsort.cu: CUB DeviceSegmentedRadixSort)
//   pnorm_dim     p-norm along a dim and its gradient (reference Norm.cu)
//
// Every tensor is viewed as [outer, n, inner] around the reduced / indexed dim.
#include "common.h"

using namespace hetu;

namespace {

constexpr int MAXD = 8;

struct NDDesc {
  int nd;
  int64_t shape[MAXD];    // iteration shape (the OUTPUT view)
  int64_t ostride[MAXD];  // output element strides
  int64_t istride[MAXD];  // input element strides
  int64_t shift[MAXD];    // input coordinate = (c + shift) % imod  (imod > 0), else c + shift
  int64_t imod[MAXD];
};

// IT: 32-bit index math when every offset fits (the host collapses mergeable dims and
// widens the element to 16 bytes where the innermost dim is contiguous on both sides)
template <typename T, typename IT>
__global__ void __launch_bounds__(256) nd_copy_k(const T* __restrict__ x, T* __restrict__ y, NDDesc d,
                                                 int64_t total) {
  IT shape[MAXD], os[MAXD], is[MAXD], sh[MAXD], md[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    shape[k] = (IT)d.shape[k]; os[k] = (IT)d.ostride[k]; is[k] = (IT)d.istride[k];
    sh[k] = (IT)d.shift[k]; md[k] = (IT)d.imod[k];
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    IT r = (IT)i, oo = 0, io = 0;
#pragma unroll
    for (int k = MAXD - 1; k >= 0; --k) {
      if (k >= d.nd) continue;
      const IT q = r / shape[k], c = r - q * shape[k];
      r = q;
      oo += c * os[k];
      IT ci = c + sh[k];
      if (md[k] > 0) ci %= md[k];
      io += ci * is[k];
    }
    y[oo] = x[io];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) fill_k(T* __restrict__ y, T v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = v;
}

template <typename T>
__global__ void __launch_bounds__(256) gather_dim_k(const T* __restrict__ x, const int64_t* __restrict__ idx,
                                                    T* __restrict__ y, int64_t outer, int64_t nidx, int64_t nsrc,
                                                    int64_t inner) {
  const int64_t total = outer * nidx * inner;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t in = i % inner, t = i / inner, o = t / nidx;
    int64_t k = idx[i];
    if (k < 0) k += nsrc;
    y[i] = (k >= 0 && k < nsrc) ? x[(o * nsrc + k) * inner + in] : T(0.f);
  }
}

// dx[o, idx[o, j, i], i] += g[o, j, i]  (dx fp32, zeroed by the caller)
template <typename T>
__global__ void __launch_bounds__(256) scatter_add_dim_k(const T* __restrict__ g, const int64_t* __restrict__ idx,
                                                         float* __restrict__ dx, int64_t outer, int64_t nidx,
                                                         int64_t nsrc, int64_t inner) {
  const int64_t total = outer * nidx * inner;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t in = i % inner, t = i / inner, o = t / nidx;
    int64_t k = idx[i];
    if (k < 0) k += nsrc;
    if (k >= 0 && k < nsrc) unsafeAtomicAdd(dx + (o * nsrc + k) * inner + in, to_f(g[i]));
  }
}

// inclusive scan of contiguous rows (inner == 1): one wave per row, 64 elements per
// step, wave prefix by shuffles, running carry
template <typename T>
__global__ void __launch_bounds__(256) scan_rows_k(const T* __restrict__ x, float* __restrict__ y, int64_t rows,
                                                   int64_t n, float bias) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * n;
  float* yr = y + row * n;
  float carry = 0.f;
  for (int64_t b = 0; b < n; b += 64) {
    const int64_t j = b + lane;
    float v = j < n ? to_f(xr[j]) : 0.f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (j < n) yr[j] = v + carry + bias;
    carry += __shfl(v, 63, 64);
  }
}

// inclusive scan along n for inner > 1: one thread per (outer, inner) line, coalesced
// across inner
template <typename T>
__global__ void __launch_bounds__(256) scan_cols_k(const T* __restrict__ x, float* __restrict__ y, int64_t outer,
                                                   int64_t n, int64_t inner, float bias) {
  const int64_t lines = outer * inner;
  for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < lines; l += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = l / inner, in = l % inner;
    float acc = 0.f;
    for (int64_t j = 0; j < n; ++j) {
      const int64_t p = (o * n + j) * inner + in;
      acc += to_f(x[p]);
      y[p] = acc + bias;
    }
  }
}

// argmax along n: one wave per (outer, inner) output; first maximum wins (torch)
template <typename T>
__global__ void __launch_bounds__(256) argmax_k(const T* __restrict__ x, int64_t* __restrict__ out, int64_t outer,
                                                int64_t n, int64_t inner) {
  const int lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (line >= outer * inner) return;
  const int64_t o = line / inner, in = line % inner;
  float best = -INFINITY;
  int64_t bi = 0x7fffffffffffffffll;
  for (int64_t j = lane; j < n; j += 64) {
    const float v = to_f(x[(o * n + j) * inner + in]);
    if (v > best || (v == best && j < bi) || (v != v && best == best)) {   // NaN is the max (torch)
      best = v;
      bi = j;
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    const float ob = __shfl_xor(best, s, 64);
    const int64_t oi = __shfl_xor(bi, s, 64);
    const bool onan = ob != ob, bnan = best != best;
    if ((onan && !bnan) || (onan == bnan && (ob > best || (ob == best && oi < bi)))) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) out[line] = bi;
}

// bitonic sort of one row in LDS: (key, index) pairs, npow = power of two >= n
// (padding slots carry index >= n and sort after every real element), up to 8192
// elements (64 KiB).  Order: key ascending / descending with NaN as the largest key
// (torch), ties by index -- a total order, so the result is deterministic.
__device__ __forceinline__ bool key_lt(float a, float b) {
  if (a != a) return false;
  if (b != b) return true;
  return a < b;
}

__device__ __forceinline__ bool before(float a, int ia, float b, int ib, int n, int desc) {
  const bool pa = ia >= n, pb = ib >= n;
  if (pa || pb) return !pa || (pb && ia < ib);
  if (desc ? key_lt(b, a) : key_lt(a, b)) return true;
  if (desc ? key_lt(a, b) : key_lt(b, a)) return false;
  return ia < ib;
}

template <typename T>
__global__ void __launch_bounds__(1024) argsort_k(const T* __restrict__ x, int64_t* __restrict__ out, int64_t n,
                                                  int npow, int desc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* key = reinterpret_cast<float*>(smem);
  int* val = reinterpret_cast<int*>(smem + (size_t)npow * 4);
  const int64_t row = blockIdx.x;
  const T* xr = x + row * n;
  for (int i = threadIdx.x; i < npow; i += blockDim.x) {
    key[i] = i < n ? to_f(xr[i]) : 0.f;
    val[i] = i;
  }
  __syncthreads();
  for (int k = 2; k <= npow; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npow; i += blockDim.x) {
        const int p = i ^ j;
        if (p > i) {
          const float a = key[i], b = key[p];
          const int ia = val[i], ib = val[p];
          const bool up = (i & k) == 0;
          const bool swap = up ? before(b, ib, a, ia, (int)n, desc) : before(a, ia, b, ib, (int)n, desc);
          if (swap) {
            key[i] = b; key[p] = a;
            val[i] = ib; val[p] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[row * n + i] = val[i];
}

// p-norm along n: one wave per line
template <typename T>
__global__ void __launch_bounds__(256) pnorm_k(const T* __restrict__ x, T* __restrict__ y, int64_t outer, int64_t n,
                                               int64_t inner, float p) {
  const int lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (line >= outer * inner) return;
  const int64_t o = line / inner, in = line % inner;
  float s = 0.f;
  for (int64_t j = lane; j < n; j += 64) {
    const float v = fabsf(to_f(x[(o * n + j) * inner + in]));
    s += p == 2.f ? v * v : (p == 1.f ? v : powf(v, p));
  }
  s = wave_sum(s);
  if (lane == 0) y[line] = from_f<T>(p == 2.f ? sqrtf(s) : (p == 1.f ? s : powf(s, 1.f / p)));
}

// dx = sign(x) |x|^(p-1) / y^(p-1) * g, y and g broadcast along n
template <typename T>
__global__ void __launch_bounds__(256) pnorm_grad_k(const T* __restrict__ x, const T* __restrict__ y,
                                                    const T* __restrict__ g, T* __restrict__ dx, int64_t outer,
                                                    int64_t n, int64_t inner, float p) {
  const int64_t total = outer * n * inner;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t in = i % inner, o = i / (n * inner);
    const int64_t line = o * inner + in;
    const float xv = to_f(x[i]), yv = to_f(y[line]);
    const float den = fmaxf(p == 2.f ? yv : powf(yv, p - 1.f), 1e-12f);
    const float num = p == 2.f ? xv : copysignf(powf(fabsf(xv), p - 1.f), xv) * (xv != 0.f);
    dx[i] = from_f<T>(num / den * to_f(g[line]));
  }
}

}  // namespace

// ---- C API -----------------------------------------------------------------------------
// y[r][c] = x[r * xs] for c < C (a row broadcast along the contiguous dim, e.g. the
// gradient of a reduction over the last axis materialised): 16-byte stores of the
// replicated element; one thread per 16-byte chunk
template <typename T>
__global__ void __launch_bounds__(256) bcast_inner_k(const T* __restrict__ x, T* __restrict__ y, int64_t R,
                                                     int64_t C, int64_t xs, int64_t ys) {
  constexpr int V = 16 / sizeof(T);
  const int64_t cv = C / V;
  const int64_t n = R * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cv, c = (i - r * cv) * V;
    const T v = x[r * xs];
    union { T e[V]; uint4 u; } pk;
#pragma unroll
    for (int t = 0; t < V; ++t) pk.e[t] = v;
    *reinterpret_cast<uint4*>(y + r * ys + c) = pk.u;
  }
}

HETU_API int hetu_nd_copy(const void* x, void* y, int elem, int nd, const int64_t* shape, const int64_t* ostride,
                          const int64_t* istride, const int64_t* shift, const int64_t* imod, hipStream_t st) {
  if (nd < 1 || nd > MAXD) return (int)hipErrorInvalidValue;
  int64_t sh_[MAXD], os_[MAXD], is_[MAXD], sf_[MAXD], md_[MAXD];
  bool plain = true;
  int64_t total = 1;
  for (int k = 0; k < nd; ++k) {
    sh_[k] = shape[k]; os_[k] = ostride[k]; is_[k] = istride[k];
    sf_[k] = shift ? shift[k] : 0; md_[k] = imod ? imod[k] : 0;
    if (sf_[k] || md_[k]) plain = false;
    total *= shape[k];
  }
  if (total == 0) return 0;
  if (plain) {
    // drop unit dims, merge neighbours contiguous on both sides (outer = inner extent x stride)
    int m = 0;
    for (int k = 0; k < nd; ++k) {
      if (sh_[k] == 1) continue;
      if (m > 0 && os_[m - 1] == sh_[k] * os_[k] && is_[m - 1] == sh_[k] * is_[k]) {
        sh_[m - 1] *= sh_[k];
        os_[m - 1] = os_[k];
        is_[m - 1] = is_[k];
      } else {
        sh_[m] = sh_[k]; os_[m] = os_[k]; is_[m] = is_[k]; sf_[m] = 0; md_[m] = 0;
        ++m;
      }
    }
    if (m == 0) { sh_[0] = 1; os_[0] = 1; is_[0] = 1; sf_[0] = 0; md_[0] = 0; m = 1; }
    nd = m;
    // widen the element while the innermost dim is unit-stride on both sides
    while (elem < 16 && os_[nd - 1] == 1 && is_[nd - 1] == 1 && sh_[nd - 1] % 2 == 0 &&
           ((uintptr_t)x % (2 * elem)) == 0 && ((uintptr_t)y % (2 * elem)) == 0) {
      bool ok = true;
      for (int k = 0; k < nd - 1; ++k) ok = ok && os_[k] % 2 == 0 && is_[k] % 2 == 0;
      if (!ok) break;
      for (int k = 0; k < nd - 1; ++k) { os_[k] /= 2; is_[k] /= 2; }
      sh_[nd - 1] /= 2;
      elem *= 2;
    }
  }
  // row broadcast along the contiguous output dim (stride-0 input): replicated 16-byte stores
  if (plain && nd == 2 && os_[1] == 1 && is_[1] == 0 && elem <= 8 && (sh_[1] * elem) % 16 == 0 &&
      (os_[0] * elem) % 16 == 0 && ((uintptr_t)y & 15) == 0) {
    const int g = stream_grid(sh_[0] * (sh_[1] * elem / 16), 256, 2);
    switch (elem) {
      case 2: hipLaunchKernelGGL(bcast_inner_k<uint16_t>, dim3(g), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)y,
                                 sh_[0], sh_[1], is_[0], os_[0]); break;
      case 4: hipLaunchKernelGGL(bcast_inner_k<uint32_t>, dim3(g), dim3(256), 0, st, (const uint32_t*)x, (uint32_t*)y,
                                 sh_[0], sh_[1], is_[0], os_[0]); break;
      case 8: hipLaunchKernelGGL(bcast_inner_k<uint64_t>, dim3(g), dim3(256), 0, st, (const uint64_t*)x, (uint64_t*)y,
                                 sh_[0], sh_[1], is_[0], os_[0]); break;
      default: hipLaunchKernelGGL(bcast_inner_k<uint8_t>, dim3(g), dim3(256), 0, st, (const uint8_t*)x, (uint8_t*)y,
                                  sh_[0], sh_[1], is_[0], os_[0]); break;
    }
    return (int)hipGetLastError();
  }
  NDDesc d{};
  d.nd = nd;
  total = 1;
  int64_t eo = 0, ei = 0;
  for (int k = 0; k < nd; ++k) {
    d.shape[k] = sh_[k]; d.ostride[k] = os_[k]; d.istride[k] = is_[k]; d.shift[k] = sf_[k]; d.imod[k] = md_[k];
    total *= sh_[k];
    eo += (sh_[k] - 1) * (os_[k] < 0 ? -os_[k] : os_[k]);
    const int64_t reach = md_[k] > 0 ? md_[k] : sh_[k] - 1 + (sf_[k] < 0 ? -sf_[k] : sf_[k]);
    ei += reach * (is_[k] < 0 ? -is_[k] : is_[k]);
  }
  const bool small = total < (1ll << 31) && eo < (1ll << 31) && ei < (1ll << 31);
  const int g = stream_grid(total, 256, 4);
#define NDC(T)                                                                                      \
  if (small) hipLaunchKernelGGL((nd_copy_k<T, int32_t>), dim3(g), dim3(256), 0, st, (const T*)x, (T*)y, d, total); \
  else hipLaunchKernelGGL((nd_copy_k<T, int64_t>), dim3(g), dim3(256), 0, st, (const T*)x, (T*)y, d, total);
  switch (elem) {
    case 1: NDC(uint8_t) break;
    case 2: NDC(uint16_t) break;
    case 4: NDC(uint32_t) break;
    case 8: NDC(uint64_t) break;
    case 16: NDC(uint4) break;
    default: return (int)hipErrorInvalidValue;
  }
#undef NDC
  return (int)hipGetLastError();
}

// y[i][c] = (idx[i] == c) as fp32 (one_hot of int32 / int64 / fp32 class ids; ids out of
// [0, C) give a zero row).  One thread per 4 outputs, 16-byte stores.
template <typename T>
__global__ void __launch_bounds__(256) one_hot_k(const T* __restrict__ idx, float* __restrict__ y, int64_t n, int C) {
  const int64_t c4 = (C + 3) / 4;
  const int64_t total = n * c4;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / c4;
    const int c0 = (int)(t - i * c4) * 4;
    const int64_t k = (int64_t)idx[i];
    float4 v;
    v.x = k == c0 ? 1.f : 0.f;
    v.y = k == c0 + 1 ? 1.f : 0.f;
    v.z = k == c0 + 2 ? 1.f : 0.f;
    v.w = k == c0 + 3 ? 1.f : 0.f;
    float* dst = y + i * C + c0;
    if ((C & 3) == 0) {
      *reinterpret_cast<float4*>(dst) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; j < 4 && c0 + j < C; ++j) dst[j] = vv[j];
    }
  }
}

HETU_API int hetu_one_hot(const void* idx, int kind, float* y, int64_t n, int C, hipStream_t st) {
  if (n <= 0 || C <= 0) return 0;
  const int g = stream_grid(n * ((C + 3) / 4), 256, 4);
  switch (kind) {
    case 0: hipLaunchKernelGGL(one_hot_k<int64_t>, dim3(g), dim3(256), 0, st, (const int64_t*)idx, y, n, C); break;
    case 1: hipLaunchKernelGGL(one_hot_k<int32_t>, dim3(g), dim3(256), 0, st, (const int32_t*)idx, y, n, C); break;
    case 2: hipLaunchKernelGGL(one_hot_k<float>, dim3(g), dim3(256), 0, st, (const float*)idx, y, n, C); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// fill n elements of `elem` bytes with the bit pattern `bits`
HETU_API int hetu_fill(void* y, int elem, int64_t n, uint64_t bits, hipStream_t st) {
  if (n <= 0) return 0;
  const int g = stream_grid(n, 256, 4);
  switch (elem) {
    case 1: hipLaunchKernelGGL(fill_k<uint8_t>, dim3(g), dim3(256), 0, st, (uint8_t*)y, (uint8_t)bits, n); break;
    case 2: hipLaunchKernelGGL(fill_k<uint16_t>, dim3(g), dim3(256), 0, st, (uint16_t*)y, (uint16_t)bits, n); break;
    case 4: hipLaunchKernelGGL(fill_k<uint32_t>, dim3(g), dim3(256), 0, st, (uint32_t*)y, (uint32_t)bits, n); break;
    case 8: hipLaunchKernelGGL(fill_k<uint64_t>, dim3(g), dim3(256), 0, st, (uint64_t*)y, (uint64_t)bits, n); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

#define HETU_DT_DISPATCH(bf, KERNEL, GRID, BLOCK, SHM, ST, ...)                                  \
  do {                                                                                          \
    if (bf) hipLaunchKernelGGL(KERNEL<bf16>, GRID, BLOCK, SHM, ST, __VA_ARGS__);                \
    else hipLaunchKernelGGL(KERNEL<float>, GRID, BLOCK, SHM, ST, __VA_ARGS__);                  \
  } while (0)

HETU_API int hetu_gather_dim(const void* x, const int64_t* idx, void* y, int64_t outer, int64_t nidx, int64_t nsrc,
                             int64_t inner, int bf, hipStream_t st) {
  const int64_t total = outer * nidx * inner;
  if (total == 0) return 0;
  const dim3 g(stream_grid(total, 256, 2));
  if (bf) hipLaunchKernelGGL(gather_dim_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, idx, (bf16*)y, outer, nidx, nsrc, inner);
  else hipLaunchKernelGGL(gather_dim_k<float>, g, dim3(256), 0, st, (const float*)x, idx, (float*)y, outer, nidx, nsrc, inner);
  return (int)hipGetLastError();
}

HETU_API int hetu_scatter_add_dim(const void* g, const int64_t* idx, float* dx, int64_t outer, int64_t nidx,
                                  int64_t nsrc, int64_t inner, int bf, hipStream_t st) {
  const int64_t total = outer * nidx * inner;
  if (total == 0) return 0;
  const dim3 gr(stream_grid(total, 256, 2));
  if (bf) hipLaunchKernelGGL(scatter_add_dim_k<bf16>, gr, dim3(256), 0, st, (const bf16*)g, idx, dx, outer, nidx, nsrc, inner);
  else hipLaunchKernelGGL(scatter_add_dim_k<float>, gr, dim3(256), 0, st, (const float*)g, idx, dx, outer, nidx, nsrc, inner);
  return (int)hipGetLastError();
}

// y (fp32) = inclusive cumsum of x along n + bias
HETU_API int hetu_scan_dim(const void* x, float* y, int64_t outer, int64_t n, int64_t inner, float bias, int bf,
                           hipStream_t st) {
  if (outer * n * inner == 0) return 0;
  if (inner == 1) {
    const dim3 g((unsigned)((outer + 3) / 4));
    if (bf) hipLaunchKernelGGL(scan_rows_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, y, outer, n, bias);
    else hipLaunchKernelGGL(scan_rows_k<float>, g, dim3(256), 0, st, (const float*)x, y, outer, n, bias);
  } else {
    const dim3 g(stream_grid(outer * inner, 256));
    if (bf) hipLaunchKernelGGL(scan_cols_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, y, outer, n, inner, bias);
    else hipLaunchKernelGGL(scan_cols_k<float>, g, dim3(256), 0, st, (const float*)x, y, outer, n, inner, bias);
  }
  return (int)hipGetLastError();
}

HETU_API int hetu_argmax_dim(const void* x, int64_t* out, int64_t outer, int64_t n, int64_t inner, int bf,
                             hipStream_t st) {
  const int64_t lines = outer * inner;
  if (lines == 0) return 0;
  const dim3 g((unsigned)((lines + 3) / 4));
  if (bf) hipLaunchKernelGGL(argmax_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, out, outer, n, inner);
  else hipLaunchKernelGGL(argmax_k<float>, g, dim3(256), 0, st, (const float*)x, out, outer, n, inner);
  return (int)hipGetLastError();
}

// rows x n (contiguous rows), n <= 8192
HETU_API int hetu_argsort_rows(const void* x, int64_t* out, int64_t rows, int64_t n, int desc, int bf,
                               hipStream_t st) {
  if (n > 8192) return (int)hipErrorInvalidValue;
  if (rows == 0 || n == 0) return 0;
  int npow = 1;
  while (npow < n) npow <<= 1;
  const size_t shm = (size_t)npow * 8;
  const int nt = npow >= 1024 ? 1024 : (npow < 64 ? 64 : npow);
  if (bf) hipLaunchKernelGGL(argsort_k<bf16>, dim3((unsigned)rows), dim3(nt), shm, st, (const bf16*)x, out, n, npow, desc);
  else hipLaunchKernelGGL(argsort_k<float>, dim3((unsigned)rows), dim3(nt), shm, st, (const float*)x, out, n, npow, desc);
  return (int)hipGetLastError();
}

HETU_API int hetu_pnorm_dim(const void* x, void* y, int64_t outer, int64_t n, int64_t inner, float p, int bf,
                            hipStream_t st) {
  const int64_t lines = outer * inner;
  if (lines == 0) return 0;
  const dim3 g((unsigned)((lines + 3) / 4));
  if (bf) hipLaunchKernelGGL(pnorm_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, (bf16*)y, outer, n, inner, p);
  else hipLaunchKernelGGL(pnorm_k<float>, g, dim3(256), 0, st, (const float*)x, (float*)y, outer, n, inner, p);
  return (int)hipGetLastError();
}

HETU_API int hetu_pnorm_grad_dim(const void* x, const void* y, const void* g, void* dx, int64_t outer, int64_t n,
                                 int64_t inner, float p, int bf, hipStream_t st) {
  const int64_t total = outer * n * inner;
  if (total == 0) return 0;
  const dim3 gr(stream_grid(total, 256, 2));
  if (bf) hipLaunchKernelGGL(pnorm_grad_k<bf16>, gr, dim3(256), 0, st, (const bf16*)x, (const bf16*)y, (const bf16*)g, (bf16*)dx, outer, n, inner, p);
  else hipLaunchKernelGGL(pnorm_grad_k<float>, gr, dim3(256), 0, st, (const float*)x, (const float*)y, (const float*)g, (float*)dx, outer, n, inner, p);
  return (int)hipGetLastError();
}
