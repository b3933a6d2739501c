// LayerNorm over the last dimension + Philox dropout, gfx950.
//
// LayerNorm replaces src/ops/LayerNorm.cu (forward: block per row with
// E[x^2]-E[x]^2 variance; backward: 3 elementwise kernels + 4 cuDNN reductions +
// chunk workspaces).  Here: one wave per row, two-pass mean/variance in fp32,
// and a backward that writes dx in the same row pass while each wave keeps its
// own dgamma/dbeta partial slab (wave-exclusive, no atomics), folded by a
// second column-sum kernel.
#include "common.h"
#include <algorithm>

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
                                                  float keep, uint64_t seed_, const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
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


// ---------------------------------------------------------------------------
// Vectorised register-resident path (N % 4 == 0, N <= 2048): one wave per row
// holds the whole row in registers (CPL chunks of 4 per lane), optionally
// fused with "dropout(x) + residual" in front of the normalisation (BERT /
// Transformer post-LN blocks: LN(dropout(sublayer) + h)).  Dropout uses the
// same Philox counters as dropout_k (counter = flat element index / 4), so a
// standalone dropout with the same seed reproduces the mask.
template <typename T> struct IO4;
template <> struct IO4<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct IO4<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[4]) {
    uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&v)[4]) {
    uint2 x;
    x.x = (unsigned)f_to_bf16_bits(v[0]) | ((unsigned)f_to_bf16_bits(v[1]) << 16);
    x.y = (unsigned)f_to_bf16_bits(v[2]) | ((unsigned)f_to_bf16_bits(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = x;
  }
};

__device__ __forceinline__ void drop4(float (&v)[4], uint64_t seed, uint64_t ctr, float keep) {
  const uint4 r = Philox::gen(seed, ctr);
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  const float inv = 1.f / keep;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = Philox::u01(rr[k]) < keep ? v[k] * inv : 0.f;
}

template <typename T, int CPL>
__global__ void __launch_bounds__(256) ln_fwd4_k(const T* __restrict__ x, const T* __restrict__ res,
                                                  const float* __restrict__ g, const float* __restrict__ b,
                                                  T* __restrict__ y, T* __restrict__ sum_out,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                  int64_t R, int N, float eps, float keep, uint64_t seed_,
                                                  const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = N >> 2;
  const int64_t base = row * N;
  float v[CPL][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nc) {
      IO4<T>::load(x + base + 4 * c, v[i]);
      if (keep < 1.f) drop4(v[i], seed, (uint64_t)(base >> 2) + c, keep);
      if (res != nullptr) {
        float r4[4];
        IO4<T>::load(res + base + 4 * c, r4);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[i][k] += r4[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) s += v[i][k];
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    if (lane + 64 * i < nc) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = v[i][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)N + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nc) {
      if (sum_out != nullptr) IO4<T>::store(sum_out + base + 4 * c, v[i]);
      const float4 gg = *reinterpret_cast<const float4*>(g + 4 * c);
      const float4 bb = *reinterpret_cast<const float4*>(b + 4 * c);
      float o[4];
      o[0] = (v[i][0] - mean) * rstd * gg.x + bb.x;
      o[1] = (v[i][1] - mean) * rstd * gg.y + bb.y;
      o[2] = (v[i][2] - mean) * rstd * gg.z + bb.z;
      o[3] = (v[i][3] - mean) * rstd * gg.w + bb.w;
      IO4<T>::store(y + base + 4 * c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward: dsum = LN'(dy) per row (wave per row, rows of one block strided
// over its 4 waves); dx_drop = dropout-mask(dsum) when the forward fused a
// dropout; dgamma/dbeta accumulate in registers, are folded across the 4
// waves in LDS and written as one partial row per workgroup (col_reduce2_k
// finishes them).  LDS: 4 * N floats (dynamic).
template <typename T, int CPL, int NW = 4>
__global__ void __launch_bounds__(64 * NW) ln_bwd4_k(const T* __restrict__ dy, const T* __restrict__ xs,
                                                  const float* __restrict__ g, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, T* __restrict__ dsum,
                                                  T* __restrict__ dx_drop, float* __restrict__ pg,
                                                  float* __restrict__ pb, int64_t R, int N, int rpb, float keep,
                                                  uint64_t seed_, const uint64_t* __restrict__ rngo,
                                                  float* __restrict__ zero_a,
                                                  float* __restrict__ zero_b, float* __restrict__ pd,
                                                  float* __restrict__ zero_d) {
  extern __shared__ float lds[];
  const uint64_t seed = rng_seed(seed_, rngo);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nc = N >> 2;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  // ad: column sums of the x-gradient (after the dropout mask) -- the bias
  // gradient of the linear layer that produced x, when pd != nullptr
  float gm[CPL][4], ag[CPL][4], ab[CPL][4], ad[CPL][4];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nc) {
      const float4 t = *reinterpret_cast<const float4*>(g + 4 * c);
      gm[i][0] = t.x; gm[i][1] = t.y; gm[i][2] = t.z; gm[i][3] = t.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) gm[i][k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) { ag[i][k] = 0.f; ab[i][k] = 0.f; ad[i][k] = 0.f; }
  }
  if (zero_a != nullptr && blockIdx.x == 0)   // col_reduce2_k accumulates its row slices into these
    for (int j = threadIdx.x; j < N; j += 64 * NW) {
      zero_a[j] = 0.f;
      zero_b[j] = 0.f;
      if (zero_d != nullptr) zero_d[j] = 0.f;
    }
  // software-pipelined over this wave's rows: the next row's loads are in flight
  // while the current row is reduced and written
  float d[CPL][4], xh[CPL][4];
  auto load_row = [&](int64_t rw, float (&dd)[CPL][4], float (&xx)[CPL][4]) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
        IO4<T>::load(dy + rw * N + 4 * c, dd[i]);
        IO4<T>::load(xs + rw * N + 4 * c, xx[i]);
      }
    }
  };
  if (r0 + w < r1) load_row(r0 + w, d, xh);
  for (int64_t row = r0 + w; row < r1; row += NW) {
    const int64_t base = row * N;
    const float mu = mean[row], rs = rstd[row];
    float dn[CPL][4], xn[CPL][4];
    if (row + NW < r1) load_row(row + NW, dn, xn);
    float a = 0.f, cc = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xh[i][k] = (xh[i][k] - mu) * rs;
          const float dg = d[i][k] * gm[i][k];
          a += dg;
          cc += dg * xh[i][k];
          ag[i][k] += d[i][k] * xh[i][k];
          ab[i][k] += d[i][k];
        }
      }
    }
    a = wave_sum(a) / (float)N;
    cc = wave_sum(cc) / (float)N;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rs * (d[i][k] * gm[i][k] - a - xh[i][k] * cc);
        if (dsum != nullptr) IO4<T>::store(dsum + base + 4 * c, o);
        if (dx_drop != nullptr) {
          drop4(o, seed, (uint64_t)(base >> 2) + c, keep);
          IO4<T>::store(dx_drop + base + 4 * c, o);
        }
        if (pd != nullptr) {
#pragma unroll
          for (int k = 0; k < 4; ++k) ad[i][k] += o[k];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) { d[i][k] = dn[i][k]; xh[i][k] = xn[i][k]; }
  }
  // fold the 4 waves' partials (dgamma, dbeta, then the x-gradient column sums) through LDS
  const int npass = pd != nullptr ? 3 : 2;
  for (int pass = 0; pass < npass; ++pass) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
#pragma unroll
        for (int k = 0; k < 4; ++k) lds[w * N + 4 * c + k] = pass == 0 ? ag[i][k] : (pass == 1 ? ab[i][k] : ad[i][k]);
      }
    }
    __syncthreads();
    float* out = (pass == 0 ? pg : (pass == 1 ? pb : pd)) + (int64_t)blockIdx.x * N;
    for (int j = threadIdx.x; j < N; j += 64 * NW) {
      float t = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) t += lds[ww * N + j];
      out[j] = t;
    }
    __syncthreads();
  }
}

// oa[j] = sum_r pa[r, j], ob[j] = sum_r pb[r, j] (and oc[j] = sum_r pc[r, j] when pc
// is given; pb may be null): 64 columns x 4 row groups per block.
// gridDim.y > 1 splits the rows into slices whose sums are atomically added into
// oa / ob / oc (zeroed beforehand by the producer kernel): the few hundred partial
// rows are otherwise reduced by only N/64 blocks, latency-bound.  gridDim.y == 1
// stores (fixed summation order: deterministic mode).
__global__ void __launch_bounds__(256) col_reduce2_k(const float* __restrict__ pa, const float* __restrict__ pb,
                                                      float* __restrict__ oa, float* __restrict__ ob, int rows,
                                                      int N, const float* __restrict__ pc = nullptr,
                                                      float* __restrict__ oc = nullptr) {
  __shared__ float sm[3][4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (rows + (int)gridDim.y - 1) / (int)gridDim.y;
  const int rlo = (int)blockIdx.y * per;
  const int rhi = rlo + per < rows ? rlo + per : rows;
  const float* src[3] = {pa, pb, pc};
  float* dst[3] = {oa, ob, oc};
  // all arrays in one loop, 4 rows each in flight (null arrays are skipped uniformly)
  float t[3][4];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int u = 0; u < 4; ++u) t[a][u] = 0.f;
  if (col < N) {
    int r = rlo + grp;
    for (; r + 12 < rhi; r += 16) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (src[a] == nullptr) continue;
#pragma unroll
        for (int u = 0; u < 4; ++u) t[a][u] += src[a][(int64_t)(r + 4 * u) * N + col];
      }
    }
    for (; r < rhi; r += 4) {
#pragma unroll
      for (int a = 0; a < 3; ++a)
        if (src[a] != nullptr) t[a][0] += src[a][(int64_t)r * N + col];
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) sm[a][grp][lane] = t[a][0] + t[a][1] + t[a][2] + t[a][3];
  __syncthreads();
  if (grp == 0 && col < N) {
    for (int a = 0; a < 3; ++a) {
      if (src[a] == nullptr) continue;
      const float t = sm[a][0][lane] + sm[a][1][lane] + sm[a][2][lane] + sm[a][3][lane];
      if (gridDim.y == 1) dst[a][col] = t;
      else unsafeAtomicAdd(dst[a] + col, t);
    }
  }
}

// g = dy * gelu'(pre) (erf form) for a [R, N] activation, plus the column sums
// of g: the bias gradient of the linear layer whose output went through the
// GELU (transformer FFN1).  Geometry as the BatchNorm partial kernels: a block
// covers W vector-columns x RP rows per pass over its chunk of rows; each block
// writes one partial row part[blockIdx.x][N] (reduced by col_reduce2_k).  Blocks
// with blockIdx.x == 0 zero ``zero_out`` for the atomic row-slice reduce.
__device__ __forceinline__ float gelu_erf_grad_f(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118f));
  const float pdf = 0.39894228040f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <typename T>
__global__ void __launch_bounds__(256) gelu_grad_colsum_k(const T* __restrict__ pre, const T* __restrict__ dy,
                                                           T* __restrict__ g, int64_t R, int N, int W, int RP,
                                                           int64_t rows_per_chunk, float* __restrict__ part,
                                                           float* __restrict__ zero_out) {
  constexpr int V = Vec<T>::N;
  __shared__ float sh[256 * V];
  const int t = threadIdx.x;
  const int col = t % W, rsub = t / W;
  const int vc = blockIdx.y * W + col;
  const bool active = (rsub < RP) && (vc * V < N);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > R) r1 = R;
  if (zero_out != nullptr && blockIdx.x == 0 && rsub == 0 && vc * V < N) {
#pragma unroll
    for (int k = 0; k < V; ++k) zero_out[vc * V + k] = 0.f;
  }
  float s[V];
#pragma unroll
  for (int k = 0; k < V; ++k) s[k] = 0.f;
  if (active) {
    int64_t r = r0 + rsub;
    for (; r + RP < r1; r += 2 * RP) {   // two rows (four vectors) in flight
      const int64_t o1 = r * N + (int64_t)vc * V, o2 = o1 + (int64_t)RP * N;
      float a1[V], b1[V], a2[V], b2[V];
      load_vec<T>(pre + o1, a1);
      load_vec<T>(dy + o1, b1);
      load_vec<T>(pre + o2, a2);
      load_vec<T>(dy + o2, b2);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        b1[k] *= gelu_erf_grad_f(a1[k]);
        b2[k] *= gelu_erf_grad_f(a2[k]);
        s[k] += b1[k] + b2[k];
      }
      store_vec<T>(g + o1, b1);
      store_vec<T>(g + o2, b2);
    }
    for (; r < r1; r += RP) {
      const int64_t o1 = r * N + (int64_t)vc * V;
      float a1[V], b1[V];
      load_vec<T>(pre + o1, a1);
      load_vec<T>(dy + o1, b1);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        b1[k] *= gelu_erf_grad_f(a1[k]);
        s[k] += b1[k];
      }
      store_vec<T>(g + o1, b1);
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) sh[t * V + k] = s[k];
  __syncthreads();
  const int nch = W * V;
  for (int c_local = t; c_local < nch; c_local += 256) {
    const int colw = c_local / V, lane_i = c_local % V;
    float S = 0.f;
    for (int rr = 0; rr < RP; ++rr) S += sh[(rr * W + colw) * V + lane_i];
    const int c = blockIdx.y * W * V + c_local;
    if (c < N) part[(int64_t)blockIdx.x * N + c] = S;
  }
}

template <typename T, int CPL>
static void launch_fwd4(const void* x, const void* res, const float* g, const float* b, void* y, void* sum_out,
                        float* mean, float* rstd, int64_t R, int N, float eps, float keep, uint64_t seed,
                        hipStream_t st) {
  hipLaunchKernelGGL((ln_fwd4_k<T, CPL>), dim3((unsigned)((R + 3) / 4)), dim3(256), 0, st, (const T*)x,
                     (const T*)res, g, b, (T*)y, (T*)sum_out, mean, rstd, R, N, eps, keep, seed,
                     hetu_rng_offset_ptr());
}

// waves: rows in flight per block (4 or 8); the per-block partial-row count (nblk) is the
// same, so 8 waves double the memory-level parallelism at no extra partial traffic
template <typename T, int CPL>
static void launch_bwd4(const void* dy, const void* xs, const float* g, const float* mean, const float* rstd,
                        void* dsum, void* dxd, float* pg, float* pb, int64_t R, int N, int nblk, int rpb,
                        float keep, uint64_t seed, float* za, float* zb, float* pd, float* zd, int waves,
                        hipStream_t st) {
  if (waves == 8)
    hipLaunchKernelGGL((ln_bwd4_k<T, CPL, 8>), dim3((unsigned)nblk), dim3(512), 8 * N * sizeof(float), st,
                       (const T*)dy, (const T*)xs, g, mean, rstd, (T*)dsum, (T*)dxd, pg, pb, R, N, rpb, keep, seed,
                       hetu_rng_offset_ptr(), za, zb, pd, zd);
  else
    hipLaunchKernelGGL((ln_bwd4_k<T, CPL, 4>), dim3((unsigned)nblk), dim3(256), 4 * N * sizeof(float), st,
                       (const T*)dy, (const T*)xs, g, mean, rstd, (T*)dsum, (T*)dxd, pg, pb, R, N, rpb, keep, seed,
                       hetu_rng_offset_ptr(), za, zb, pd, zd);
}

#define HETU_CPL_DISPATCH(CPL_NEEDED, FN, ...)                 \
  do {                                                         \
    const int cpl_ = (CPL_NEEDED);                             \
    if (cpl_ <= 1) FN<1>(__VA_ARGS__);                         \
    else if (cpl_ <= 2) FN<2>(__VA_ARGS__);                    \
    else if (cpl_ <= 3) FN<3>(__VA_ARGS__);                    \
    else if (cpl_ <= 4) FN<4>(__VA_ARGS__);                    \
    else if (cpl_ <= 6) FN<6>(__VA_ARGS__);                    \
    else FN<8>(__VA_ARGS__);                                   \
  } while (0)

template <int CPL> static void fwd4_bf16(const void* x, const void* res, const float* g, const float* b, void* y,
                                         void* so, float* m, float* r, int64_t R, int N, float eps, float keep,
                                         uint64_t seed, hipStream_t st) {
  launch_fwd4<bf16, CPL>(x, res, g, b, y, so, m, r, R, N, eps, keep, seed, st);
}
template <int CPL> static void fwd4_f32(const void* x, const void* res, const float* g, const float* b, void* y,
                                        void* so, float* m, float* r, int64_t R, int N, float eps, float keep,
                                        uint64_t seed, hipStream_t st) {
  launch_fwd4<float, CPL>(x, res, g, b, y, so, m, r, R, N, eps, keep, seed, st);
}
template <int CPL> static void bwd4_bf16(const void* dy, const void* xs, const float* g, const float* m,
                                         const float* r, void* ds, void* dxd, float* pg, float* pb, int64_t R,
                                         int N, int nblk, int rpb, float keep, uint64_t seed, float* za,
                                         float* zb, float* pd, float* zd, int waves, hipStream_t st) {
  launch_bwd4<bf16, CPL>(dy, xs, g, m, r, ds, dxd, pg, pb, R, N, nblk, rpb, keep, seed, za, zb, pd, zd, waves, st);
}
template <int CPL> static void bwd4_f32(const void* dy, const void* xs, const float* g, const float* m,
                                        const float* r, void* ds, void* dxd, float* pg, float* pb, int64_t R,
                                        int N, int nblk, int rpb, float keep, uint64_t seed, float* za,
                                        float* zb, float* pd, float* zd, int waves, hipStream_t st) {
  launch_bwd4<float, CPL>(dy, xs, g, m, r, ds, dxd, pg, pb, R, N, nblk, rpb, keep, seed, za, zb, pd, zd, waves, st);
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
  hipLaunchKernelGGL(col_reduce2_k, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, st, wg, wb, dg, db, nwaves, N,
                     (const float*)nullptr, (float*)nullptr);
  HETU_LAUNCH_CHECK();
  return 0;
}

// vector form (n % 8 == 0, 16-byte aligned x / y): 8 elements per thread per step -- two
// Philox counters (i / 4, i / 4 + 1, the scalar kernel's mask) and 16-byte (bf16) or
// 2 x 16-byte (fp32) accesses; the scalar form's per-element 2-byte accesses ran the MoE
// experts' [65536 x 2048] dropouts at half the HBM bandwidth
template <typename T>
__global__ void __launch_bounds__(256) dropout8_k(const T* __restrict__ x, T* __restrict__ y, int64_t n8,
                                                  float keep, uint64_t seed_, const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
  const float inv = 1.f / keep;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n8; j += (int64_t)gridDim.x * blockDim.x) {
    float a[4], b[4];
    IO4<T>::load(x + 8 * j, a);
    IO4<T>::load(x + 8 * j + 4, b);
    const uint4 r0 = Philox::gen(seed, (uint64_t)(2 * j));
    const uint4 r1 = Philox::gen(seed, (uint64_t)(2 * j + 1));
    const uint32_t q0[4] = {r0.x, r0.y, r0.z, r0.w}, q1[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = Philox::u01(q0[k]) < keep ? a[k] * inv : 0.f;
      b[k] = Philox::u01(q1[k]) < keep ? b[k] * inv : 0.f;
    }
    IO4<T>::store(y + 8 * j, a);
    IO4<T>::store(y + 8 * j + 4, b);
  }
}

HETU_API int hetu_dropout(const void* x, void* y, int64_t n, float keep, int64_t seed, int is_bf16,
                          hipStream_t st) {
  if ((n & 7) == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
    const int g8 = stream_grid(n / 8, 256, 2);
    if (is_bf16) hipLaunchKernelGGL(dropout8_k<bf16>, dim3(g8), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n / 8, keep, (uint64_t)seed, hetu_rng_offset_ptr());
    else hipLaunchKernelGGL(dropout8_k<float>, dim3(g8), dim3(256), 0, st, (const float*)x, (float*)y, n / 8, keep, (uint64_t)seed, hetu_rng_offset_ptr());
    HETU_LAUNCH_CHECK();
    return 0;
  }
  int grid = stream_grid((n + 3) / 4, 256, 1);
  if (is_bf16) hipLaunchKernelGGL(dropout_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n, keep, (uint64_t)seed, hetu_rng_offset_ptr());
  else hipLaunchKernelGGL(dropout_k<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, n, keep, (uint64_t)seed, hetu_rng_offset_ptr());
  HETU_LAUNCH_CHECK();
  return 0;
}

// Fused [dropout(x) + residual ->] LayerNorm forward.  res / sum_out may be null;
// keep >= 1 disables dropout.  Requires N % 4 == 0 and N <= 2048 (returns
// hipErrorInvalidValue otherwise -- the caller falls back to hetu_layernorm_fwd).
HETU_API int hetu_ln_fused_fwd(const void* x, const void* res, const float* g, const float* b, void* y,
                               void* sum_out, float* mean, float* rstd, int64_t R, int N, float eps, float keep,
                               int64_t seed, int is_bf16, hipStream_t st) {
  if ((N & 3) || N > 2048 || R <= 0) return (int)hipErrorInvalidValue;
  const int cpl = (N / 4 + 63) / 64;
  if (is_bf16) HETU_CPL_DISPATCH(cpl, fwd4_bf16, x, res, g, b, y, sum_out, mean, rstd, R, N, eps, keep, (uint64_t)seed, st);
  else HETU_CPL_DISPATCH(cpl, fwd4_f32, x, res, g, b, y, sum_out, mean, rstd, R, N, eps, keep, (uint64_t)seed, st);
  HETU_LAUNCH_CHECK();
  return 0;
}

// Backward of the fused forward.  xs = the normalised input (x + res after
// dropout, or x).  dsum (grad of xs / of the residual) and dx_drop (grad of x
// through the dropout) may each be null.  ws: 2 * nblk * N floats.
// deterministic != 0: the dgamma/dbeta partial rows are summed in a fixed order
// (one block per 64 columns) instead of by row slices with fp32 atomics.
// dlin (may be null): also the column sums of the x-gradient (dx_drop, or dsum
// without dropout) -- the bias gradient of the linear layer that produced x --
// from the same row pass.  ws: (2 + (dlin != null)) * nblk * N floats.
// waves: 4 or 8 rows in flight per block (hetu_ln_fused_bwd2 = 4)
HETU_API int hetu_ln_fused_bwd3(const void* dy, const void* xs, const float* g, const float* mean, const float* rstd,
                                void* dsum, void* dx_drop, float* dg, float* db, float* dlin, float* ws, int64_t R,
                                int N, int nblk, float keep, int64_t seed, int is_bf16, int deterministic, int waves,
                                hipStream_t st) {
  if (waves != 4 && waves != 8) return (int)hipErrorInvalidValue;
  if ((N & 3) || N > 2048 || R <= 0 || nblk <= 0) return (int)hipErrorInvalidValue;
  const int cpl = (N / 4 + 63) / 64;
  const int rpb = (int)((R + nblk - 1) / nblk);
  float* pg = ws;
  float* pb = ws + (int64_t)nblk * N;
  float* pd = dlin != nullptr ? ws + 2 * (int64_t)nblk * N : nullptr;
  // ~16 partial rows per slice: one pass of 4 loads per array and thread, and hundreds of
  // blocks instead of N/64 x 8 (the reduce was latency-bound at 6-9 us per LayerNorm)
  const int slices = deterministic ? 1 : std::max(1, std::min(64, nblk / 16));
  float* za = slices > 1 ? dg : nullptr;
  float* zb = slices > 1 ? db : nullptr;
  float* zd = slices > 1 ? dlin : nullptr;
  if (is_bf16) HETU_CPL_DISPATCH(cpl, bwd4_bf16, dy, xs, g, mean, rstd, dsum, dx_drop, pg, pb, R, N, nblk, rpb, keep, (uint64_t)seed, za, zb, pd, zd, waves, st);
  else HETU_CPL_DISPATCH(cpl, bwd4_f32, dy, xs, g, mean, rstd, dsum, dx_drop, pg, pb, R, N, nblk, rpb, keep, (uint64_t)seed, za, zb, pd, zd, waves, st);
  hipLaunchKernelGGL(col_reduce2_k, dim3((unsigned)((N + 63) / 64), (unsigned)slices), dim3(256), 0, st, pg, pb, dg,
                     db, nblk, N, (const float*)pd, dlin);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_ln_fused_bwd2(const void* dy, const void* xs, const float* g, const float* mean, const float* rstd,
                                void* dsum, void* dx_drop, float* dg, float* db, float* dlin, float* ws, int64_t R,
                                int N, int nblk, float keep, int64_t seed, int is_bf16, int deterministic,
                                hipStream_t st) {
  return hetu_ln_fused_bwd3(dy, xs, g, mean, rstd, dsum, dx_drop, dg, db, dlin, ws, R, N, nblk, keep, seed, is_bf16,
                            deterministic, 4, st);
}

HETU_API int hetu_ln_fused_bwd(const void* dy, const void* xs, const float* g, const float* mean, const float* rstd,
                               void* dsum, void* dx_drop, float* dg, float* db, float* ws, int64_t R, int N,
                               int nblk, float keep, int64_t seed, int is_bf16, int deterministic, hipStream_t st) {
  return hetu_ln_fused_bwd2(dy, xs, g, mean, rstd, dsum, dx_drop, dg, db, nullptr, ws, R, N, nblk, keep, seed,
                            is_bf16, deterministic, st);
}

// g = dy * gelu'(pre) and out[N] = column sums of g (the FFN1 bias gradient).
// Requires N % (16 / sizeof(T)) == 0 and 16-byte aligned rows; ``chunks`` partial
// rows in ws (chunks * N floats).
HETU_API int hetu_gelu_grad_colsum(const void* pre, const void* dy, void* g, float* out, float* ws, int64_t R,
                                   int N, int chunks, int is_bf16, int deterministic, hipStream_t st) {
  const int V = is_bf16 ? 8 : 4;
  if (N % V || R <= 0 || chunks <= 0) return (int)hipErrorInvalidValue;
  const int cv = N / V;
  const int W = cv < 64 ? cv : 64;
  const int RP = 256 / W;
  const int tiles = (cv + W - 1) / W;
  const int64_t rpc = (R + chunks - 1) / chunks;
  const int slices = deterministic ? 1 : std::max(1, std::min(64, chunks / 16));
  float* zo = slices > 1 ? out : nullptr;
  if (is_bf16)
    hipLaunchKernelGGL(gelu_grad_colsum_k<bf16>, dim3((unsigned)chunks, (unsigned)tiles), dim3(256), 0, st,
                       (const bf16*)pre, (const bf16*)dy, (bf16*)g, R, N, W, RP, rpc, ws, zo);
  else
    hipLaunchKernelGGL(gelu_grad_colsum_k<float>, dim3((unsigned)chunks, (unsigned)tiles), dim3(256), 0, st,
                       (const float*)pre, (const float*)dy, (float*)g, R, N, W, RP, rpc, ws, zo);
  hipLaunchKernelGGL(col_reduce2_k, dim3((unsigned)((N + 63) / 64), (unsigned)slices), dim3(256), 0, st, ws,
                     (const float*)nullptr, out, (float*)nullptr, chunks, N, (const float*)nullptr, (float*)nullptr);
  HETU_LAUNCH_CHECK();
  return 0;
}
