// Embedding gather, row scatter-add and row-sparse optimizer updates.
//
// Replaces src/ops/EmbeddingLookup.cu (one THREAD per id copying a whole row
// serially), IndexedSlices.cu and OptimizersSparse.cu.  Here one 64-lane wave
// moves one row with 16-byte lanes (8 bf16 / 4 fp32 per lane), ids are int64
// (no float-encoded ids), out-of-range ids produce zero rows like
// the reference.  Sparse updates run on de-duplicated rows (unique ids), so
// every row is owned by exactly one wave: no atomics, deterministic.
#include "common.h"
#include <algorithm>

namespace hetu {

template <typename T>
__global__ void __launch_bounds__(256) gather_rows_k(const T* __restrict__ table, const int64_t* __restrict__ ids,
                                                      T* __restrict__ out, int64_t n, int64_t dim,
                                                      int64_t nrows) {
  constexpr int V = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    const bool ok = id >= 0 && id < nrows;
    T* o = out + r * dim;
    if (dim % V == 0) {
      for (int64_t j = lane * V; j < dim; j += 64 * V) {
        float v[V];
        if (ok) load_vec<T>(table + id * dim + j, v);
        else {
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = 0.f;
        }
        store_vec<T>(o + j, v);
      }
    } else {
      for (int64_t j = lane; j < dim; j += 64) o[j] = ok ? table[id * dim + j] : from_f<T>(0.f);
    }
  }
}

// dst[ids[r], :] += src[r, :]  (fp32 destination, atomics; used for dense grads)
template <typename T>
__global__ void __launch_bounds__(256) scatter_add_rows_k(float* __restrict__ dst, const int64_t* __restrict__ ids,
                                                           const T* __restrict__ src, int64_t n,
                                                           int64_t dim, int64_t nrows) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= nrows) continue;
    for (int64_t j = lane; j < dim; j += 64) atomicAdd(dst + id * dim + j, to_f(src[r * dim + j]));
  }
}

// Deterministic scatter-add (Executor(deterministic=True)): the
// rows are pre-sorted by destination (stable), segment s = rows perm[off[s]..off[s+1])
// all go to dst row seg_row[s]; one wave owns a segment and sums its rows in order,
// so every destination row is written once, by one wave: bitwise reproducible.
template <typename T>
__global__ void __launch_bounds__(256) segment_sum_rows_k(float* __restrict__ dst,
                                                           const int64_t* __restrict__ seg_row,
                                                           const int64_t* __restrict__ off,
                                                           const int64_t* __restrict__ perm,
                                                           const T* __restrict__ src, int64_t nseg,
                                                           int64_t dim, int64_t nrows) {
  const int lane = threadIdx.x & 63;
  for (int64_t sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); sg < nseg; sg += (int64_t)gridDim.x * 4) {
    const int64_t id = seg_row[sg];
    if (id < 0 || id >= nrows) continue;
    const int64_t q0 = off[sg], q1 = off[sg + 1];
    for (int64_t j = lane; j < dim; j += 64) {
      float acc = dst[id * dim + j];
      for (int64_t q = q0; q < q1; ++q) acc += to_f(src[perm[q] * dim + j]);
      dst[id * dim + j] = acc;
    }
  }
}

enum { SP_SGD = 0, SP_MOMENTUM = 1, SP_NESTEROV = 2, SP_ADAGRAD = 3, SP_ADAM = 4, SP_ADAMW = 5 };

template <int MODE>
__global__ void __launch_bounds__(256) sparse_opt_k(float* __restrict__ table, float* __restrict__ s1,
                                                     float* __restrict__ s2, const int64_t* __restrict__ ids,
                                                     const float* __restrict__ g, int64_t n, int64_t dim,
                                                     int64_t nrows, float lr, float l2, float mu,
                                                     float b1, float b2, float b1t, float b2t,
                                                     float eps, float wd) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= nrows) continue;
    for (int64_t j = lane; j < dim; j += 64) {
      const int64_t o = id * dim + j;
      float p = table[o];
      float gr = g[r * dim + j] + l2 * p;
      if (MODE == SP_SGD) {
        p -= lr * gr;
      } else if (MODE == SP_MOMENTUM) {
        float v = mu * s1[o] - lr * gr;
        s1[o] = v;
        p += v;
      } else if (MODE == SP_NESTEROV) {
        float t = lr * gr;
        float v = mu * (s1[o] - t);
        s1[o] = v;
        p += v - t;
      } else if (MODE == SP_ADAGRAD) {
        float a = s1[o] + gr * gr;
        s1[o] = a;
        p -= lr * gr / (sqrtf(a) + eps);
      } else {
        float m = b1 * s1[o] + (1.f - b1) * gr;
        float v = b2 * s2[o] + (1.f - b2) * gr * gr;
        s1[o] = m;
        s2[o] = v;
        float u = (m / (1.f - b1t)) / (sqrtf(v / (1.f - b2t)) + eps);
        p -= (MODE == SP_ADAM) ? lr * u : lr * (u + wd * p);
      }
      table[o] = p;
    }
  }
}

}  // namespace hetu

using namespace hetu;

static inline int rows_blocks(int64_t n) {
  int64_t b = (n + 3) / 4;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

// ---- sync-free dedup of a small table's row gradients (BERT position / token-type
// embeddings): rows scattered into K private replicas (row r -> replica r % K) with a
// hit mark per destination, then the replicas summed and ids[r] = r or -1 (untouched).
// Three launches, nothing depends on the number of distinct ids (no host sync).
template <typename T>
__global__ void __launch_bounds__(256) dedup_scatter_k(float* __restrict__ scratch, int* __restrict__ hit,
                                                        const int64_t* __restrict__ ids, const T* __restrict__ src,
                                                        int64_t n, int64_t dim, int64_t nrows, int K) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= nrows) continue;
    if (lane == 0) hit[id] = 1;
    float* d = scratch + ((r % K) * nrows + id) * dim;
    for (int64_t j = lane; j < dim; j += 64) atomicAdd(d + j, to_f(src[r * dim + j]));
  }
}

__global__ void __launch_bounds__(256) dedup_reduce_k(const float* __restrict__ scratch, const int* __restrict__ hit,
                                                       float* __restrict__ merged, int64_t* __restrict__ out_ids,
                                                       int64_t nrows, int64_t dim, int K) {
  const int64_t total = nrows * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += scratch[k * total + i];
    merged[i] = s;
    const int64_t row = i / dim;
    if (i - row * dim == 0) out_ids[row] = hit[row] ? row : -1;
  }
}

// scratch: K*nrows*dim fp32 and hit: nrows int32, both zeroed by the caller (hetu_fill)
HETU_API int hetu_dedup_rows_dense(const int64_t* ids, const void* src, int src_bf16, int64_t n, int64_t dim,
                                   int64_t nrows, int K, float* scratch, int* hit, float* merged, int64_t* out_ids,
                                   hipStream_t st) {
  if (K < 1) K = 1;
  if (n > 0) {
    if (src_bf16)
      hipLaunchKernelGGL(dedup_scatter_k<bf16>, dim3(rows_blocks(n)), dim3(256), 0, st, scratch, hit, ids,
                         (const bf16*)src, n, dim, nrows, K);
    else
      hipLaunchKernelGGL(dedup_scatter_k<float>, dim3(rows_blocks(n)), dim3(256), 0, st, scratch, hit, ids,
                         (const float*)src, n, dim, nrows, K);
  }
  const int64_t total = nrows * dim;
  int64_t nb = (total + 255) / 256;
  if (nb > 2048) nb = 2048;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(dedup_reduce_k, dim3((unsigned)nb), dim3(256), 0, st, scratch, hit, merged, out_ids, nrows, dim, K);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_gather_rows(const void* table, const int64_t* ids, void* out, int64_t n,
                              int64_t dim, int64_t nrows, int is_bf16, hipStream_t st) {
  if (n <= 0) return 0;
  if (is_bf16) hipLaunchKernelGGL(gather_rows_k<bf16>, dim3(rows_blocks(n)), dim3(256), 0, st, (const bf16*)table, ids, (bf16*)out, n, dim, nrows);
  else hipLaunchKernelGGL(gather_rows_k<float>, dim3(rows_blocks(n)), dim3(256), 0, st, (const float*)table, ids, (float*)out, n, dim, nrows);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_scatter_add_rows(float* dst, const int64_t* ids, const void* src, int64_t n,
                                   int64_t dim, int64_t nrows, int src_bf16, hipStream_t st) {
  if (n <= 0) return 0;
  if (src_bf16) hipLaunchKernelGGL(scatter_add_rows_k<bf16>, dim3(rows_blocks(n)), dim3(256), 0, st, dst, ids, (const bf16*)src, n, dim, nrows);
  else hipLaunchKernelGGL(scatter_add_rows_k<float>, dim3(rows_blocks(n)), dim3(256), 0, st, dst, ids, (const float*)src, n, dim, nrows);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_segment_sum_rows(float* dst, const int64_t* seg_row, const int64_t* off,
                                   const int64_t* perm, const void* src, int64_t nseg, int64_t dim,
                                   int64_t nrows, int src_bf16, hipStream_t st) {
  if (nseg <= 0) return 0;
  int grid = (int)std::min<int64_t>((nseg + 3) / 4, 65535);
  if (src_bf16)
    hipLaunchKernelGGL(segment_sum_rows_k<bf16>, dim3(grid), dim3(256), 0, st, dst, seg_row, off, perm,
                       (const bf16*)src, nseg, dim, nrows);
  else
    hipLaunchKernelGGL(segment_sum_rows_k<float>, dim3(grid), dim3(256), 0, st, dst, seg_row, off, perm,
                       (const float*)src, nseg, dim, nrows);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_sparse_opt(int mode, float* table, float* s1, float* s2, const int64_t* ids,
                             const float* g, int64_t n, int64_t dim, int64_t nrows, float lr,
                             float l2, float mu, float b1, float b2, float b1t, float b2t,
                             float eps, float wd, hipStream_t st) {
  if (n <= 0) return 0;
  dim3 grid(rows_blocks(n));
#define SPC(M) case M: hipLaunchKernelGGL(sparse_opt_k<M>, grid, dim3(256), 0, st, table, s1, s2, ids, g, n, dim, nrows, lr, l2, mu, b1, b2, b1t, b2t, eps, wd); break;
  switch (mode) {
    SPC(SP_SGD) SPC(SP_MOMENTUM) SPC(SP_NESTEROV) SPC(SP_ADAGRAD) SPC(SP_ADAM) SPC(SP_ADAMW)
    default: return (int)hipErrorInvalidValue;
  }
#undef SPC
  HETU_LAUNCH_CHECK();
  return 0;
}
