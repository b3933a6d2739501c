// BatchNorm for channels-last activations ([M, C], M = N*H*W) on gfx950.
//
// Replaces the reference's cuDNN BN path (src/ops/CudnnBn.cu:22-194) with a
// three-kernel schedule per direction, fused with the ops that surround BN in
// ResNet:
//   fwd:  partial stats (Welford-merge) -> finalize (running stats, fold affine
//         into a,b) -> apply y = relu?(x*a + b (+ residual))
//   bwd:  partial sums of dy' and dy'*xhat (dy' = dy masked by y>0 when ReLU was
//         fused) -> finalize (dscale, dbias, fold dx = A*dy' + B*x + C) -> apply
//         (also emits d(residual) = dy' when a residual add was fused).
// Each streaming kernel moves 16 B per lane (8 bf16 or 4 fp32 channels).
#include "common.h"
#include <stdlib.h>

namespace hetu {

// ---------------------------------------------------------------------------
// geometry: a block covers W vector-columns (W*VEC channels) x RP rows/pass.
struct BnGeom {
  int W, RP, tiles, chunks;
  int64_t rows_per_chunk;
};

// launch-shape tunables (hetu_bn_tune; scripts/bench_bn.py sweeps them): target
// partial-statistics blocks per launch, and the block cap of the streaming kernels
static int g_bn_chunk_target = 512;
static int g_bn_apply_blocks = 2048;
// at least this many row passes per thread in the partial kernels: small layers
// (14x14, 7x7) otherwise spread over ~1024 blocks of a dozen rows each, writing
// as many partial sums as they read activations
static int g_bn_min_passes = 16;

static int bn_apply_grid(int64_t nvec, int C, int V) {
  int64_t b = (nvec + 1023) / 1024;
  if (b > g_bn_apply_blocks) b = g_bn_apply_blocks;
  if (b < 1) b = 1;
  const int need = (int)((C / V + 255) / 256);   // channel-stationary kernels need >= C/V threads
  return b < need ? need : (int)b;
}

static BnGeom bn_geom(int64_t M, int C, int vec) {
  BnGeom g;
  int cv = C / vec;
  g.W = cv < 64 ? cv : 64;
  g.RP = 256 / g.W;
  g.tiles = (cv + g.W - 1) / g.W;
  int want = (int)((g_bn_chunk_target + g.tiles - 1) / g.tiles);
  int64_t max_chunks = (M + g.RP - 1) / g.RP;
  const int64_t pass_cap = M / ((int64_t)g.RP * g_bn_min_passes);
  if (max_chunks > pass_cap) max_chunks = pass_cap;
  if (want > max_chunks) want = (int)max_chunks;
  if (want < 1) want = 1;
  g.chunks = want;
  g.rows_per_chunk = (M + g.chunks - 1) / g.chunks;
  return g;
}

// partial statistics: ws_mean/ws_m2 [C][chunks] (raw sums); counts derivable on host side
template <typename T>
__global__ void __launch_bounds__(256) bn_stats_partial(const T* __restrict__ x, int64_t M, int C,
                                                         int W, int RP, int64_t rows_per_chunk,
                                                         float* __restrict__ ws_mean,
                                                         float* __restrict__ ws_m2) {
  constexpr int V = Vec<T>::N;
  __shared__ float sh_s[256 * V];
  __shared__ float sh_q[256 * V];
  const int t = threadIdx.x;
  const int col = t % W, rsub = t / W;
  const int vc = blockIdx.y * W + col;  // vector column
  const bool active = (rsub < RP) && (vc * V < C);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > M) r1 = M;
  float s[V], q[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { s[i] = 0.f; q[i] = 0.f; }
  if (active) {
    int64_t r = r0 + rsub;
    // four rows in flight: a read-only stream needs more bytes outstanding per
    // lane than the two-tensor backward partial; the small 14x14 / 7x7 layers
    // are bound by this latency chain (>= 16 row passes per thread)
    for (; r + 3 * RP < r1; r += 4 * RP) {
      float v[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_vec<T>(x + (r + u * RP) * C + (int64_t)vc * V, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < V; ++i) { s[i] += v[u][i]; q[i] += v[u][i] * v[u][i]; }
    }
    for (; r < r1; r += RP) {
      float v[V];
      load_vec<T>(x + r * C + (int64_t)vc * V, v);
#pragma unroll
      for (int i = 0; i < V; ++i) { s[i] += v[i]; q[i] += v[i] * v[i]; }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) { sh_s[t * V + i] = s[i]; sh_q[t * V + i] = q[i]; }
  __syncthreads();
  // fold the RP row-partials per channel of the tile; a tile holds W*V channels
  // (up to 512 for bf16), more than the 256 threads, so each thread folds
  // every 256th channel
  const int nch = W * V;
  for (int c_local = t; c_local < nch; c_local += 256) {
    const int colw = c_local / V, lane_i = c_local % V;
    float S = 0.f, Q = 0.f;
    for (int rr = 0; rr < RP; ++rr) {
      int tt = rr * W + colw;
      S += sh_s[tt * V + lane_i];
      Q += sh_q[tt * V + lane_i];
    }
    const int c = blockIdx.y * W * V + c_local;
    if (c < C) {  // [C][chunks]: the finalize wave reads one channel contiguously
      ws_mean[(int64_t)c * gridDim.x + blockIdx.x] = S;  // raw per-chunk sums; merged in fp64
      ws_m2[(int64_t)c * gridDim.x + blockIdx.x] = Q;
    }
  }
}

// Merge of the chunk sums in fp64 (mean = S/n, var = Q/n - mean^2); writes
// save_mean/save_invstd, running stats and the folded affine a = scale*invstd,
// b = bias - mean*a.  One wave per channel over its contiguous [chunks] row:
// every lane issues all its loads up front (no serial latency chain).
__global__ void __launch_bounds__(256) bn_stats_finalize(const float* __restrict__ ws_s, const float* __restrict__ ws_q,
                                  int chunks, int64_t rows_per_chunk, int64_t M, int C,
                                  const float* __restrict__ scale, const float* __restrict__ bias,
                                  float* __restrict__ run_mean, float* __restrict__ run_var,
                                  float factor, float eps, float* __restrict__ save_mean,
                                  float* __restrict__ save_invstd, float* __restrict__ fold_a,
                                  float* __restrict__ fold_b) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const float* ps = ws_s + (int64_t)c * chunks;
  const float* pq = ws_q + (int64_t)c * chunks;
  double S = 0.0, Q = 0.0;
#pragma unroll 8
  for (int p = lane; p < chunks; p += 64) {
    S += (double)ps[p];
    Q += (double)pq[p];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    S += __shfl_xor(S, o, 64);
    Q += __shfl_xor(Q, o, 64);
  }
  if (lane == 0) {
    const double n = (double)M;
    const double mean = S / n;
    double var = Q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = rsqrtf((float)var + eps);
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    if (run_mean != nullptr) {
      const float unb = n > 1.0 ? (float)(var * n / (n - 1.0)) : (float)var;
      run_mean[c] = (1.f - factor) * run_mean[c] + factor * (float)mean;
      run_var[c] = (1.f - factor) * run_var[c] + factor * unb;
    }
    const float aa = scale[c] * invstd;
    fold_a[c] = aa;
    fold_b[c] = bias[c] - (float)mean * aa;
  }
}

// Same merge from per-channel totals (sum, sum of squares) accumulated elsewhere: by
// the convolution epilogue that produced x (gemm.hip colstats) or by bn_sums_merge.
// The totals are zeroed once read: a persistent per-layer buffer is ready for the next
// accumulation without a fill launch.
// S, Q = sums over the rep replicas ([rep][2C]) of channel c, then the replicas zeroed: all
// loads first (in flight together), the stores after -- interleaved, each load waited
// behind the previous store
__device__ __forceinline__ void fold_replicas(float* __restrict__ sums, int rep, int C, int c, double& S,
                                              double& Q) {
  int r = 0;
  for (; r + 8 <= rep; r += 8) {
    float a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[k] = sums[(int64_t)(r + k) * 2 * C + c];
      b[k] = sums[(int64_t)(r + k) * 2 * C + C + c];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      S += a[k];
      Q += b[k];
    }
  }
  for (; r < rep; ++r) {
    S += sums[(int64_t)r * 2 * C + c];
    Q += sums[(int64_t)r * 2 * C + C + c];
  }
  for (r = 0; r < rep; ++r) {
    sums[(int64_t)r * 2 * C + c] = 0.f;
    sums[(int64_t)r * 2 * C + C + c] = 0.f;
  }
}

// sums: rep replicas [rep][2C] of the per-channel sum / sum of squares, folded and zeroed
__global__ void __launch_bounds__(256) bn_sums_finalize(float* __restrict__ sums, int rep, int64_t M, int C,
                                 const float* __restrict__ scale, const float* __restrict__ bias,
                                 float* __restrict__ run_mean, float* __restrict__ run_var,
                                 float factor, float eps, float* __restrict__ save_mean,
                                 float* __restrict__ save_invstd, float* __restrict__ fold_a,
                                 float* __restrict__ fold_b) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double n = (double)M;
  double S = 0.0, Q = 0.0;
  fold_replicas(sums, rep, C, c, S, Q);
  const double mean = S / n;
  double var = Q / n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = rsqrtf((float)var + eps);
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  if (run_mean != nullptr) {
    const float unb = n > 1.0 ? (float)(var * n / (n - 1.0)) : (float)var;
    run_mean[c] = (1.f - factor) * run_mean[c] + factor * (float)mean;
    run_var[c] = (1.f - factor) * run_var[c] + factor * unb;
  }
  const float aa = scale[c] * invstd;
  fold_a[c] = aa;
  fold_b[c] = bias[c] - (float)mean * aa;
}

// per-channel totals from the [C][chunks] partials of bn_stats_partial
__global__ void __launch_bounds__(256) bn_sums_merge(const float* __restrict__ ws_s, const float* __restrict__ ws_q,
                                                      int chunks, int C, float* __restrict__ sums) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double S = 0.0, Q = 0.0;
  for (int p = lane; p < chunks; p += 64) {
    S += (double)ws_s[(int64_t)c * chunks + p];
    Q += (double)ws_q[(int64_t)c * chunks + p];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    S += __shfl_xor(S, o, 64);
    Q += __shfl_xor(Q, o, 64);
  }
  if (lane == 0) {
    sums[c] = (float)S;
    sums[C + c] = (float)Q;
  }
}

// sums[c] += total of the [C][chunks] partials (accumulating form of bn_sums_merge)
__global__ void __launch_bounds__(256) bn_sums_add(const float* __restrict__ ws_s, const float* __restrict__ ws_q,
                                                    int chunks, int C, float* __restrict__ sums) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double S = 0.0, Q = 0.0;
  for (int p = lane; p < chunks; p += 64) {
    S += (double)ws_s[(int64_t)c * chunks + p];
    Q += (double)ws_q[(int64_t)c * chunks + p];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    S += __shfl_xor(S, o, 64);
    Q += __shfl_xor(Q, o, 64);
  }
  if (lane == 0) {
    sums[c] += (float)S;
    sums[C + c] += (float)Q;
  }
}

// inference: fold running stats
__global__ void bn_infer_fold(const float* __restrict__ run_mean, const float* __restrict__ run_var,
                              const float* __restrict__ scale, const float* __restrict__ bias, int C,
                              float eps, float* __restrict__ fold_a, float* __restrict__ fold_b) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = scale[c] * rsqrtf(run_var[c] + eps);
  fold_a[c] = a;
  fold_b[c] = bias[c] - run_mean[c] * a;
}

// ReLU keep-bit of each lane of a vector, packed into one byte (bit k = lane k)
template <int V>
__device__ __forceinline__ uint8_t relu_bits(const float (&o)[V]) {
  unsigned m = 0;
#pragma unroll
  for (int k = 0; k < V; ++k) m |= (o[k] > 0.f ? 1u : 0u) << k;
  return (uint8_t)m;
}

// Non-temporal vector loads (default, HETU_BN_NT=0: off): the apply passes read each input byte once
typedef unsigned bn_u4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ void load_vec_nt(const T* p, float (&v)[Vec<T>::N]);
template <>
__device__ __forceinline__ void load_vec_nt<float>(const float* p, float (&v)[4]) {
  const bn_u4 x = __builtin_nontemporal_load(reinterpret_cast<const bn_u4*>(p));
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(x[i]);
}
template <>
__device__ __forceinline__ void load_vec_nt<bf16>(const bf16* p, float (&v)[8]) {
  const bn_u4 x = __builtin_nontemporal_load(reinterpret_cast<const bn_u4*>(p));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(x[i] << 16);
    v[2 * i + 1] = __uint_as_float(x[i] & 0xffff0000u);
  }
}
template <typename T>
__device__ __forceinline__ void ldv(const T* p, float (&v)[Vec<T>::N], int nt) {
  if (nt) load_vec_nt<T>(p, v);
  else load_vec<T>(p, v);
}

// MASK: also store the ReLU keep-bits (1 byte per 16-byte vector, 1/16 of y) so the
// backward of a fused add+ReLU reads them instead of re-reading y
template <typename T, bool RELU, bool RES, bool MASK = false>
__global__ void __launch_bounds__(256) bn_apply(const T* __restrict__ x, const T* __restrict__ res,
                                                 const float* __restrict__ fa,
                                                 const float* __restrict__ fb, T* __restrict__ y,
                                                 int64_t nvec, int C, uint8_t* __restrict__ mask, int nt = 0) {
  // channel-stationary threads: the grid stride is a multiple of C/V, so every
  // thread keeps one channel group's folded affine in registers (no per-element
  // parameter loads, no 64-bit modulo) and streams U vectors per iteration
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const int64_t stride = nth - nth % cv;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= stride) return;
  const int c0 = (int)(tid % cv) * V;
  float a[V], bb[V];
#pragma unroll
  for (int k = 0; k < V; ++k) { a[k] = fa[c0 + k]; bb[k] = fb[c0 + k]; }
  // U vectors in flight per lane: 4 without a residual stream, 2 with one (4 loads either way)
  constexpr int U = RES ? 2 : 4;
  int64_t i = tid;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    float v[U][V], r[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) ldv<T>(x + (i + u * stride) * V, v[u], nt);
    if (RES) {
#pragma unroll
      for (int u = 0; u < U; ++u) ldv<T>(res + (i + u * stride) * V, r[u], nt);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        float o = v[u][k] * a[k] + bb[k];
        if (RES) o += r[u][k];
        if (RELU) o = fmaxf(o, 0.f);
        v[u][k] = o;
      }
      store_vec<T>(y + (i + u * stride) * V, v[u]);
      if (MASK) mask[i + u * stride] = relu_bits<V>(v[u]);
    }
  }
  for (; i < nvec; i += stride) {
    float v[V], r[V];
    ldv<T>(x + i * V, v, nt);
    if (RES) ldv<T>(res + i * V, r, nt);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float o = v[k] * a[k] + bb[k];
      if (RES) o += r[k];
      if (RELU) o = fmaxf(o, 0.f);
      v[k] = o;
    }
    store_vec<T>(y + i * V, v);
    if (MASK) mask[i] = relu_bits<V>(v);
  }
}

// ---------------------------------------------------------------------------
// backward
// RELU == 2: the ReLU mask is recomputed from x and the forward affine
// a = scale*invstd, b = bias - mean*a (folded per thread, no separate fold launch)
// RELU == 3: the ReLU mask is the forward's keep-bit byte per vector (``mask``)
template <typename T, int RELU>
__global__ void __launch_bounds__(256) bn_bwd_partial(const T* __restrict__ dy, const T* __restrict__ y,
                                                       const uint8_t* __restrict__ mask,
                                                       const T* __restrict__ x,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ fscale,
                                                       const float* __restrict__ fbias, int64_t M,
                                                       int C, int W, int RP, int64_t rows_per_chunk,
                                                       float* __restrict__ ws_sdy,
                                                       float* __restrict__ ws_sdyx) {
  constexpr int V = Vec<T>::N;
  __shared__ float sh_s[256 * V];
  __shared__ float sh_q[256 * V];
  const int t = threadIdx.x;
  const int col = t % W, rsub = t / W;
  const int vc = blockIdx.y * W + col;
  const bool active = (rsub < RP) && (vc * V < C);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > M) r1 = M;
  float s[V], q[V], mu[V], is[V], ka[V], kb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { s[i] = 0.f; q[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      // null mean / invstd: sums of dy' * x instead of dy' * xhat (hetu_bn_bwd_sums)
      mu[i] = mean ? mean[vc * V + i] : 0.f;
      is[i] = invstd ? invstd[vc * V + i] : 1.f;
      if (RELU == 2) { ka[i] = fscale[vc * V + i] * is[i]; kb[i] = fbias[vc * V + i] - mu[i] * ka[i]; }
    }
    // two rows (four vectors) in flight per iteration (all loads issued before any use)
    int64_t r = r0 + rsub;
    for (; r + RP < r1; r += 2 * RP) {
      const int64_t off = r * C + (int64_t)vc * V, off2 = off + (int64_t)RP * C;
      float g[V], xv[V], g2[V], xv2[V], yv[V], yv2[V];
      load_vec<T>(dy + off, g);
      load_vec<T>(x + off, xv);
      load_vec<T>(dy + off2, g2);
      load_vec<T>(x + off2, xv2);
      if (RELU == 1) {
        load_vec<T>(y + off, yv);
        load_vec<T>(y + off2, yv2);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          g[i] = yv[i] > 0.f ? g[i] : 0.f;
          g2[i] = yv2[i] > 0.f ? g2[i] : 0.f;
        }
      } else if (RELU == 2) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          g[i] = (xv[i] * ka[i] + kb[i]) > 0.f ? g[i] : 0.f;
          g2[i] = (xv2[i] * ka[i] + kb[i]) > 0.f ? g2[i] : 0.f;
        }
      } else if (RELU == 3) {
        const unsigned m1 = mask[off / V], m2 = mask[off2 / V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
          g[i] = (m1 >> i) & 1u ? g[i] : 0.f;
          g2[i] = (m2 >> i) & 1u ? g2[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < V; ++i) {
        s[i] += g[i] + g2[i];
        q[i] += (g[i] * (xv[i] - mu[i]) + g2[i] * (xv2[i] - mu[i])) * is[i];
      }
    }
    for (; r < r1; r += RP) {
      const int64_t off = r * C + (int64_t)vc * V;
      float g[V], xv[V];
      load_vec<T>(dy + off, g);
      load_vec<T>(x + off, xv);
      if (RELU == 1) {
        float yv[V];
        load_vec<T>(y + off, yv);
#pragma unroll
        for (int i = 0; i < V; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
      } else if (RELU == 2) {
#pragma unroll
        for (int i = 0; i < V; ++i) g[i] = (xv[i] * ka[i] + kb[i]) > 0.f ? g[i] : 0.f;
      } else if (RELU == 3) {
        const unsigned m1 = mask[off / V];
#pragma unroll
        for (int i = 0; i < V; ++i) g[i] = (m1 >> i) & 1u ? g[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < V; ++i) {
        s[i] += g[i];
        q[i] += g[i] * (xv[i] - mu[i]) * is[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) { sh_s[t * V + i] = s[i]; sh_q[t * V + i] = q[i]; }
  __syncthreads();
  const int nch = W * V;   // up to 512 channels per tile (bf16): 2 per thread
  for (int c_local = t; c_local < nch; c_local += 256) {
    const int colw = c_local / V, lane_i = c_local % V;
    float S = 0.f, Q = 0.f;
    for (int rr = 0; rr < RP; ++rr) {
      int tt = rr * W + colw;
      S += sh_s[tt * V + lane_i];
      Q += sh_q[tt * V + lane_i];
    }
    const int c = blockIdx.y * W * V + c_local;
    if (c < C) {
      ws_sdy[(int64_t)c * gridDim.x + blockIdx.x] = S;
      ws_sdyx[(int64_t)c * gridDim.x + blockIdx.x] = Q;
    }
  }
}

__global__ void __launch_bounds__(256) bn_bwd_finalize(const float* __restrict__ ws_sdy, const float* __restrict__ ws_sdyx,
                                int chunks, int64_t M, int C, const float* __restrict__ scale,
                                const float* __restrict__ mean, const float* __restrict__ invstd,
                                float* __restrict__ dscale, float* __restrict__ dbias,
                                float* __restrict__ cA, float* __restrict__ cB,
                                float* __restrict__ cC) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const float* p1 = ws_sdy + (int64_t)c * chunks;
  const float* p2 = ws_sdyx + (int64_t)c * chunks;
  float sdy = 0.f, sdyx = 0.f;
#pragma unroll 8
  for (int p = lane; p < chunks; p += 64) {
    sdy += p1[p];
    sdyx += p2[p];
  }
  sdy = wave_sum(sdy);
  sdyx = wave_sum(sdyx);
  if (lane == 0) {
    if (dscale) dscale[c] = sdyx;
    if (dbias) dbias[c] = sdy;
    const float invM = 1.f / (float)M;
    const float is = invstd[c];
    const float k1 = scale[c] * is;
    const float B = -k1 * is * sdyx * invM;
    cA[c] = k1;
    cB[c] = B;
    cC[c] = -k1 * sdy * invM - mean[c] * B;
  }
}

// bn_bwd_finalize from per-channel totals S = sum(dy'), Qx = sum(dy' * x) accumulated by
// the data-gradient epilogue that produced dy (gemm_core.h Epi::bnx):
// sum(dy' * xhat) = invstd * (Qx - mean * S).  The totals are zeroed once read.
// sums: rep replicas [rep][2C] (see gemm_core.h Epi::cs_rep), folded here and all zeroed
__global__ void __launch_bounds__(256) bn_bwd_sums_finalize(float* __restrict__ sums, int rep, int64_t M, int C,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           float* __restrict__ dscale, float* __restrict__ dbias,
                                                           float* __restrict__ cA, float* __restrict__ cB,
                                                           float* __restrict__ cC) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double S = 0.0, Q = 0.0;
  fold_replicas(sums, rep, C, c, S, Q);
  const float sdy = (float)S;
  const float is = invstd[c];
  const float sdyx = (float)((double)is * (Q - (double)mean[c] * S));
  if (dscale) dscale[c] = sdyx;
  if (dbias) dbias[c] = sdy;
  const float invM = 1.f / (float)M;
  const float k1 = scale[c] * is;
  const float B = -k1 * is * sdyx * invM;
  cA[c] = k1;
  cB[c] = B;
  cC[c] = -k1 * sdy * invM - mean[c] * B;
}

// SUMS: the coefficients come straight from the epilogue totals (sums = S, Qx per
// channel; see bn_bwd_sums_finalize) -- no finalize launch: every thread folds its own
// channels, the first thread of each channel group writes dscale / dbias and clears that
// group in ``znext`` (the other half of the double-buffered totals, consumed one call ago)
struct BnSums {
  const float* sums;
  float* znext;
  float* dscale;
  float* dbias;
  const float* scale;
  int64_t M;
};

template <typename T, int RELU, bool DRES, bool SUMS = false>
__global__ void __launch_bounds__(256) bn_bwd_apply(const T* __restrict__ dy, const T* __restrict__ y,
                                                     const uint8_t* __restrict__ mask,
                                                     const T* __restrict__ x,
                                                     const float* __restrict__ cA,
                                                     const float* __restrict__ cB,
                                                     const float* __restrict__ cC,
                                                     const float* __restrict__ fscale,
                                                     const float* __restrict__ fbias,
                                                     const float* __restrict__ fmean,
                                                     const float* __restrict__ finvstd,
                                                     T* __restrict__ dx, T* __restrict__ dres,
                                                     int64_t nvec, int C, BnSums bs = BnSums{}, int nt = 0) {
  // channel-stationary threads (see bn_apply): per-channel coefficients live in
  // registers for the whole grid-stride loop
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const int64_t stride = nth - nth % cv;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= stride) return;
  const int c0 = (int)(tid % cv) * V;
  float A[V], Bc[V], Cc[V], ka[V], kb[V];
  if (SUMS) {
    const double invM = 1.0 / (double)bs.M;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int c = c0 + k;
      const double S = bs.sums[c], mu = fmean[c], is = finvstd[c];
      const double sdyx = is * ((double)bs.sums[C + c] - mu * S);
      const double k1 = (double)bs.scale[c] * is;
      const double B = -k1 * is * sdyx * invM;
      A[k] = (float)k1;
      Bc[k] = (float)B;
      Cc[k] = (float)(-k1 * S * invM - mu * B);
      if (tid < cv) {
        if (bs.dscale) bs.dscale[c] = (float)sdyx;
        if (bs.dbias) bs.dbias[c] = (float)S;
        if (bs.znext) {
          bs.znext[c] = 0.f;
          bs.znext[C + c] = 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    if (!SUMS) { A[k] = cA[c0 + k]; Bc[k] = cB[c0 + k]; Cc[k] = cC[c0 + k]; }
    if (RELU == 2) {
      ka[k] = fscale[c0 + k] * finvstd[c0 + k];
      kb[k] = fbias[c0 + k] - fmean[c0 + k] * ka[k];
    }
  }
  int64_t i = tid;
  for (; i + stride < nvec; i += 2 * stride) {   // two vectors in flight
    const int64_t j = i + stride;
    float g[V], xv[V], g2[V], xv2[V], yv[V], yv2[V];
    ldv<T>(dy + i * V, g, nt);
    ldv<T>(x + i * V, xv, nt);
    ldv<T>(dy + j * V, g2, nt);
    ldv<T>(x + j * V, xv2, nt);
    if (RELU == 1) {
      ldv<T>(y + i * V, yv, nt);
      ldv<T>(y + j * V, yv2, nt);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        g[k] = yv[k] > 0.f ? g[k] : 0.f;
        g2[k] = yv2[k] > 0.f ? g2[k] : 0.f;
      }
    } else if (RELU == 2) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        g[k] = (xv[k] * ka[k] + kb[k]) > 0.f ? g[k] : 0.f;
        g2[k] = (xv2[k] * ka[k] + kb[k]) > 0.f ? g2[k] : 0.f;
      }
    } else if (RELU == 3) {
      const unsigned m1 = mask[i], m2 = mask[j];
#pragma unroll
      for (int k = 0; k < V; ++k) {
        g[k] = (m1 >> k) & 1u ? g[k] : 0.f;
        g2[k] = (m2 >> k) & 1u ? g2[k] : 0.f;
      }
    }
    if (DRES) {
      store_vec<T>(dres + i * V, g);
      store_vec<T>(dres + j * V, g2);
    }
    float o[V], o2[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      o[k] = A[k] * g[k] + Bc[k] * xv[k] + Cc[k];
      o2[k] = A[k] * g2[k] + Bc[k] * xv2[k] + Cc[k];
    }
    store_vec<T>(dx + i * V, o);
    store_vec<T>(dx + j * V, o2);
  }
  for (; i < nvec; i += stride) {
    float g[V], xv[V];
    ldv<T>(dy + i * V, g, nt);
    ldv<T>(x + i * V, xv, nt);
    if (RELU == 1) {
      float yv[V];
      ldv<T>(y + i * V, yv, nt);
#pragma unroll
      for (int k = 0; k < V; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
    } else if (RELU == 2) {
#pragma unroll
      for (int k = 0; k < V; ++k) g[k] = (xv[k] * ka[k] + kb[k]) > 0.f ? g[k] : 0.f;
    } else if (RELU == 3) {
      const unsigned m1 = mask[i];
#pragma unroll
      for (int k = 0; k < V; ++k) g[k] = (m1 >> k) & 1u ? g[k] : 0.f;
    }
    if (DRES) store_vec<T>(dres + i * V, g);
    float o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = A[k] * g[k] + Bc[k] * xv[k] + Cc[k];
    store_vec<T>(dx + i * V, o);
  }
}

}  // namespace hetu

using namespace hetu;

// Non-temporal input loads in the BatchNorm apply passes (default; HETU_BN_NT=0 turns them
// off): ResNet-50 10 663 / 10 704 vs 10 439 / 10 446 img/s interleaved on one box
// (profiles/bn_nt_ab_r5.txt)
static int bn_nt() {
  static const int v = [] {
    const char* e = getenv("HETU_BN_NT");
    return e != nullptr && e[0] == '0' ? 0 : 1;
  }();
  return v;
}

HETU_API void hetu_bn_tune(int chunk_target, int apply_blocks, int min_passes) {
  if (chunk_target > 0) g_bn_chunk_target = chunk_target;
  if (apply_blocks > 0) g_bn_apply_blocks = apply_blocks;
  if (min_passes > 0) g_bn_min_passes = min_passes;
}

// workspace floats needed: 2 * chunks * C + 5 * C  (partials + fold/bwd coefficients)
HETU_API int64_t hetu_bn_workspace_floats(int64_t M, int C, int is_bf16) {
  BnGeom g = bn_geom(M, C, is_bf16 ? 8 : 4);
  return 2 * (int64_t)g.chunks * C + 5 * (int64_t)C;
}

template <typename T>
static int bn_fwd_impl(const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
                       const float* bias, float* run_mean, float* run_var, float factor, float eps,
                       float* save_mean, float* save_invstd, float* ws, int relu, int training,
                       float* sums, uint8_t* mask, int srep, hipStream_t st) {
  constexpr int V = Vec<T>::N;
  if (C % V != 0) return (int)hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C, V);
  float* fa = ws + 2 * (int64_t)g.chunks * C;
  float* fb = fa + C;
  if (training && sums) {   // statistics already reduced (fused into the producer)
    hipLaunchKernelGGL(bn_sums_finalize, dim3((C + 255) / 256), dim3(256), 0, st, sums, max(srep, 1), M, C, scale,
                       bias, run_mean, run_var, factor, eps, save_mean, save_invstd, fa, fb);
  } else if (training) {
    float* wm = ws;
    float* wq = ws + (int64_t)g.chunks * C;
    hipLaunchKernelGGL(bn_stats_partial<T>, dim3(g.chunks, g.tiles), dim3(256), 0, st,
                       (const T*)x, M, C, g.W, g.RP, g.rows_per_chunk, wm, wq);
    hipLaunchKernelGGL(bn_stats_finalize, dim3((C + 3) / 4), dim3(256), 0, st, wm, wq,
                       g.chunks, g.rows_per_chunk, M, C, scale, bias, run_mean, run_var, factor,
                       eps, save_mean, save_invstd, fa, fb);
  } else {
    hipLaunchKernelGGL(bn_infer_fold, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var,
                       scale, bias, C, eps, fa, fb);
  }
  int64_t nvec = M * C / V;
  const int grid = bn_apply_grid(nvec, C, V);
  const T* xr = (const T*)x;
  const T* rr = (const T*)res;
  T* yr = (T*)y;
  if (relu && res && mask)
    hipLaunchKernelGGL((bn_apply<T, true, true, true>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  else if (relu && res)
    hipLaunchKernelGGL((bn_apply<T, true, true>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  else if (relu && mask)
    hipLaunchKernelGGL((bn_apply<T, true, false, true>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  else if (relu)
    hipLaunchKernelGGL((bn_apply<T, true, false>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  else if (res)
    hipLaunchKernelGGL((bn_apply<T, false, true>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  else
    hipLaunchKernelGGL((bn_apply<T, false, false>), dim3(grid), dim3(256), 0, st, xr, rr, fa, fb, yr, nvec, C, mask, bn_nt());
  HETU_LAUNCH_CHECK();
  return 0;
}

// x,y,res: [M,C] channels-last; res may be null; run_* may be null (no update);
// mask (relu only, may be null): [M*C/V] bytes of ReLU keep-bits (V = 8 bf16 / 4 fp32)
HETU_API int hetu_bn_fwd(const void* x, const void* res, void* y, int64_t M, int C, int is_bf16,
                         const float* scale, const float* bias, float* run_mean, float* run_var,
                         float factor, float eps, float* save_mean, float* save_invstd, float* ws,
                         int relu, int training, float* sums, uint8_t* mask, int srep, hipStream_t st) {
  if (is_bf16)
    return bn_fwd_impl<bf16>(x, res, y, M, C, scale, bias, run_mean, run_var, factor, eps,
                             save_mean, save_invstd, ws, relu, training, sums, mask, srep, st);
  return bn_fwd_impl<float>(x, res, y, M, C, scale, bias, run_mean, run_var, factor, eps,
                            save_mean, save_invstd, ws, relu, training, sums, mask, srep, st);
}

// sums[0..C) / sums[C..2C) = per-channel sum / sum of squares of x [M, C] (fp64 merge)
HETU_API int hetu_col_sums(const void* x, int64_t M, int C, int is_bf16, float* ws, float* sums,
                           hipStream_t st) {
  const int V = is_bf16 ? 8 : 4;
  if (C % V != 0) return (int)hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C, V);
  float* wm = ws;
  float* wq = ws + (int64_t)g.chunks * C;
  if (is_bf16)
    hipLaunchKernelGGL(bn_stats_partial<bf16>, dim3(g.chunks, g.tiles), dim3(256), 0, st, (const bf16*)x,
                       M, C, g.W, g.RP, g.rows_per_chunk, wm, wq);
  else
    hipLaunchKernelGGL(bn_stats_partial<float>, dim3(g.chunks, g.tiles), dim3(256), 0, st, (const float*)x,
                       M, C, g.W, g.RP, g.rows_per_chunk, wm, wq);
  hipLaunchKernelGGL(bn_sums_merge, dim3((C + 3) / 4), dim3(256), 0, st, wm, wq, g.chunks, C, sums);
  HETU_LAUNCH_CHECK();
  return 0;
}

template <typename T, int RELU>
static void bn_bwd_launch(const BnGeom& g, const T* dy, const T* y, const uint8_t* mask, const T* x, T* dx, T* dres,
                          int64_t M, int C, const float* mean, const float* invstd,
                          const float* bias, float* w1, float* w2, float* cA,
                          float* cB, float* cC, const float* scale, float* dscale, float* dbias,
                          float* bsums, float* bnext, int brep, hipStream_t st) {
  constexpr int V = Vec<T>::N;
  if (bsums && bnext && brep <= 1) {   // coefficients folded in the apply kernel itself
    int64_t nvec = M * C / V;
    const int grid = bn_apply_grid(nvec, C, V);
    BnSums bs{bsums, bnext, dscale, dbias, scale, M};
    if (dres)
      hipLaunchKernelGGL((bn_bwd_apply<T, RELU, true, true>), dim3(grid), dim3(256), 0, st, dy, y, mask, x, cA, cB, cC,
                         scale, bias, mean, invstd, dx, dres, nvec, C, bs, bn_nt());
    else
      hipLaunchKernelGGL((bn_bwd_apply<T, RELU, false, true>), dim3(grid), dim3(256), 0, st, dy, y, mask, x, cA, cB,
                         cC, scale, bias, mean, invstd, dx, dres, nvec, C, bs, bn_nt());
    return;
  }
  if (bsums) {
    hipLaunchKernelGGL(bn_bwd_sums_finalize, dim3((C + 255) / 256), dim3(256), 0, st, bsums, max(brep, 1), M, C,
                       scale, mean, invstd, dscale, dbias, cA, cB, cC);
  } else {
    hipLaunchKernelGGL((bn_bwd_partial<T, RELU>), dim3(g.chunks, g.tiles), dim3(256), 0, st, dy, y, mask, x,
                       mean, invstd, scale, bias, M, C, g.W, g.RP, g.rows_per_chunk, w1, w2);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + 3) / 4), dim3(256), 0, st, w1, w2, g.chunks, M,
                       C, scale, mean, invstd, dscale, dbias, cA, cB, cC);
  }
  int64_t nvec = M * C / V;
  const int grid = bn_apply_grid(nvec, C, V);
  if (dres)
    hipLaunchKernelGGL((bn_bwd_apply<T, RELU, true>), dim3(grid), dim3(256), 0, st, dy, y, mask, x, cA, cB, cC, scale,
                       bias, mean, invstd, dx, dres, nvec, C, BnSums{}, bn_nt());
  else
    hipLaunchKernelGGL((bn_bwd_apply<T, RELU, false>), dim3(grid), dim3(256), 0, st, dy, y, mask, x, cA, cB, cC, scale,
                       bias, mean, invstd, dx, dres, nvec, C, BnSums{}, bn_nt());
}

template <typename T>
static int bn_bwd_impl(const void* dy, const void* y, const uint8_t* mask, const void* x, void* dx, void* dres,
                       int64_t M, int C, const float* scale, const float* bias, const float* mean,
                       const float* invstd, float* dscale, float* dbias, float* ws, int relu,
                       float* bsums, float* bnext, int brep, hipStream_t st) {
  constexpr int V = Vec<T>::N;
  if (C % V != 0) return (int)hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C, V);
  float* w1 = ws;
  float* w2 = ws + (int64_t)g.chunks * C;
  float* cA = ws + 2 * (int64_t)g.chunks * C;
  float* cB = cA + C;
  float* cC = cB + C;
  const T *dyr = (const T*)dy, *yr = (const T*)y, *xr = (const T*)x;
  T *dxr = (T*)dx, *drr = (T*)dres;
  // mask source: the saved output y when a residual was added (mask depends on it),
  // otherwise recomputed from x and the folded forward affine (one less stream)
  // (or, with the forward's keep-bit mask, from that: 1/16 of the bytes of y)
  int mode = !relu ? 0 : (mask ? 3 : ((dres || !bias) ? 1 : 2));
  if (mode == 0) bn_bwd_launch<T, 0>(g, dyr, yr, mask, xr, dxr, drr, M, C, mean, invstd, bias, w1, w2, cA, cB, cC, scale, dscale, dbias, bsums, bnext, brep, st);
  else if (mode == 1) bn_bwd_launch<T, 1>(g, dyr, yr, mask, xr, dxr, drr, M, C, mean, invstd, bias, w1, w2, cA, cB, cC, scale, dscale, dbias, bsums, bnext, brep, st);
  else if (mode == 2) bn_bwd_launch<T, 2>(g, dyr, yr, mask, xr, dxr, drr, M, C, mean, invstd, bias, w1, w2, cA, cB, cC, scale, dscale, dbias, bsums, bnext, brep, st);
  else bn_bwd_launch<T, 3>(g, dyr, yr, mask, xr, dxr, drr, M, C, mean, invstd, bias, w1, w2, cA, cB, cC, scale, dscale, dbias, bsums, bnext, brep, st);
  HETU_LAUNCH_CHECK();
  return 0;
}

// dy,y,x,dx,dres: [M,C]; y only read when relu (and no mask); dres may be null
// bias may be null (then the ReLU mask is read from y); mask: hetu_bn_fwd's keep-bits.
// bsums (nullable): [2C] totals sum(dy'), sum(dy' * x) already accumulated (by the
// epilogue that produced dy, or hetu_bn_bwd_sums): the reduction pass is skipped and the
// totals are zeroed.  bnext (nullable): the other half of double-buffered totals -- the
// apply kernel then folds the coefficients itself (no finalize launch) and clears bnext
// instead of bsums.  brep: bsums holds that many replicas [brep][2C] (epilogue blocks spread
// their atomics over them), folded by the finalize kernel (bnext is then not used)
HETU_API int hetu_bn_bwd(const void* dy, const void* y, const void* x, void* dx, void* dres,
                         int64_t M, int C, int is_bf16, const float* scale, const float* bias,
                         const float* mean, const float* invstd, float* dscale, float* dbias,
                         float* ws, int relu, const uint8_t* mask, float* bsums, float* bnext, int brep,
                         hipStream_t st) {
  if (is_bf16)
    return bn_bwd_impl<bf16>(dy, y, mask, x, dx, dres, M, C, scale, bias, mean, invstd, dscale, dbias, ws, relu,
                             bsums, bnext, brep, st);
  return bn_bwd_impl<float>(dy, y, mask, x, dx, dres, M, C, scale, bias, mean, invstd, dscale, dbias, ws, relu,
                            bsums, bnext, brep, st);
}

// sums[0..C) += sum(dy'), sums[C..2C) += sum(dy' * x) over [M, C] bf16 rows, dy' = dy masked
// by the ReLU keep-bits (nullable): the epilogue-fused reduction, as a pass of its own for
// data gradients that come from a library kernel.  ws: hetu_bn_workspace_floats.
HETU_API int hetu_bn_bwd_sums(const void* dy, const void* x, const uint8_t* mask, int64_t M, int C, float* ws,
                              float* sums, hipStream_t st) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C, 8);
  float* w1 = ws;
  float* w2 = ws + (int64_t)g.chunks * C;
  if (mask)
    hipLaunchKernelGGL((bn_bwd_partial<bf16, 3>), dim3(g.chunks, g.tiles), dim3(256), 0, st, (const bf16*)dy,
                       (const bf16*)nullptr, mask, (const bf16*)x, (const float*)nullptr, (const float*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, M, C, g.W, g.RP, g.rows_per_chunk, w1, w2);
  else
    hipLaunchKernelGGL((bn_bwd_partial<bf16, 0>), dim3(g.chunks, g.tiles), dim3(256), 0, st, (const bf16*)dy,
                       (const bf16*)nullptr, mask, (const bf16*)x, (const float*)nullptr, (const float*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, M, C, g.W, g.RP, g.rows_per_chunk, w1, w2);
  hipLaunchKernelGGL(bn_sums_add, dim3((C + 3) / 4), dim3(256), 0, st, w1, w2, g.chunks, C, sums);
  HETU_LAUNCH_CHECK();
  return 0;
}
