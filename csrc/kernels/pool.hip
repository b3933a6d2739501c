// Pooling and axis reductions for channels-last tensors on gfx950.
//
// Replaces MaxPool.cu / AvgPool.cu / CudnnMaxPool.cu / CudnnAvgPool.cu (NCHW,
// one thread per output, backward with atomics) and ReduceSumAxisZero.cu /
// ReduceSum.cu / Conv2dReduceSum.cu (per-call cudaMalloc + H2D metadata).
//   * max-pool fwd stores the winning tap (uint8) so the backward is a
//     deterministic GATHER: each input element sums the <= ceil(k/s)^2 windows
//     that selected it -- no atomics.
//   * avg-pool fwd/bwd likewise gather-based.
//   * reduce_mid: y[b, c] = scale * sum_r x[b, r, c] covers bias gradients
//     (B = 1), global average pooling (R = H*W) and reduce-over-axis-0; long R is
//     split across workgroups with fp32 partial slabs and a second pass.
#include "common.h"

namespace hetu {

template <typename T>
__global__ void __launch_bounds__(256) maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                      uint8_t* __restrict__ idx, int N, int H, int W,
                                                      int C, int Ho, int Wo, int kh, int kw, int sh,
                                                      int sw, int ph, int pw) {
  const int64_t total = (int64_t)N * Ho * Wo * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int wo = (int)(t % Wo); t /= Wo;
    int ho = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int a = 0; a < kh; ++a) {
      int h = ho * sh - ph + a;
      if (h < 0 || h >= H) continue;
      for (int b = 0; b < kw; ++b) {
        int w = wo * sw - pw + b;
        if (w < 0 || w >= W) continue;
        float v = to_f(x[(((int64_t)n * H + h) * W + w) * C + c]);
        if (v > best) { best = v; bi = a * kw + b; }
      }
    }
    y[i] = from_f<T>(best);
    if (idx) idx[i] = (uint8_t)bi;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      T* __restrict__ dx, int N, int H, int W, int C,
                                                      int Ho, int Wo, int kh, int kw, int sh, int sw,
                                                      int ph, int pw) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int w = (int)(t % W); t /= W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    int ho0 = (h + ph - kh + sh) / sh; if (h + ph - kh + 1 < 0) ho0 = 0;
    int ho1 = (h + ph) / sh; if (ho1 >= Ho) ho1 = Ho - 1;
    int wo0 = (w + pw - kw + sw) / sw; if (w + pw - kw + 1 < 0) wo0 = 0;
    int wo1 = (w + pw) / sw; if (wo1 >= Wo) wo1 = Wo - 1;
    float acc = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho) {
      int a = h + ph - ho * sh;
      if (a < 0 || a >= kh) continue;
      for (int wo = wo0; wo <= wo1; ++wo) {
        int b = w + pw - wo * sw;
        if (b < 0 || b >= kw) continue;
        int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C + c;
        if (idx[o] == (uint8_t)(a * kw + b)) acc += to_f(dy[o]);
      }
    }
    dx[i] = from_f<T>(acc);
  }
}


// Vectorized channels-last variants: one thread owns V = 16/sizeof(T) channels of
// one pixel (16-byte loads/stores, 8-byte winning-tap words); 32-bit index math.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_fwd_vec(const T* __restrict__ x, T* __restrict__ y,
                                                        uint8_t* __restrict__ idx, int N, int H, int W,
                                                        int C, int Ho, int Wo, int kh, int kw, int sh,
                                                        int sw, int ph, int pw) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int total = N * Ho * Wo * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cg = i % cv;
    int t = i / cv;
    const int wo = t % Wo;
    t /= Wo;
    const int ho = t % Ho;
    const int n = t / Ho;
    float best[V];
    uint8_t bi[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int a = 0; a < kh; ++a) {
      const int h = ho * sh - ph + a;
      if (h < 0 || h >= H) continue;
      for (int b = 0; b < kw; ++b) {
        const int w = wo * sw - pw + b;
        if (w < 0 || w >= W) continue;
        float v[V];
        load_vec<T>(x + ((int64_t)(n * H + h) * W + w) * C + cg * V, v);
        const uint8_t tap = (uint8_t)(a * kw + b);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (v[k] > best[k]) { best[k] = v[k]; bi[k] = tap; }
      }
    }
    store_vec<T>(y + (int64_t)i * V, best);
    if (idx) {
      if (V == 8) {
        uint2 pk;
        pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
        pk.y = bi[4 % V] | (bi[5 % V] << 8) | (bi[6 % V] << 16) | ((uint32_t)bi[7 % V] << 24);
        *reinterpret_cast<uint2*>(idx + (int64_t)i * V) = pk;
      } else {
        *reinterpret_cast<uint32_t*>(idx + (int64_t)i * V) =
            bi[0] | (bi[1 % V] << 8) | (bi[2 % V] << 16) | ((uint32_t)bi[3 % V] << 24);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_vec(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                        T* __restrict__ dx, int N, int H, int W, int C,
                                                        int Ho, int Wo, int kh, int kw, int sh, int sw,
                                                        int ph, int pw) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int total = N * H * W * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cg = i % cv;
    int t = i / cv;
    const int w = t % W;
    t /= W;
    const int h = t % H;
    const int n = t / H;
    int ho0 = (h + ph - kh + sh) / sh; if (h + ph - kh + 1 < 0) ho0 = 0;
    int ho1 = (h + ph) / sh; if (ho1 >= Ho) ho1 = Ho - 1;
    int wo0 = (w + pw - kw + sw) / sw; if (w + pw - kw + 1 < 0) wo0 = 0;
    int wo1 = (w + pw) / sw; if (wo1 >= Wo) wo1 = Wo - 1;
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    if (kh <= sh + 1 && kw <= sw + 1) {
      // at most 2 x 2 windows hold this pixel (ResNet's 3x3 / stride-2 pool): every
      // candidate's winning-tap word and gradient are requested before any is used
      // (the loop form waits one round trip per window)
      uint2 pk[4];
      float g[4][V];
      int tp[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ho = ho0 + (q >> 1), wo = wo0 + (q & 1);
        const int a = h + ph - ho * sh, b = w + pw - wo * sw;
        const bool ok = ho <= ho1 && wo <= wo1 && a >= 0 && a < kh && b >= 0 && b < kw;
        tp[q] = ok ? a * kw + b : -1;
        const int64_t o = ok ? ((int64_t)(n * Ho + ho) * Wo + wo) * C + cg * V : 0;
        if (V == 8) {
          pk[q] = ok ? *reinterpret_cast<const uint2*>(idx + o) : make_uint2(0, 0);
        } else {
          pk[q] = make_uint2(ok ? *reinterpret_cast<const uint32_t*>(idx + o) : 0u, 0u);
        }
        if (ok) {
          load_vec<T>(dy + o, g[q]);
        } else {
#pragma unroll
          for (int k = 0; k < V; ++k) g[q][k] = 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const uint32_t word = k < 4 ? pk[q].x : pk[q].y;
          const int ix = (int)((word >> (8 * (k & 3))) & 255u);
          if (ix == tp[q]) acc[k] += g[q][k];
        }
      }
      store_vec<T>(dx + (int64_t)i * V, acc);
      continue;
    }
    for (int ho = ho0; ho <= ho1; ++ho) {
      const int a = h + ph - ho * sh;
      if (a < 0 || a >= kh) continue;
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int b = w + pw - wo * sw;
        if (b < 0 || b >= kw) continue;
        const int64_t o = ((int64_t)(n * Ho + ho) * Wo + wo) * C + cg * V;
        const uint8_t tap = (uint8_t)(a * kw + b);
        uint8_t ix[V];
        if (V == 8) {
          uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
#pragma unroll
          for (int k = 0; k < 4; ++k) { ix[k] = (pk.x >> (8 * k)) & 255; ix[(4 + k) % V] = (pk.y >> (8 * k)) & 255; }
        } else {
          uint32_t pk = *reinterpret_cast<const uint32_t*>(idx + o);
#pragma unroll
          for (int k = 0; k < V; ++k) ix[k] = (pk >> (8 * k)) & 255;
        }
        float g[V];
        load_vec<T>(dy + o, g);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (ix[k] == tap) acc[k] += g[k];
      }
    }
    store_vec<T>(dx + (int64_t)i * V, acc);
  }
}

// The same backward for pools where at most 2 x 2 windows hold a pixel, one block per input
// row (n, h): the row's output-window range is block-uniform and each thread keeps one
// channel group, stepping over w -- the flat form's six integer divisions per 16-byte
// output (index decomposition) made it ALU-bound (254 us at ResNet-50's 112 x 112 x 64 x 256).
// Requires 256 % (C / V) == 0.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_rows(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                         T* __restrict__ dx, int H, int W, int C, int Ho, int Wo,
                                                         int kh, int kw, int sh, int sw, int ph, int pw) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int h = blockIdx.x, n = blockIdx.y;
  int ho0 = (h + ph - kh + sh) / sh; if (h + ph - kh + 1 < 0) ho0 = 0;
  int ho1 = (h + ph) / sh; if (ho1 >= Ho) ho1 = Ho - 1;
  const int cg = threadIdx.x % cv, wstep = 256 / cv;
  T* drow = dx + ((int64_t)n * H + h) * W * C + cg * V;
  for (int w = threadIdx.x / cv; w < W; w += wstep) {
    int wo0 = (w + pw - kw + sw) / sw; if (w + pw - kw + 1 < 0) wo0 = 0;
    int wo1 = (w + pw) / sw; if (wo1 >= Wo) wo1 = Wo - 1;
    uint2 pk[4];
    float g[4][V];
    int tp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ho = ho0 + (q >> 1), wo = wo0 + (q & 1);
      const int a = h + ph - ho * sh, b = w + pw - wo * sw;
      const bool ok = ho <= ho1 && wo <= wo1 && a >= 0 && a < kh && b >= 0 && b < kw;
      tp[q] = ok ? a * kw + b : -1;
      const int64_t o = ok ? ((int64_t)(n * Ho + ho) * Wo + wo) * C + cg * V : 0;
      if (V == 8) {
        pk[q] = ok ? *reinterpret_cast<const uint2*>(idx + o) : make_uint2(0, 0);
      } else {
        pk[q] = make_uint2(ok ? *reinterpret_cast<const uint32_t*>(idx + o) : 0u, 0u);
      }
      if (ok) {
        load_vec<T>(dy + o, g[q]);
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) g[q][k] = 0.f;
      }
    }
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const uint32_t word = k < 4 ? pk[q].x : pk[q].y;
        const int ix = (int)((word >> (8 * (k & 3))) & 255u);
        if (ix == tp[q]) acc[k] += g[q][k];
      }
    }
    store_vec<T>(drow + (int64_t)w * C, acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N,
                                                      int H, int W, int C, int Ho, int Wo, int kh,
                                                      int kw, int sh, int sw, int ph, int pw) {
  const int64_t total = (int64_t)N * Ho * Wo * C;
  const float inv = 1.f / (float)(kh * kw);  // count_include_pad semantics (cuDNN default)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int wo = (int)(t % Wo); t /= Wo;
    int ho = (int)(t % Ho);
    int n = (int)(t / Ho);
    float s = 0.f;
    for (int a = 0; a < kh; ++a) {
      int h = ho * sh - ph + a;
      if (h < 0 || h >= H) continue;
      for (int b = 0; b < kw; ++b) {
        int w = wo * sw - pw + b;
        if (w < 0 || w >= W) continue;
        s += to_f(x[(((int64_t)n * H + h) * W + w) * C + c]);
      }
    }
    y[i] = from_f<T>(s * inv);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int N,
                                                      int H, int W, int C, int Ho, int Wo, int kh,
                                                      int kw, int sh, int sw, int ph, int pw) {
  const int64_t total = (int64_t)N * H * W * C;
  const float inv = 1.f / (float)(kh * kw);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int w = (int)(t % W); t /= W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    int ho0 = (h + ph - kh + sh) / sh; if (h + ph - kh + 1 < 0) ho0 = 0;
    int ho1 = (h + ph) / sh; if (ho1 >= Ho) ho1 = Ho - 1;
    int wo0 = (w + pw - kw + sw) / sw; if (w + pw - kw + 1 < 0) wo0 = 0;
    int wo1 = (w + pw) / sw; if (wo1 >= Wo) wo1 = Wo - 1;
    float acc = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho) {
      int a = h + ph - ho * sh;
      if (a < 0 || a >= kh) continue;
      for (int wo = wo0; wo <= wo1; ++wo) {
        int b = w + pw - wo * sw;
        if (b < 0 || b >= kw) continue;
        acc += to_f(dy[(((int64_t)n * Ho + ho) * Wo + wo) * C + c]);
      }
    }
    dx[i] = from_f<T>(acc * inv);
  }
}

// y[b, c] = scale * sum_{r in chunk} x[b, r, c]; partial (fp32) when chunks > 1
template <typename T>
__global__ void __launch_bounds__(256) reduce_mid_k(const T* __restrict__ x, float* __restrict__ part,
                                                     int64_t B, int64_t R, int64_t C,
                                                     int64_t rows_per_chunk) {
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int rsub = threadIdx.x >> 6;  // 4 row lanes
  const int64_t b = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.z * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > R) r1 = R;
  __shared__ float sh[256];
  float s = 0.f;
  if (c < C) {   // 4 rows in flight per lane (one element per load: latency-bound otherwise)
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = r0 + rsub;
    for (; r + 12 < r1; r += 16) {
      s += to_f(x[(b * R + r) * C + c]);
      s1 += to_f(x[(b * R + r + 4) * C + c]);
      s2 += to_f(x[(b * R + r + 8) * C + c]);
      s3 += to_f(x[(b * R + r + 12) * C + c]);
    }
    for (; r < r1; r += 4) s += to_f(x[(b * R + r) * C + c]);
    s += s1 + s2 + s3;
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  if (rsub == 0 && c < C) {
    s = sh[threadIdx.x] + sh[threadIdx.x + 64] + sh[threadIdx.x + 128] + sh[threadIdx.x + 192];
    part[((int64_t)blockIdx.z * B + b) * C + c] = s;
  }
}

// vectorised variant (C % VEC == 0, 16-byte aligned rows): each lane sums VEC
// adjacent columns with 16-byte loads, so a wave streams 1 KiB (bf16) per row
template <typename T>
__global__ void __launch_bounds__(256) reduce_mid_vec_k(const T* __restrict__ x, float* __restrict__ part,
                                                         int64_t B, int64_t R, int64_t C,
                                                         int64_t rows_per_chunk) {
  constexpr int VEC = Vec<T>::N;
  __shared__ float sh[4][64 * VEC];
  const int lane = threadIdx.x & 63, rsub = threadIdx.x >> 6;
  const int64_t c = ((int64_t)blockIdx.x * 64 + lane) * VEC;
  const int64_t b = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.z * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > R) r1 = R;
  float acc[VEC], acc2[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) { acc[k] = 0.f; acc2[k] = 0.f; }
  if (c < C) {
    int64_t r = r0 + rsub;
    for (; r + 4 < r1; r += 8) {          // two rows in flight per lane
      float v[VEC], w[VEC];
      load_vec<T>(x + (b * R + r) * C + c, v);
      load_vec<T>(x + (b * R + r + 4) * C + c, w);
#pragma unroll
      for (int k = 0; k < VEC; ++k) { acc[k] += v[k]; acc2[k] += w[k]; }
    }
    for (; r < r1; r += 4) {
      float v[VEC];
      load_vec<T>(x + (b * R + r) * C + c, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < VEC; ++k) sh[rsub][lane * VEC + k] = acc[k] + acc2[k];
  __syncthreads();
  for (int j = threadIdx.x; j < 64 * VEC; j += 256) {
    const int64_t cc = (int64_t)blockIdx.x * 64 * VEC + j;
    if (cc < C) part[((int64_t)blockIdx.z * B + b) * C + cc] = sh[0][j] + sh[1][j] + sh[2][j] + sh[3][j];
  }
}

template <typename TO>
__global__ void reduce_mid_final_k(const float* __restrict__ part, TO* __restrict__ y, int64_t BC,
                                   int chunks, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < BC;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < chunks; ++k) s += part[(int64_t)k * BC + i];
    y[i] = from_f<TO>(s * scale);
  }
}

// final pass over the chunk partials: 64 columns x 4 chunk groups per block,
// 4 independent accumulators per thread (loads in flight), LDS fold
template <typename TO>
__global__ void __launch_bounds__(256) reduce_mid_final2_k(const float* __restrict__ part, TO* __restrict__ y,
                                                            int64_t BC, int chunks, float scale) {
  __shared__ float sh[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < BC) {
    int k = grp;
    for (; k + 12 < chunks; k += 16) {
      a0 += part[(int64_t)k * BC + i];
      a1 += part[(int64_t)(k + 4) * BC + i];
      a2 += part[(int64_t)(k + 8) * BC + i];
      a3 += part[(int64_t)(k + 12) * BC + i];
    }
    for (; k < chunks; k += 4) a0 += part[(int64_t)k * BC + i];
  }
  sh[grp][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (grp == 0 && i < BC) y[i] = from_f<TO>((sh[0][lane] + sh[1][lane] + sh[2][lane] + sh[3][lane]) * scale);
}

// y[r] = scale * sum_c x[r, c]  (one wave per row)
template <typename T, typename TO>
__global__ void __launch_bounds__(256) reduce_last_k(const T* __restrict__ x, TO* __restrict__ y, int64_t R,
                                                      int64_t C, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  float s = 0.f;
  for (int64_t j = lane; j < C; j += 64) s += to_f(x[row * C + j]);
  s = wave_sum(s);
  if (lane == 0) y[row] = from_f<TO>(s * scale);
}

// vector form (C % V == 0, 16-byte aligned rows): 16-byte loads, 4 in flight per lane --
// the scalar form's 2-byte loads (128 bytes per wave instruction) read the MoE bench's
// [65536, 2048] bf16 row sums at ~1.8 TB/s
template <typename T, typename TO>
__global__ void __launch_bounds__(256) reduce_last_vec_k(const T* __restrict__ x, TO* __restrict__ y, int64_t R,
                                                          int64_t C, float scale) {
  constexpr int V = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + row * C;
  const int64_t nv = C / V;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int64_t j = lane;
  for (; j + 192 < nv; j += 256) {
    float a[V], b[V], c[V], d[V];
    load_vec<T>(xr + j * V, a);
    load_vec<T>(xr + (j + 64) * V, b);
    load_vec<T>(xr + (j + 128) * V, c);
    load_vec<T>(xr + (j + 192) * V, d);
#pragma unroll
    for (int k = 0; k < V; ++k) { s0 += a[k]; s1 += b[k]; s2 += c[k]; s3 += d[k]; }
  }
  for (; j < nv; j += 64) {
    float a[V];
    load_vec<T>(xr + j * V, a);
#pragma unroll
    for (int k = 0; k < V; ++k) s0 += a[k];
  }
  const float s = wave_sum((s0 + s1) + (s2 + s3));
  if (lane == 0) y[row] = from_f<TO>(s * scale);
}

// broadcast y[b, r, c] = scale * x[b, c] (global-avg-pool backward)
template <typename T>
__global__ void bcast_mid_k(const T* __restrict__ x, T* __restrict__ y, int64_t B, int64_t R,
                            int64_t C, float scale) {
  const int64_t total = B * R * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t c = i % C, b = i / (R * C);
    y[i] = from_f<T>(to_f(x[b * C + c]) * scale);
  }
}

}  // namespace hetu

using namespace hetu;

HETU_API int hetu_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C,
                              int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw,
                              int is_bf16, hipStream_t st) {
  int64_t total = (int64_t)N * Ho * Wo * C;
  const int V = is_bf16 ? 8 : 4;
  if (C % V == 0 && total < (1LL << 31) && (int64_t)N * H * W * C < (1LL << 31)) {
    int64_t nb = (total / V + 255) / 256;
    int grid = (int)(nb < 65536 ? nb : 65536);
    if (is_bf16) hipLaunchKernelGGL(maxpool_fwd_vec<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, idx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    else hipLaunchKernelGGL(maxpool_fwd_vec<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, idx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    HETU_LAUNCH_CHECK();
    return 0;
  }
  int grid = stream_grid(total, 256, 2);
  if (is_bf16) hipLaunchKernelGGL(maxpool_fwd_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, idx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else hipLaunchKernelGGL(maxpool_fwd_k<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, idx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W,
                              int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph,
                              int pw, int is_bf16, hipStream_t st) {
  int64_t total = (int64_t)N * H * W * C;
  const int V = is_bf16 ? 8 : 4;
  if (C % V == 0 && 256 % (C / V) == 0 && kh <= sh + 1 && kw <= sw + 1 && H <= 65535 && N <= 65535 &&
      !getenv("HETU_MAXPOOL_FLAT")) {
    const dim3 grid((unsigned)H, (unsigned)N);
    if (is_bf16) hipLaunchKernelGGL(maxpool_bwd_rows<bf16>, grid, dim3(256), 0, st, (const bf16*)dy, idx, (bf16*)dx, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    else hipLaunchKernelGGL(maxpool_bwd_rows<float>, grid, dim3(256), 0, st, (const float*)dy, idx, (float*)dx, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    HETU_LAUNCH_CHECK();
    return 0;
  }
  if (C % V == 0 && total < (1LL << 31)) {
    int64_t nb = (total / V + 255) / 256;
    int grid = (int)(nb < 65536 ? nb : 65536);
    if (is_bf16) hipLaunchKernelGGL(maxpool_bwd_vec<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)dy, idx, (bf16*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    else hipLaunchKernelGGL(maxpool_bwd_vec<float>, dim3(grid), dim3(256), 0, st, (const float*)dy, idx, (float*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
    HETU_LAUNCH_CHECK();
    return 0;
  }
  int grid = stream_grid(total, 256, 2);
  if (is_bf16) hipLaunchKernelGGL(maxpool_bwd_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)dy, idx, (bf16*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else hipLaunchKernelGGL(maxpool_bwd_k<float>, dim3(grid), dim3(256), 0, st, (const float*)dy, idx, (float*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_avgpool_fwd(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo,
                              int kh, int kw, int sh, int sw, int ph, int pw, int is_bf16,
                              hipStream_t st) {
  int64_t total = (int64_t)N * Ho * Wo * C;
  int grid = stream_grid(total, 256, 2);
  if (is_bf16) hipLaunchKernelGGL(avgpool_fwd_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else hipLaunchKernelGGL(avgpool_fwd_k<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_avgpool_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                              int kh, int kw, int sh, int sw, int ph, int pw, int is_bf16,
                              hipStream_t st) {
  int64_t total = (int64_t)N * H * W * C;
  int grid = stream_grid(total, 256, 2);
  if (is_bf16) hipLaunchKernelGGL(avgpool_bwd_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)dy, (bf16*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else hipLaunchKernelGGL(avgpool_bwd_k<float>, dim3(grid), dim3(256), 0, st, (const float*)dy, (float*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  HETU_LAUNCH_CHECK();
  return 0;
}

// workspace: chunks * B * C floats; returns needed floats when ws == null
static int64_t reduce_mid_cols_per_tile(int64_t C, int x_bf16) {
  const int vec = x_bf16 ? 8 : 4;
  return (C % vec == 0) ? 64 * vec : 64;
}

HETU_API int64_t hetu_reduce_mid_ws(int64_t B, int64_t R, int64_t C) {
  int64_t ctiles = (C + 511) / 512;   // widest tile (bf16 vector path) -> most chunks
  int64_t blocks = ctiles * B;
  int64_t chunks = blocks >= 1024 ? 1 : (1024 + blocks - 1) / blocks;
  int64_t maxc = (R + 63) / 64;
  if (chunks > maxc) chunks = maxc;
  if (chunks < 1) chunks = 1;
  return chunks * B * C;
}

HETU_API int hetu_reduce_mid(const void* x, void* y, int64_t B, int64_t R, int64_t C, float scale,
                             int x_bf16, int y_bf16, float* ws, hipStream_t st) {
  const int64_t cpt = reduce_mid_cols_per_tile(C, x_bf16);
  const bool vec = cpt > 64 && ((uintptr_t)x % 16) == 0;
  int64_t ctiles = (C + (vec ? cpt : 64) - 1) / (vec ? cpt : 64);
  int64_t blocks = ctiles * B;
  const int64_t target = vec ? 1024 : 2048;   // the scalar path moves 4x fewer bytes per block
  int64_t chunks = blocks >= target ? 1 : (target + blocks - 1) / blocks;
  int64_t maxc = (R + 63) / 64;
  if (chunks > maxc) chunks = maxc;
  if (chunks < 1) chunks = 1;
  // never more chunks than the workspace sized by hetu_reduce_mid_ws holds
  const int64_t ws_chunks = hetu_reduce_mid_ws(B, R, C) / (B * C);
  if (chunks > ws_chunks) chunks = ws_chunks;
  // a few output columns (e.g. [T, E] gate statistics over T): the final pass is a handful
  // of blocks walking every chunk partial -- 1024 chunks kept one block busy for 24 us
  // after a 5 us first pass; 256 balances the two
  if (B * C <= 16 * 64 && chunks > 256) chunks = 256;
  int64_t rpc = (R + chunks - 1) / chunks;
  dim3 grid((unsigned)ctiles, (unsigned)B, (unsigned)chunks);
  if (vec) {
    if (x_bf16) hipLaunchKernelGGL(reduce_mid_vec_k<bf16>, grid, dim3(256), 0, st, (const bf16*)x, ws, B, R, C, rpc);
    else hipLaunchKernelGGL(reduce_mid_vec_k<float>, grid, dim3(256), 0, st, (const float*)x, ws, B, R, C, rpc);
  } else if (x_bf16) {
    hipLaunchKernelGGL(reduce_mid_k<bf16>, grid, dim3(256), 0, st, (const bf16*)x, ws, B, R, C, rpc);
  } else {
    hipLaunchKernelGGL(reduce_mid_k<float>, grid, dim3(256), 0, st, (const float*)x, ws, B, R, C, rpc);
  }
  if (chunks >= 16) {
    const unsigned g2 = (unsigned)((B * C + 63) / 64);
    if (y_bf16) hipLaunchKernelGGL(reduce_mid_final2_k<bf16>, dim3(g2), dim3(256), 0, st, ws, (bf16*)y, B * C, (int)chunks, scale);
    else hipLaunchKernelGGL(reduce_mid_final2_k<float>, dim3(g2), dim3(256), 0, st, ws, (float*)y, B * C, (int)chunks, scale);
  } else {
    int g2 = stream_grid(B * C, 256, 1);
    if (y_bf16) hipLaunchKernelGGL(reduce_mid_final_k<bf16>, dim3(g2), dim3(256), 0, st, ws, (bf16*)y, B * C, (int)chunks, scale);
    else hipLaunchKernelGGL(reduce_mid_final_k<float>, dim3(g2), dim3(256), 0, st, ws, (float*)y, B * C, (int)chunks, scale);
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_reduce_last(const void* x, void* y, int64_t R, int64_t C, float scale, int x_bf16,
                              int y_bf16, hipStream_t st) {
  dim3 grid((unsigned)((R + 3) / 4));
  const int V = x_bf16 ? 8 : 4;
  if (C % V == 0 && ((uintptr_t)x & 15) == 0) {
    if (x_bf16 && y_bf16) hipLaunchKernelGGL((reduce_last_vec_k<bf16, bf16>), grid, dim3(256), 0, st, (const bf16*)x, (bf16*)y, R, C, scale);
    else if (x_bf16) hipLaunchKernelGGL((reduce_last_vec_k<bf16, float>), grid, dim3(256), 0, st, (const bf16*)x, (float*)y, R, C, scale);
    else if (y_bf16) hipLaunchKernelGGL((reduce_last_vec_k<float, bf16>), grid, dim3(256), 0, st, (const float*)x, (bf16*)y, R, C, scale);
    else hipLaunchKernelGGL((reduce_last_vec_k<float, float>), grid, dim3(256), 0, st, (const float*)x, (float*)y, R, C, scale);
    HETU_LAUNCH_CHECK();
    return 0;
  }
  if (x_bf16 && y_bf16) hipLaunchKernelGGL((reduce_last_k<bf16, bf16>), grid, dim3(256), 0, st, (const bf16*)x, (bf16*)y, R, C, scale);
  else if (x_bf16) hipLaunchKernelGGL((reduce_last_k<bf16, float>), grid, dim3(256), 0, st, (const bf16*)x, (float*)y, R, C, scale);
  else if (y_bf16) hipLaunchKernelGGL((reduce_last_k<float, bf16>), grid, dim3(256), 0, st, (const float*)x, (bf16*)y, R, C, scale);
  else hipLaunchKernelGGL((reduce_last_k<float, float>), grid, dim3(256), 0, st, (const float*)x, (float*)y, R, C, scale);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_bcast_mid(const void* x, void* y, int64_t B, int64_t R, int64_t C, float scale,
                            int is_bf16, hipStream_t st) {
  int grid = stream_grid(B * R * C, 256, 2);
  if (is_bf16) hipLaunchKernelGGL(bcast_mid_k<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)x, (bf16*)y, B, R, C, scale);
  else hipLaunchKernelGGL(bcast_mid_k<float>, dim3(grid), dim3(256), 0, st, (const float*)x, (float*)y, B, R, C, scale);
  HETU_LAUNCH_CHECK();
  return 0;
}
