// Mixture-of-Experts routing kernels for gfx950 (reference src/ops/LayoutTransform.cu,
// TopKIdx.cu, TopKVal.cu, CumSum.cu).
//
// The reference dispatch scatters token rows with one thread per token and
// combines with atomicAdd; its gate gradient is a 32-lane shuffle dot product.
// Here every data-moving kernel is a *gather* (deterministic, no atomics) run as
// one wave64 per output row with 16-byte vector accesses:
//
//   slot_map      slot_src[e*cap + loc] = t*k + j  for every routed (t, j) with loc < cap
//   gather_slots  out[s, :] = w[slot_src[s]] * src[slot_src[s] / k, :]   (0 for empty slots)
//                 -> dispatch forward (w = 1) and combine backward-data (w = gate)
//   combine       out[t, :] = sum_j w[t, j] * y[slot(t, j), :]            (dropped -> 0)
//                 -> combine forward (w = gate) and dispatch backward (w = 1)
//   gate_grad     dgate[t, j] = <dout[t, :], y[slot(t, j), :]>            (wave64 dot)
//
// The gate itself is fused: `gate_topk` (softmax + top-k, one wave per token,
// k rounds of wave arg-max, experts held in registers) and `locations` (slot of
// every (token, choice) inside its expert's capacity, choice-major like the
// reference's cumsum chain, one workgroup per expert using ballot/popcount
// prefix sums; it also emits the per-expert load-balancing terms).  The gate
// backward `gate_backward` folds the gate-value gradient and the balance-loss
// gradient into one softmax backward per token.
#include "common.h"
#include <stdlib.h>
#include <algorithm>

namespace hetu {

constexpr int kMaxEPL = 8;   // experts per lane (E <= 512)
constexpr int kMaxK = 16;    // choices per token (the dense-to-sparse gate starts at k = E = 16 on 8 GPUs)

// ---------------------------------------------------------------------------
// softmax + top-k per row
template <typename T>
__global__ void __launch_bounds__(256) gate_topk_k(const T* __restrict__ logits, float* __restrict__ probs,
                                                    int64_t* __restrict__ idx, float* __restrict__ val,
                                                    int rows, int E, int k, int do_softmax) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = logits + (int64_t)row * E;
  float v[kMaxEPL];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < kMaxEPL; ++i) {
    const int e = lane + 64 * i;
    v[i] = (e < E) ? to_f(x[e]) : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  if (do_softmax) {
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      v[i] = (e < E) ? __expf(v[i] - m) : 0.f;
      s += v[i];
    }
    s = wave_sum(s);
    const float inv = 1.f / s;
#pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      if (e < E) {
        v[i] *= inv;
        probs[(int64_t)row * E + e] = v[i];
      } else {
        v[i] = -INFINITY;
      }
    }
  }
  for (int j = 0; j < k; ++j) {
    // lane-local best (lowest expert id on ties), then wave arg-max
    float bv = -INFINITY;
    int be = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      if (e < E && (v[i] > bv || (v[i] == bv && e < be))) { bv = v[i]; be = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oe = __shfl_xor(be, o, 64);
      if (ov > bv || (ov == bv && oe < be)) { bv = ov; be = oe; }
    }
    if (lane == 0) {
      idx[(int64_t)row * k + j] = be;
      val[(int64_t)row * k + j] = bv;
    }
#pragma unroll
    for (int i = 0; i < kMaxEPL; ++i)
      if (lane + 64 * i == be) v[i] = -INFINITY;
  }
}

// ---------------------------------------------------------------------------
// Dense-to-sparse gate (Nie et al., Hetu README paper #6), one wave per token:
//   y = softmax((logits + gumbel) / tau)           gumbel = -log(-log(u)), u ~ Philox(seed, t*E + e)
//   choices j < k in descending y; choice j > 0 is active only while y >= thr (the
//   top-1 choice is always kept): inactive choices get idx = -1, val = 0 -- the slot
//   map, combine and gate-gradient kernels skip them, so they take no capacity.
//   hist[n] += 1 for a token with n active choices (n = 1..k): the host shrinks the
//   expert budget k (and the capacity) once the threshold leaves fewer experts active.
template <typename T>
__global__ void __launch_bounds__(256) dts_gate_k(const T* __restrict__ logits, float* __restrict__ probs,
                                                   int64_t* __restrict__ idx, float* __restrict__ val,
                                                   int* __restrict__ hist, int rows, int E, int k, float inv_tau,
                                                   float thr, uint64_t seed_, const uint64_t* __restrict__ rngo,
                                                   int noise) {
  // the active-choice histogram is folded per block in LDS (one global atomic per bin per
  // block instead of one per token: 65536 tokens into <= 17 counters serialised on them)
  __shared__ int bh[kMaxK + 1];
  const uint64_t seed = rng_seed(seed_, rngo);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x <= kMaxK) bh[threadIdx.x] = 0;
  __syncthreads();
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const T* x = logits + (int64_t)row * E;
    float v[kMaxEPL];
    float m = -INFINITY;
  #pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      float z = -INFINITY;
      if (e < E) {
        z = to_f(x[e]);
        if (noise) {
          const float u = Philox::u01(Philox::gen(seed, (uint64_t)row * (uint64_t)E + (uint64_t)e).x);
          z -= __logf(-__logf(u));
        }
        z *= inv_tau;
      }
      v[i] = z;
      m = fmaxf(m, z);
    }
    m = wave_max(m);
    float s = 0.f;
  #pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      v[i] = (e < E) ? __expf(v[i] - m) : 0.f;
      s += v[i];
    }
    s = wave_sum(s);
    const float inv = 1.f / s;
  #pragma unroll
    for (int i = 0; i < kMaxEPL; ++i) {
      const int e = lane + 64 * i;
      if (e < E) {
        v[i] *= inv;
        probs[(int64_t)row * E + e] = v[i];
      } else {
        v[i] = -INFINITY;
      }
    }
    int active = 0;
    for (int j = 0; j < k; ++j) {
      float bv = -INFINITY;
      int be = 0x7fffffff;
  #pragma unroll
      for (int i = 0; i < kMaxEPL; ++i) {
        const int e = lane + 64 * i;
        if (e < E && (v[i] > bv || (v[i] == bv && e < be))) { bv = v[i]; be = e; }
      }
  #pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oe = __shfl_xor(be, o, 64);
        if (ov > bv || (ov == bv && oe < be)) { bv = ov; be = oe; }
      }
      const bool on = j == 0 || bv >= thr;     // wave-uniform
      if (lane == 0) {
        idx[(int64_t)row * k + j] = on ? be : -1;
        val[(int64_t)row * k + j] = on ? bv : 0.f;
      }
      active += on ? 1 : 0;
  #pragma unroll
      for (int i = 0; i < kMaxEPL; ++i)
        if (lane + 64 * i == be) v[i] = -INFINITY;
    }
    if (lane == 0 && hist != nullptr) atomicAdd(bh + active, 1);
  }
  __syncthreads();
  if (hist != nullptr && threadIdx.x <= k && bh[threadIdx.x] != 0) atomicAdd(hist + threadIdx.x, bh[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// capacity slots, choice-major: loc(t, j) = #{(t', j') before (t, j) in order
// (j' < j) or (j' == j, t' < t) with idx == idx(t, j)}.  One workgroup per
// expert; also counts[e] = routed (t, j) pairs (before drops) and
// psum[e] = sum_t probs[t, e] (balance loss).
__global__ void __launch_bounds__(256) locations_k(const int64_t* __restrict__ idx,
                                                   const float* __restrict__ probs,
                                                   int64_t* __restrict__ loc, int* __restrict__ counts,
                                                   float* __restrict__ psum, int T, int k, int E) {
  // 16 consecutive choices per thread per pass (4096 per pass): one block-wide exclusive
  // scan of the per-thread hit counts per pass instead of one per 256 choices -- with few
  // experts (one block each) the scan latency, not the bandwidth, was the cost
  constexpr int PT = 16;
  __shared__ int wsum[4];
  __shared__ float fsum[4];
  const int e = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int base = 0;
  const int total = T * k;
  for (int c0 = 0; c0 < total; c0 += 256 * PT) {
    const int cb = c0 + threadIdx.x * PT;
    unsigned hits = 0u;
    const int j0 = cb / T, t0 = cb - j0 * T;   // choice-major flat index c = j * T + t
    {
      int j = j0, t = t0;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        if (cb + i < total && idx[(int64_t)t * k + j] == e) hits |= 1u << i;
        if (++t == T) { t = 0; ++j; }
      }
    }
    const int h = __popc(hits);
    // inclusive scan of h over the wave
    int incl = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int off = base + incl - h;
    for (int q = 0; q < w; ++q) off += wsum[q];
    {
      int j = j0, t = t0;
      for (int i = 0; i < PT; ++i) {
        if (hits & (1u << i)) loc[(int64_t)t * k + j] = off++;
        if (++t == T) { t = 0; ++j; }
      }
    }
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  float s = 0.f;
  if (probs != nullptr)
    for (int t = threadIdx.x; t < T; t += 256) s += probs[(int64_t)t * E + e];
  s = wave_sum(s);
  if (lane == 0) fsum[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    counts[e] = base;
    if (psum != nullptr) psum[e] = fsum[0] + fsum[1] + fsum[2] + fsum[3];
  }
}

// Segmented form of locations_k for large T*k: the choice range is cut into S segments of
// `seg` choices and every (expert, segment) pair is a block, so the scan runs on E*S blocks
// instead of E (two of them for the bench's 2 experts: 0.2 ms of latency per step).
// Pass 1 counts each segment's hits; pass 2 starts every segment at the sum of its
// predecessors' counts and ranks its own hits with the block scan of locations_k (segment 0
// also sums the expert's gate probabilities, in a fixed order).
__global__ void __launch_bounds__(256) loc_count_k(const int64_t* __restrict__ idx, int* __restrict__ cnt, int T,
                                                   int k, int seg, int S) {
  __shared__ int ws[4];
  const int e = blockIdx.x / S, sg = blockIdx.x - e * S;
  const int total = T * k;
  const int c0 = sg * seg, c1 = min(total, c0 + seg);
  int h = 0;
  for (int c = c0 + (int)threadIdx.x; c < c1; c += 256) {
    const int j = c / T, t = c - j * T;
    h += idx[(int64_t)t * k + j] == e ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void __launch_bounds__(256) loc_scan_k(const int64_t* __restrict__ idx, const float* __restrict__ probs,
                                                  int64_t* __restrict__ loc, int* __restrict__ counts,
                                                  float* __restrict__ psum, const int* __restrict__ cnt, int T, int k,
                                                  int E, int seg, int S) {
  constexpr int PT = 8;
  __shared__ int wsum[4];
  __shared__ float fsum[4];
  const int e = blockIdx.x / S, sg = blockIdx.x - e * S;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int total = T * k;
  const int c0 = sg * seg, c1 = min(total, c0 + seg);
  // this segment's start: the predecessors' hit counts
  int pre = 0;
  for (int q = threadIdx.x; q < sg; q += 256) pre += cnt[e * S + q];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane == 0) wsum[w] = pre;
  __syncthreads();
  int base = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  for (int p0 = c0; p0 < c1; p0 += 256 * PT) {
    const int cb = p0 + threadIdx.x * PT;
    unsigned hits = 0u;
    const int j0 = cb / T, t0 = cb - j0 * T;
    {
      int j = j0, t = t0;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        if (cb + i < c1 && idx[(int64_t)t * k + j] == e) hits |= 1u << i;
        if (++t == T) { t = 0; ++j; }
      }
    }
    const int h = __popc(hits);
    int incl = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int off = base + incl - h;
    for (int q = 0; q < w; ++q) off += wsum[q];
    {
      int j = j0, t = t0;
      for (int i = 0; i < PT; ++i) {
        if (hits & (1u << i)) loc[(int64_t)t * k + j] = off++;
        if (++t == T) { t = 0; ++j; }
      }
    }
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (sg == S - 1 && threadIdx.x == 0) counts[e] = base;
  if (probs != nullptr && psum != nullptr && sg == 0) {
    // the tokens' gate probabilities, in a fixed order (deterministic balance loss); eight
    // independent loads per thread in flight (one block walks all T tokens)
    float sq[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) sq[u] = 0.f;
    int t = threadIdx.x;
    for (; t + 7 * 256 < T; t += 8 * 256) {
#pragma unroll
      for (int u = 0; u < 8; ++u) sq[u] += probs[(int64_t)(t + u * 256) * E + e];
    }
    for (; t < T; t += 256) sq[0] += probs[(int64_t)t * E + e];
    float sp = ((sq[0] + sq[1]) + (sq[2] + sq[3])) + ((sq[4] + sq[5]) + (sq[6] + sq[7]));
    sp = wave_sum(sp);
    if (lane == 0) fsum[w] = sp;
    __syncthreads();
    if (threadIdx.x == 0) psum[e] = fsum[0] + fsum[1] + fsum[2] + fsum[3];
  }
}

// dlogits[t, :] = scale * softmax_bwd(p, dp) with
// dp[t, e] = sum_j [idx(t, j) == e] * dgate[t, j] + aux_coef[e]
// (scale = 1 / tau for the tempered softmax of the dense-to-sparse gate; choices with
// idx = -1 -- inactive -- carry no gradient: the threshold mask's derivative)
__global__ void __launch_bounds__(256) gate_backward_k(const float* __restrict__ probs,
                                                       const int64_t* __restrict__ idx,
                                                       const float* __restrict__ dgate,
                                                       const float* __restrict__ aux_coef,
                                                       float* __restrict__ dlogits, int rows, int E, int k,
                                                       float scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  int ie[kMaxK];
  float ig[kMaxK];
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) {
    ie[j] = (j < k) ? (int)idx[(int64_t)row * k + j] : -1;
    ig[j] = (j < k && dgate != nullptr) ? dgate[(int64_t)row * k + j] : 0.f;
  }
  float p[kMaxEPL], dp[kMaxEPL];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxEPL; ++i) {
    const int e = lane + 64 * i;
    p[i] = 0.f; dp[i] = 0.f;
    if (e < E) {
      p[i] = probs[(int64_t)row * E + e];
      float d = aux_coef != nullptr ? aux_coef[e] : 0.f;
#pragma unroll
      for (int j = 0; j < kMaxK; ++j) d += (ie[j] == e) ? ig[j] : 0.f;
      dp[i] = d;
      dot += p[i] * d;
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int i = 0; i < kMaxEPL; ++i) {
    const int e = lane + 64 * i;
    if (e < E) dlogits[(int64_t)row * E + e] = scale * p[i] * (dp[i] - dot);
  }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) slot_map_k(const int64_t* __restrict__ idx,
                                                  const int64_t* __restrict__ loc, int* __restrict__ slot_src,
                                                  int Tk, int cap, int nslots) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Tk) return;
  const int64_t l = loc[i], e = idx[i];
  if (l < cap && l >= 0 && e >= 0) {
    const int64_t s = e * cap + l;
    if (s < nslots) slot_src[s] = i;
  }
}

// row copy helpers: one wave moves one row of d elements (vectorised when aligned)
template <typename T>
__device__ __forceinline__ void row_scale_copy(const T* __restrict__ src, T* __restrict__ dst, float w, int d,
                                               int lane, bool vec) {
  constexpr int N = Vec<T>::N;
  if (vec) {
    // four 16-byte pieces per lane in flight before their stores (a d = 2048 bf16 row is
    // exactly one group): one memory latency per row instead of one per piece
    int c = lane * N;
    for (; c + 3 * 64 * N < d; c += 4 * 64 * N) {
      float v[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_vec<T>(src + c + u * 64 * N, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int q = 0; q < N; ++q) v[u][q] *= w;
        store_vec<T>(dst + c + u * 64 * N, v[u]);
      }
    }
    for (; c < d; c += 64 * N) {
      float v[N];
      load_vec<T>(src + c, v);
#pragma unroll
      for (int q = 0; q < N; ++q) v[q] *= w;
      store_vec<T>(dst + c, v);
    }
  } else {
    for (int c = lane; c < d; c += 64) dst[c] = from_f<T>(w * to_f(src[c]));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gather_slots_k(const T* __restrict__ src, const int* __restrict__ slot_src,
                                                      const float* __restrict__ w, T* __restrict__ out,
                                                      int nslots, int d, int k, int vec) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslots) return;
  const int si = slot_src[s];
  T* o = out + (int64_t)s * d;
  if (si < 0) {
    constexpr int N = Vec<T>::N;
    if (vec) {
      float z[N];
#pragma unroll
      for (int q = 0; q < N; ++q) z[q] = 0.f;
      for (int c = lane * N; c < d; c += 64 * N) store_vec<T>(o + c, z);
    } else {
      for (int c = lane; c < d; c += 64) o[c] = from_f<T>(0.f);
    }
    return;
  }
  const float ww = w != nullptr ? w[si] : 1.f;
  row_scale_copy<T>(src + (int64_t)(si / k) * d, o, ww, d, lane, vec != 0);
}

template <typename T>
__global__ void __launch_bounds__(256) combine_k(const T* __restrict__ y, const int64_t* __restrict__ idx,
                                                 const int64_t* __restrict__ loc, const float* __restrict__ w,
                                                 T* __restrict__ out, int Tn, int k, int cap, int d, int vec) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= Tn) return;
  const T* rows[kMaxK];
  float ws[kMaxK];
  int nv = 0;
  for (int j = 0; j < k && j < kMaxK; ++j) {
    const int64_t l = loc[(int64_t)t * k + j];
    if (l < cap && l >= 0) {
      rows[nv] = y + ((int64_t)idx[(int64_t)t * k + j] * cap + l) * d;
      ws[nv] = w != nullptr ? w[(int64_t)t * k + j] : 1.f;
      ++nv;
    }
  }
  T* o = out + (int64_t)t * d;
  if (vec) {
    // four 16-byte pieces of a source row per lane in flight at once (row_scale_copy)
    int c = lane * N;
    for (; c + 3 * 64 * N < d; c += 4 * 64 * N) {
      float acc[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < N; ++q) acc[u][q] = 0.f;
      for (int r = 0; r < nv; ++r) {
        float v[4][N];
#pragma unroll
        for (int u = 0; u < 4; ++u) load_vec<T>(rows[r] + c + u * 64 * N, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < N; ++q) acc[u][q] += ws[r] * v[u][q];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) store_vec<T>(o + c + u * 64 * N, acc[u]);
    }
    for (; c < d; c += 64 * N) {
      float acc[N];
#pragma unroll
      for (int q = 0; q < N; ++q) acc[q] = 0.f;
      for (int r = 0; r < nv; ++r) {
        float v[N];
        load_vec<T>(rows[r] + c, v);
#pragma unroll
        for (int q = 0; q < N; ++q) acc[q] += ws[r] * v[q];
      }
      store_vec<T>(o + c, acc);
    }
  } else {
    for (int c = lane; c < d; c += 64) {
      float acc = 0.f;
      for (int r = 0; r < nv; ++r) acc += ws[r] * to_f(rows[r][c]);
      o[c] = from_f<T>(acc);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gate_grad_k(const T* __restrict__ g, const T* __restrict__ y,
                                                   const int64_t* __restrict__ idx, const int64_t* __restrict__ loc,
                                                   float* __restrict__ out, int Tk, int k, int cap, int d, int vec) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= Tk) return;
  const int64_t l = loc[i];
  if (l >= cap || l < 0) {
    if (lane == 0) out[i] = 0.f;
    return;
  }
  const T* gr = g + (int64_t)(i / k) * d;
  const T* yr = y + ((int64_t)idx[i] * cap + l) * d;
  float s = 0.f;
  if (vec) {
    // four 16-byte pieces of both rows per lane in flight at once
    int c = lane * N;
    for (; c + 3 * 64 * N < d; c += 4 * 64 * N) {
      float a[4][N], b[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        load_vec<T>(gr + c + u * 64 * N, a[u]);
        load_vec<T>(yr + c + u * 64 * N, b[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < N; ++q) s += a[u][q] * b[u][q];
    }
    for (; c < d; c += 64 * N) {
      float a[N], b[N];
      load_vec<T>(gr + c, a);
      load_vec<T>(yr + c, b);
#pragma unroll
      for (int q = 0; q < N; ++q) s += a[q] * b[q];
    }
  } else {
    for (int c = lane; c < d; c += 64) s += to_f(gr[c]) * to_f(yr[c]);
  }
  s = wave_sum(s);
  if (lane == 0) out[i] = s;
}

// Backward of the gate-weighted combine, both gradients from one read of the token
// gradient g: wave s (slot) writes dslot[s] = w[si] * g[si / k] (zeros for an empty slot)
// and the gate gradient gout[si] = <g[si / k], y[s]>; wave i < Tk also zeroes gout[i] of a
// (token, choice) pair dropped at capacity.  (gather_slots_k + gate_grad_k read g twice.)
template <typename T>
__global__ void __launch_bounds__(256) gather_slots_gate_k(const T* __restrict__ g, const T* __restrict__ y,
                                                           const int* __restrict__ slot_src,
                                                           const float* __restrict__ w,
                                                           const int64_t* __restrict__ loc, T* __restrict__ out,
                                                           float* __restrict__ gout, int nslots, int Tk, int d,
                                                           int k, int cap, int vec) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s < Tk && lane == 0) {
    const int64_t l = loc[s];
    if (l >= cap || l < 0) gout[s] = 0.f;
  }
  if (s >= nslots) return;
  const int si = slot_src[s];
  T* o = out + (int64_t)s * d;
  if (si < 0) {
    if (vec) {
      float z[N];
#pragma unroll
      for (int q = 0; q < N; ++q) z[q] = 0.f;
      for (int c = lane * N; c < d; c += 64 * N) store_vec<T>(o + c, z);
    } else {
      for (int c = lane; c < d; c += 64) o[c] = from_f<T>(0.f);
    }
    return;
  }
  const float ww = w != nullptr ? w[si] : 1.f;
  const T* gr = g + (int64_t)(si / k) * d;
  const T* yr = y + (int64_t)s * d;
  float acc = 0.f;
  if (vec) {
    int c = lane * N;
    for (; c + 3 * 64 * N < d; c += 4 * 64 * N) {
      float a[4][N], b[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        load_vec<T>(gr + c + u * 64 * N, a[u]);
        load_vec<T>(yr + c + u * 64 * N, b[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int q = 0; q < N; ++q) {
          acc += a[u][q] * b[u][q];
          a[u][q] *= ww;
        }
        store_vec<T>(o + c + u * 64 * N, a[u]);
      }
    }
    for (; c < d; c += 64 * N) {
      float a[N], b[N];
      load_vec<T>(gr + c, a);
      load_vec<T>(yr + c, b);
#pragma unroll
      for (int q = 0; q < N; ++q) {
        acc += a[q] * b[q];
        a[q] *= ww;
      }
      store_vec<T>(o + c, a);
    }
  } else {
    for (int c = lane; c < d; c += 64) {
      const float a = to_f(gr[c]);
      acc += a * to_f(yr[c]);
      o[c] = from_f<T>(ww * a);
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) gout[si] = acc;
}

template <typename T>
static bool vec_ok(const void* a, const void* b, int d) {
  constexpr int N = Vec<T>::N;
  return (d % N) == 0 && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0;
}

}  // namespace hetu

using namespace hetu;

HETU_API int hetu_moe_gate_topk(const void* logits, float* probs, int64_t* idx, float* val, int rows, int E,
                                int k, int do_softmax, int bf16_in, hipStream_t s) {
  if (E > 64 * kMaxEPL || k > kMaxK || k > E) return (int)hipErrorInvalidValue;
  const int g = (rows + 3) / 4;
  if (g == 0) return 0;
  if (bf16_in)
    gate_topk_k<bf16><<<g, 256, 0, s>>>((const bf16*)logits, probs, idx, val, rows, E, k, do_softmax);
  else
    gate_topk_k<float><<<g, 256, 0, s>>>((const float*)logits, probs, idx, val, rows, E, k, do_softmax);
  HETU_LAUNCH_CHECK();
  return 0;
}

// hist: [k + 1] active-choice histogram, zeroed here (the host reads it a step later)
HETU_API int hetu_moe_dts_gate(const void* logits, float* probs, int64_t* idx, float* val, int* hist, int rows,
                               int E, int k, float inv_tau, float thr, uint64_t seed, int noise, int bf16_in,
                               hipStream_t s) {
  if (E > 64 * kMaxEPL || k > kMaxK || k > E || k < 1) return (int)hipErrorInvalidValue;
  if (hist != nullptr) {
    hipError_t e = hipMemsetAsync(hist, 0, (size_t)(k + 1) * sizeof(int), s);
    if (e != hipSuccess) return (int)e;
  }
  // <= 8 blocks per CU of 4 tokens per pass: each block folds >= 32 tokens' histogram
  int g = (rows + 3) / 4;
  if (g == 0) return 0;
  if (g > 2048) g = 2048;
  const uint64_t* ro = noise ? hetu_rng_offset_ptr() : nullptr;
  if (bf16_in)
    dts_gate_k<bf16><<<g, 256, 0, s>>>((const bf16*)logits, probs, idx, val, hist, rows, E, k, inv_tau, thr, seed,
                                       ro, noise);
  else
    dts_gate_k<float><<<g, 256, 0, s>>>((const float*)logits, probs, idx, val, hist, rows, E, k, inv_tau, thr,
                                        seed, ro, noise);
  HETU_LAUNCH_CHECK();
  return 0;
}

// Balance-loss terms of a top-k gate in one tiny launch (one wave): coef[e] = counts[e] / T,
// l_aux = E * sum_e (psum[e] / T) * coef[e]  (reference TopGate.py's load-balancing loss).
__global__ void __launch_bounds__(64) moe_aux_k(const int* __restrict__ counts, const float* __restrict__ psum,
                                                float* __restrict__ coef, float* __restrict__ l_aux, int T, int E) {
  const float inv = 1.f / (float)T;
  float acc = 0.f;
  for (int e = threadIdx.x; e < E; e += 64) {
    const float c = (float)counts[e] * inv;
    coef[e] = c;
    acc += psum[e] * inv * c;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0) l_aux[0] = acc * (float)E;
}

HETU_API int hetu_moe_aux(const int* counts, const float* psum, float* coef, float* l_aux, int T, int E,
                          hipStream_t st) {
  hipLaunchKernelGGL(moe_aux_k, dim3(1), dim3(64), 0, st, counts, psum, coef, l_aux, T, E);
  return (int)hipGetLastError();
}

static void loc_segments(int64_t total, int& seg, int& S) {
  seg = 2048;
  while ((total + seg - 1) / seg > 1024) seg *= 2;
  S = (int)((total + seg - 1) / seg);
}

// int32 workspace (per-segment hit counts) hetu_moe_locations2 needs; 0 = single-block scan
HETU_API int64_t hetu_moe_locations_ws(int T, int k, int E) {
  int seg, S;
  loc_segments((int64_t)T * k, seg, S);
  return S > 1 ? (int64_t)E * S : 0;
}

// ws: hetu_moe_locations_ws(T, k, E) ints (null, or HETU_MOE_LOC_SEGMENTED=0: one block per
// expert scans every choice)
HETU_API int hetu_moe_locations2(const int64_t* idx, const float* probs, int64_t* loc, int* counts, float* psum,
                                 int T, int k, int E, int* ws, hipStream_t s) {
  if (E <= 0) return 0;
  int seg, S;
  loc_segments((int64_t)T * k, seg, S);
  const char* env = getenv("HETU_MOE_LOC_SEGMENTED");
  const bool segmented = ws != nullptr && (env == nullptr || env[0] != '0') && S > 1;
  if (!segmented) {
    locations_k<<<E, 256, 0, s>>>(idx, probs, loc, counts, psum, T, k, E);
  } else {
    loc_count_k<<<E * S, 256, 0, s>>>(idx, ws, T, k, seg, S);
    loc_scan_k<<<E * S, 256, 0, s>>>(idx, probs, loc, counts, psum, ws, T, k, E, seg, S);
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_moe_locations(const int64_t* idx, const float* probs, int64_t* loc, int* counts, float* psum,
                                int T, int k, int E, hipStream_t s) {
  return hetu_moe_locations2(idx, probs, loc, counts, psum, T, k, E, nullptr, s);
}

HETU_API int hetu_moe_gate_backward(const float* probs, const int64_t* idx, const float* dgate,
                                    const float* aux_coef, float* dlogits, int rows, int E, int k, float scale,
                                    hipStream_t s) {
  if (E > 64 * kMaxEPL || k > kMaxK) return (int)hipErrorInvalidValue;
  const int g = (rows + 3) / 4;
  if (g == 0) return 0;
  gate_backward_k<<<g, 256, 0, s>>>(probs, idx, dgate, aux_coef, dlogits, rows, E, k, scale);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_moe_slot_map(const int64_t* idx, const int64_t* loc, int* slot_src, int Tk, int cap,
                               int nslots, hipStream_t s) {
  hipError_t e = hipMemsetAsync(slot_src, 0xff, (size_t)nslots * sizeof(int), s);
  if (e != hipSuccess) return (int)e;
  if (Tk > 0) slot_map_k<<<(Tk + 255) / 256, 256, 0, s>>>(idx, loc, slot_src, Tk, cap, nslots);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_moe_gather_slots(const void* src, const int* slot_src, const float* w, void* out, int nslots,
                                   int d, int k, int bf16_io, hipStream_t s) {
  const int g = (nslots + 3) / 4;
  if (g == 0) return 0;
  if (bf16_io)
    gather_slots_k<bf16><<<g, 256, 0, s>>>((const bf16*)src, slot_src, w, (bf16*)out, nslots, d, k,
                                           vec_ok<bf16>(src, out, d));
  else
    gather_slots_k<float><<<g, 256, 0, s>>>((const float*)src, slot_src, w, (float*)out, nslots, d, k,
                                            vec_ok<float>(src, out, d));
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_moe_combine(const void* y, const int64_t* idx, const int64_t* loc, const float* w, void* out,
                              int T, int k, int cap, int d, int bf16_io, hipStream_t s) {
  if (k > kMaxK) return (int)hipErrorInvalidValue;
  const int g = (T + 3) / 4;
  if (g == 0) return 0;
  if (bf16_io)
    combine_k<bf16><<<g, 256, 0, s>>>((const bf16*)y, idx, loc, w, (bf16*)out, T, k, cap, d,
                                      vec_ok<bf16>(y, out, d));
  else
    combine_k<float><<<g, 256, 0, s>>>((const float*)y, idx, loc, w, (float*)out, T, k, cap, d,
                                       vec_ok<float>(y, out, d));
  HETU_LAUNCH_CHECK();
  return 0;
}

// both gradients of the gate-weighted combine (gather_slots_gate_k): y [nslots, d] the
// expert outputs the forward combined, g [T, d], out [nslots, d], gout [Tk] fp32
HETU_API int hetu_moe_gather_slots_gate(const void* g, const void* y, const int* slot_src, const float* w,
                                        const int64_t* loc, void* out, float* gout, int nslots, int Tk, int d, int k,
                                        int cap, int bf16_io, hipStream_t s) {
  const int n = nslots > Tk ? nslots : Tk;
  const int gr = (n + 3) / 4;
  if (gr == 0) return 0;
  if (bf16_io)
    gather_slots_gate_k<bf16><<<gr, 256, 0, s>>>((const bf16*)g, (const bf16*)y, slot_src, w, loc, (bf16*)out, gout,
                                                 nslots, Tk, d, k, cap,
                                                 vec_ok<bf16>(g, y, d) && vec_ok<bf16>(out, out, d));
  else
    gather_slots_gate_k<float><<<gr, 256, 0, s>>>((const float*)g, (const float*)y, slot_src, w, loc, (float*)out,
                                                  gout, nslots, Tk, d, k, cap,
                                                  vec_ok<float>(g, y, d) && vec_ok<float>(out, out, d));
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_moe_gate_grad(const void* g, const void* y, const int64_t* idx, const int64_t* loc, float* out,
                                int Tk, int k, int cap, int d, int bf16_io, hipStream_t s) {
  const int gr = (Tk + 3) / 4;
  if (gr == 0) return 0;
  if (bf16_io)
    gate_grad_k<bf16><<<gr, 256, 0, s>>>((const bf16*)g, (const bf16*)y, idx, loc, out, Tk, k, cap, d,
                                         vec_ok<bf16>(g, y, d));
  else
    gate_grad_k<float><<<gr, 256, 0, s>>>((const float*)g, (const float*)y, idx, loc, out, Tk, k, cap, d,
                                          vec_ok<float>(g, y, d));
  HETU_LAUNCH_CHECK();
  return 0;
}
