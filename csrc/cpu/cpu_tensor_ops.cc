// Native CPU backend, part 2 (C++ / OpenMP): the elementwise, layout, softmax, dropout
// and initializer kernels of the reference's CPU path (src/dnnl_ops/AddElewise.cpp,
// Softmax.cpp, Pad.cpp, Concat.cpp, Transpose.cpp, Dropout.cpp, Initializers.cpp,
// ReduceSumAxisZero.cpp).  fp32, OpenMP over flat index ranges.
//
// * elementwise: the op codes of csrc/kernels/elementwise.hip (U / B tables in
//   kernels/elementwise.py), so the CPU and GPU backends implement ONE op table;
//   binary ops take a general N-d broadcast (per-dim strides, 0 = broadcast).
// * layout: one strided N-d copy serves transpose / permute, slice, concat (copy into
//   an output slice) and pad (fill, then copy into the interior).
// * random: Philox4x32-10 at counter = flat index / 4 (the device generator of
//   common.h), so a CPU dropout mask equals the GPU mask for the same seed, and
//   initialisers draw the same numbers on every backend.
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#define API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxDims = 8;

// ---- Philox4x32-10 (same constants and key schedule as hetu::Philox in common.h) ----
struct U4 { uint32_t x, y, z, w; };

inline U4 philox(uint64_t seed, uint64_t counter) {
  uint32_t c0 = (uint32_t)counter, c1 = (uint32_t)(counter >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f); }

inline float gelu(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118f)); }

inline float unary_op(int op, float v, float c, float c2) {
  switch (op) {
    case 0: return v > 0.f ? v : 0.f;                       // relu
    case 1: return 1.f / (1.f + expf(-v));                  // sigmoid
    case 2: return tanhf(v);
    case 3: return expf(v);
    case 4: return logf(v);
    case 5: return sqrtf(v);
    case 6: return 1.f / sqrtf(v);                          // rsqrt
    case 7: return fabsf(v);
    case 8: return -v;
    case 9: return gelu(v);
    case 10: return v > 0.f ? v : c * v;                    // leaky_relu
    case 11: return floorf(v);
    case 12: return sinf(v);
    case 13: return cosf(v);
    case 14: return v + c;                                  // add_c
    case 15: return v * c;                                  // mul_c
    case 16: return c - v;                                  // rsub_c
    case 17: return c / v;                                  // rdiv_c
    case 18: return powf(v, c);                             // pow_c
    case 19: return powf(c, v);                             // cpow
    case 20: return std::min(std::max(v, c), c2);           // clamp
    case 21: return (float)((v > 0.f) - (v < 0.f));         // sign
    case 22: return v > c ? 1.f : 0.f;                      // gt_c
    case 23: return 1.f / v;                                // recip
    case 24: return v * v;                                  // square
    default: {                                              // 25 gelu_tanh
      const float k = 0.7978845608f;
      return 0.5f * v * (1.f + tanhf(k * (v + 0.044715f * v * v * v)));
    }
  }
}

inline float binary_op(int op, float a, float b, float c) {
  switch (op) {
    case 0: return a + b;
    case 1: return a - b;
    case 2: return a * b;
    case 3: return a / b;
    case 4: return std::max(a, b);
    case 5: return std::min(a, b);
    case 6: return a > 0.f ? b : 0.f;                        // relu_grad (a = x, b = dy)
    case 7: {                                                // gelu_grad
      const float cdf = 0.5f * (1.f + erff(a * 0.70710678118f));
      const float pdf = expf(-0.5f * a * a) * 0.3989422804f;
      return b * (cdf + a * pdf);
    }
    case 8: return b * (1.f - a * a);                        // tanh_grad (a = y)
    case 9: return b * a * (1.f - a);                        // sigmoid_grad (a = y)
    case 10: return a > 0.f ? b : c * b;                     // leaky_relu_grad
    case 11: return (float)((a > 0.f) - (a < 0.f)) * b;      // abs_grad
    case 12: return powf(a, b);
    case 13: return std::max(a + b, 0.f);                    // add_relu
    case 14: return b / a;                                   // log_grad
    case 15: return b * 0.5f / a;                            // sqrt_grad (a = y)
    case 17: return a > 0.f ? b * c : 0.f;                   // relu_grad_c (a = y)
    default: {                                               // 16 gelu_tanh_grad
      const float k = 0.7978845608f;
      const float t = tanhf(k * (a + 0.044715f * a * a * a));
      return b * (0.5f * (1.f + t) + 0.5f * a * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * a * a));
    }
  }
}

// offsets of flat output index i in two strided operands (row-major `shape`)
struct NDIter {
  int nd;
  int64_t shape[kMaxDims], sa[kMaxDims], sb[kMaxDims];
  inline void offsets(int64_t i, int64_t& oa, int64_t& ob) const {
    oa = 0; ob = 0;
    for (int d = nd - 1; d >= 0; --d) {
      const int64_t q = i / shape[d], r = i - q * shape[d];
      oa += r * sa[d];
      ob += r * sb[d];
      i = q;
    }
  }
};

// contiguous chunks of the flat range per thread: the N-d offsets are computed once per
// chunk and then advanced like an odometer (no division per element)
template <class F>
void nd_for(const NDIter& it, int64_t n, F&& body) {
#pragma omp parallel if(n >= (1 << 16))
  {
    const int nt = omp_get_num_threads(), t = omp_get_thread_num();
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    if (lo < hi) {
      int64_t idx[kMaxDims];
      int64_t rem = lo;
      for (int d = it.nd - 1; d >= 0; --d) {
        idx[d] = rem % it.shape[d];
        rem /= it.shape[d];
      }
      int64_t oa, ob;
      it.offsets(lo, oa, ob);
      const int last = it.nd - 1;
      for (int64_t i = lo; i < hi; ++i) {
        body(i, oa, ob);
        // advance
        int d = last;
        ++idx[d];
        oa += it.sa[d];
        ob += it.sb[d];
        while (d > 0 && idx[d] == it.shape[d]) {
          oa -= it.sa[d] * it.shape[d];
          ob -= it.sb[d] * it.shape[d];
          idx[d] = 0;
          --d;
          ++idx[d];
          oa += it.sa[d];
          ob += it.sb[d];
        }
      }
    }
  }
}

NDIter make_iter(int nd, const int64_t* shape, const int64_t* sa, const int64_t* sb) {
  NDIter it{};
  it.nd = std::max(1, std::min(nd, kMaxDims));
  for (int d = 0; d < it.nd; ++d) {
    it.shape[d] = nd > 0 ? shape[d] : 1;
    it.sa[d] = nd > 0 ? sa[d] : 0;
    it.sb[d] = nd > 0 && sb ? sb[d] : 0;
  }
  return it;
}

int64_t numel(int nd, const int64_t* shape) {
  int64_t n = 1;
  for (int d = 0; d < nd; ++d) n *= shape[d];
  return n;
}

}  // namespace

// y[i] = unary(op, x[i]) over n contiguous elements (op codes of elementwise.hip)
API int hetu_cpu_unary_ext(int op, const float* x, float* y, int64_t n, float c, float c2) {
  if (op < 0 || op > 25) return -1;
#pragma omp parallel for simd schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) y[i] = unary_op(op, x[i], c, c2);
  return 0;
}

// y (contiguous, broadcast shape) = binary(op, a, b): a / b read through per-dim strides
// (0 on broadcast dims), nd <= 8
API int hetu_cpu_binary_nd(int op, const float* a, const float* b, float* y, int nd, const int64_t* shape,
                           const int64_t* sa, const int64_t* sb, float c) {
  if (op < 0 || op > 17 || nd > kMaxDims) return -1;
  const NDIter it = make_iter(nd, shape, sa, sb);
  const int64_t n = numel(nd, shape);
  nd_for(it, n, [&](int64_t i, int64_t oa, int64_t ob) { y[i] = binary_op(op, a[oa], b[ob], c); });
  return 0;
}

// dst (strided, e.g. a slice of a concat / pad output) = src (strided), nd <= 8, any
// element size (4 = fp32 / int32, 8 = int64 / double, 2 = bf16 / fp16, 1 = bytes)
API int hetu_cpu_copy_nd(const void* src, void* dst, int esize, int nd, const int64_t* shape, const int64_t* ss,
                         const int64_t* sd) {
  if (nd > kMaxDims) return -1;
  const NDIter it = make_iter(nd, shape, ss, sd);
  const int64_t n = numel(nd, shape);
  const char* s = (const char*)src;
  char* d = (char*)dst;
  switch (esize) {
    case 4:
      nd_for(it, n, [&](int64_t, int64_t os, int64_t od) { ((float*)d)[od] = ((const float*)s)[os]; });
      break;
    case 8:
      nd_for(it, n, [&](int64_t, int64_t os, int64_t od) { ((int64_t*)d)[od] = ((const int64_t*)s)[os]; });
      break;
    case 2:
      nd_for(it, n, [&](int64_t, int64_t os, int64_t od) { ((uint16_t*)d)[od] = ((const uint16_t*)s)[os]; });
      break;
    case 1:
      nd_for(it, n, [&](int64_t, int64_t os, int64_t od) { d[od] = s[os]; });
      break;
    default:
      return -1;
  }
  return 0;
}

API void hetu_cpu_fill(float* y, int64_t n, float v) {
#pragma omp parallel for simd schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) y[i] = v;
}

// row softmax over the last dim: y[r] = exp(x[r] - max) / sum (log_softmax when `log`)
API void hetu_cpu_softmax(const float* x, float* y, int64_t R, int64_t C, int log) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x + r * C;
    float* yr = y + r * C;
    float m = -INFINITY;
    for (int64_t c = 0; c < C; ++c) m = std::max(m, xr[c]);
    double s = 0.0;
    for (int64_t c = 0; c < C; ++c) s += exp((double)(xr[c] - m));
    if (log) {
      const float l = m + (float)::log(s);
      for (int64_t c = 0; c < C; ++c) yr[c] = xr[c] - l;
    } else {
      const float inv = (float)(1.0 / s);
      for (int64_t c = 0; c < C; ++c) yr[c] = expf(xr[c] - m) * inv;
    }
  }
}

// dx = y * (dy - sum(dy * y)) per row (softmax backward from the saved output)
API void hetu_cpu_softmax_bwd(const float* y, const float* dy, float* dx, int64_t R, int64_t C) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* yr = y + r * C;
    const float* gr = dy + r * C;
    double s = 0.0;
    for (int64_t c = 0; c < C; ++c) s += (double)gr[c] * yr[c];
    const float sf = (float)s;
    for (int64_t c = 0; c < C; ++c) dx[r * C + c] = yr[c] * (gr[c] - sf);
  }
}

// y = x * (u < keep) / keep, u = Philox(seed, i / 4)[i % 4] -- the GPU dropout_k mask;
// the backward is the same call on the output gradient
API void hetu_cpu_dropout(const float* x, float* y, int64_t n, float keep, int64_t seed) {
  const float inv = 1.f / keep;
  const int64_t n4 = (n + 3) / 4;
#pragma omp parallel for schedule(static) if((int64_t)(n4) * (4) >= (1 << 16))
  for (int64_t q = 0; q < n4; ++q) {
    const U4 r = philox((uint64_t)seed, (uint64_t)q);
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
    for (int k = 0; k < 4; ++k) {
      const int64_t i = q * 4 + k;
      if (i < n) y[i] = u01(rr[k]) < keep ? x[i] * inv : 0.f;
    }
  }
}

// initialisers: 0 uniform [a, b); 1 normal (mean a, std b); 2 truncated normal (mean a,
// std b, redrawn outside 2 std -- counter words of later rounds); Box-Muller on word pairs
API void hetu_cpu_random_init(float* y, int64_t n, int kind, float a, float b, int64_t seed) {
  const int64_t n4 = (n + 3) / 4;
#pragma omp parallel for schedule(static) if((int64_t)(n4) * (4) >= (1 << 16))
  for (int64_t q = 0; q < n4; ++q) {
    float v[4];
    if (kind == 0) {
      const U4 r = philox((uint64_t)seed, (uint64_t)q);
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
      for (int k = 0; k < 4; ++k) v[k] = a + (b - a) * (u01(rr[k]) - 0.5f / 16777216.0f);
    } else {
      for (int k = 0; k < 4; k += 2) {
        float z0 = 0.f, z1 = 0.f;
        for (uint64_t round = 0;; ++round) {
          const U4 r = philox((uint64_t)seed ^ (round * 0x9E3779B97F4A7C15ull), (uint64_t)q);
          const float u1 = u01(k ? r.z : r.x), u2 = u01(k ? r.w : r.y);
          const float rad = sqrtf(-2.f * logf(u1));
          z0 = rad * cosf(6.28318530718f * u2);
          z1 = rad * sinf(6.28318530718f * u2);
          if (kind == 1 || (fabsf(z0) <= 2.f && fabsf(z1) <= 2.f) || round >= 64) break;
        }
        v[k] = a + b * z0;
        v[k + 1] = a + b * z1;
      }
    }
    for (int k = 0; k < 4; ++k)
      if (q * 4 + k < n) y[q * 4 + k] = v[k];
  }
}

// y[c] = scale * sum over rows of x[r, c] with the rows split across threads and the
// partial sums combined in a fixed order (deterministic): reduce_sum over axis 0 and,
// after a permute, over any set of leading axes
API void hetu_cpu_reduce_axis0(const float* x, float* y, int64_t R, int64_t C, float scale) {
  const int nt = omp_get_max_threads();
  const int64_t chunks = std::min<int64_t>(nt, std::max<int64_t>(1, R / 16));
  double* part = new double[(size_t)chunks * C]();
#pragma omp parallel for schedule(static) if((int64_t)(chunks) * (C) >= (1 << 16))
  for (int64_t t = 0; t < chunks; ++t) {
    double* p = part + (size_t)t * C;
    const int64_t lo = R * t / chunks, hi = R * (t + 1) / chunks;
    for (int64_t r = lo; r < hi; ++r)
      for (int64_t c = 0; c < C; ++c) p[c] += x[r * C + c];
  }
#pragma omp parallel for schedule(static) if((int64_t)(C) * (R) >= (1 << 16))
  for (int64_t c = 0; c < C; ++c) {
    double s = 0.0;
    for (int64_t t = 0; t < chunks; ++t) s += part[(size_t)t * C + c];
    y[c] = (float)(s * scale);
  }
  delete[] part;
}

// y[r] = scale * sum over the last dim of x[r, :] (reduce over trailing axes)
API void hetu_cpu_reduce_lastdim(const float* x, float* y, int64_t R, int64_t C, float scale) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    double s = 0.0;
    for (int64_t c = 0; c < C; ++c) s += x[r * C + c];
    y[r] = (float)(s * scale);
  }
}

// sparse-label softmax cross-entropy: loss[r] = lse[r] - x[r, lab[r]] (0 where the label
// is ignored / out of range); the backward dx = g[r] * (softmax - onehot) on valid rows
API void hetu_cpu_softmax_ce_sparse(const float* x, const int64_t* lab, float* loss, float* lse, int64_t R,
                                    int64_t C, int64_t ignored) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x + r * C;
    float m = -INFINITY;
    for (int64_t c = 0; c < C; ++c) m = std::max(m, xr[c]);
    double s = 0.0;
    for (int64_t c = 0; c < C; ++c) s += exp((double)(xr[c] - m));
    const float l = m + (float)log(s);
    lse[r] = l;
    const int64_t y = lab[r];
    loss[r] = (y != ignored && y >= 0 && y < C) ? l - xr[y] : 0.f;
  }
}

API void hetu_cpu_softmax_ce_sparse_bwd(const float* x, const int64_t* lab, const float* g, int g_scalar,
                                        const float* lse, float* dx, int64_t R, int64_t C, int64_t ignored) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x + r * C;
    float* dr = dx + r * C;
    const int64_t y = lab[r];
    if (!(y != ignored && y >= 0 && y < C)) {
      for (int64_t c = 0; c < C; ++c) dr[c] = 0.f;
      continue;
    }
    const float gr = g_scalar ? g[0] : g[r], l = lse[r];
    for (int64_t c = 0; c < C; ++c) dr[c] = gr * expf(xr[c] - l);
    dr[y] -= gr;
  }
}
