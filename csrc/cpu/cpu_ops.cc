// Native CPU backend (C++ / OpenMP) -- the role of the reference's DNNL / OpenMP
// kernels (src/dnnl_ops/*.cpp: MatrixMult.cpp:19-55, Softmax*, Relu*, ReduceSum*,
// Optimizers, EmbeddingLookup).  fp32, row-major,
// OpenMP over rows / blocks; the GEMM packs a K x N panel of B per thread block
// so the inner loop streams contiguous, auto-vectorised rows.
//
// C ABI, loaded by hetu_61a7_amd/kernels/cpu_native.py; selected with
// HETU_CPU_BACKEND=native for CPU executors (the BASELINE "logreg MNIST on the
// CPU path" configuration).
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int64_t MB = 64, NB = 256, KB = 256;

inline float at(const float* X, int64_t r, int64_t c, int64_t ld, int trans) {
  return trans ? X[c * ld + r] : X[r * ld + c];
}

// Skinny products (logistic regression 784 -> 10 and its weight gradient): B packed once
// into zero-padded rows of NP = 16 / 32 floats, 16-row blocks of C accumulated over the
// whole K in a stack tile with a fixed-width inner loop (one or two AVX-512 FMAs per (row, k);
// cloned for AVX-512 / AVX2 / baseline at load time), rows split over the threads from ~1M MACs.
template <int NP>
__attribute__((target_clones("avx512f", "avx2", "default")))
static void skinny_rows(const float* A, const float* bp, float* C, const float* bias, int64_t i0, int64_t i1,
                        int64_t N, int64_t K, int64_t lda, int64_t ldc, int transA, float alpha, float beta) {
  float acc[16][NP];
  for (int64_t i = 0; i < 16; ++i)
    for (int j = 0; j < NP; ++j) acc[i][j] = 0.f;
  const int64_t nr = i1 - i0;
  for (int64_t k = 0; k < K; ++k) {
    const float* __restrict__ b = bp + k * NP;
    for (int64_t r = 0; r < nr; ++r) {
      const float av = transA ? A[k * lda + i0 + r] : A[(i0 + r) * lda + k];
#pragma omp simd
      for (int j = 0; j < NP; ++j) acc[r][j] += av * b[j];
    }
  }
  for (int64_t r = 0; r < nr; ++r) {
    float* c = C + (i0 + r) * ldc;
    for (int64_t j = 0; j < N; ++j) {
      float v = alpha * acc[r][j] + (beta == 0.f ? 0.f : beta * c[j]);
      if (bias != nullptr) v += bias[j];
      c[j] = v;
    }
  }
}

static void skinny_gemm(const float* A, const float* B, float* C, const float* bias, int64_t M, int64_t N,
                        int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int transA, float alpha, float beta) {
  const int NP = N <= 16 ? 16 : 32;
  std::vector<float> bp((size_t)K * NP, 0.f);
  for (int64_t k = 0; k < K; ++k) memcpy(bp.data() + k * NP, B + k * ldb, N * sizeof(float));
  const int64_t nblk = (M + 15) / 16;
#pragma omp parallel for schedule(static) if (M * N * K >= (1 << 20))
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const int64_t i0 = blk * 16, i1 = std::min(M, i0 + 16);
    if (NP == 16)
      skinny_rows<16>(A, bp.data(), C, bias, i0, i1, N, K, lda, ldc, transA, alpha, beta);
    else
      skinny_rows<32>(A, bp.data(), C, bias, i0, i1, N, K, lda, ldc, transA, alpha, beta);
  }
}

}  // namespace

// C[M,N] = alpha * op(A)[M,K] @ op(B)[K,N] + beta * C (+ bias[N])
API void hetu_cpu_gemm(const float* A, const float* B, float* C, const float* bias, int64_t M, int64_t N,
                       int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int transA, int transB, float alpha,
                       float beta) {
  if (N <= 32 && !transB) {
    skinny_gemm(A, B, C, bias, M, N, K, lda, ldb, ldc, transA, alpha, beta);
    return;
  }
  const int64_t mblocks = (M + MB - 1) / MB, nblocks = (N + NB - 1) / NB;
#pragma omp parallel if(M * N * K >= (1 << 21))
  {
    std::vector<float> bp((size_t)KB * NB);   // packed B panel [kb][nb]
    std::vector<float> ap((size_t)MB * KB);   // packed A block [mb][kb]
#pragma omp for collapse(2) schedule(static)
    for (int64_t mb = 0; mb < mblocks; ++mb) {
      for (int64_t nb = 0; nb < nblocks; ++nb) {
        const int64_t m0 = mb * MB, m1 = std::min(M, m0 + MB);
        const int64_t n0 = nb * NB, n1 = std::min(N, n0 + NB), nn = n1 - n0;
        for (int64_t i = m0; i < m1; ++i) {
          float* c = C + i * ldc + n0;
          if (beta == 0.f) {
            for (int64_t j = 0; j < nn; ++j) c[j] = 0.f;
          } else if (beta != 1.f) {
            for (int64_t j = 0; j < nn; ++j) c[j] *= beta;
          }
        }
        for (int64_t k0 = 0; k0 < K; k0 += KB) {
          const int64_t k1 = std::min(K, k0 + KB), kk = k1 - k0;
          for (int64_t k = 0; k < kk; ++k) {
            float* dst = bp.data() + k * NB;
            if (!transB) {
              memcpy(dst, B + (k0 + k) * ldb + n0, nn * sizeof(float));
            } else {
              for (int64_t j = 0; j < nn; ++j) dst[j] = B[(n0 + j) * ldb + k0 + k];
            }
          }
          for (int64_t i = m0; i < m1; ++i)
            for (int64_t k = 0; k < kk; ++k) ap[(i - m0) * KB + k] = alpha * at(A, i, k0 + k, lda, transA);
          for (int64_t i = m0; i < m1; ++i) {
            float* __restrict__ c = C + i * ldc + n0;
            const float* __restrict__ a = ap.data() + (i - m0) * KB;
            for (int64_t k = 0; k < kk; ++k) {
              const float av = a[k];
              const float* __restrict__ b = bp.data() + k * NB;
#pragma omp simd
              for (int64_t j = 0; j < nn; ++j) c[j] += av * b[j];
            }
          }
        }
        if (bias != nullptr)
          for (int64_t i = m0; i < m1; ++i)
            for (int64_t j = n0; j < n1; ++j) C[i * ldc + j] += bias[j];
      }
    }
  }
}

// loss[r] = -sum_c y[r,c] * log_softmax(x)[r,c]; lse[r] saved for the backward
API void hetu_cpu_softmax_ce(const float* x, const float* y, float* loss, float* lse, int64_t R, int64_t C) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x + r * C;
    const float* yr = y + r * C;
    float m = -INFINITY;
    for (int64_t c = 0; c < C; ++c) m = std::max(m, xr[c]);
    double s = 0.0;
    for (int64_t c = 0; c < C; ++c) s += exp((double)(xr[c] - m));
    const float l = m + (float)log(s);
    double acc = 0.0;
    for (int64_t c = 0; c < C; ++c) acc += (double)yr[c] * (double)(l - xr[c]);
    loss[r] = (float)acc;
    if (lse) lse[r] = l;
  }
}

// dx[r,c] = g[r] * (softmax(x)[r,c] * sum_c y - y[r,c])
API void hetu_cpu_softmax_ce_bwd(const float* x, const float* y, const float* g, const float* lse, float* dx,
                                 int64_t R, int64_t C, int g_scalar) {
#pragma omp parallel for schedule(static) if((int64_t)(R) * (C) >= (1 << 16))
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x + r * C;
    const float* yr = y + r * C;
    float ys = 0.f;
    for (int64_t c = 0; c < C; ++c) ys += yr[c];
    const float gr = g_scalar ? g[0] : g[r];
    const float l = lse[r];
    for (int64_t c = 0; c < C; ++c) dx[r * C + c] = gr * (expf(xr[c] - l) * ys - yr[c]);
  }
}

// elementwise: op 0 relu, 1 sigmoid, 2 tanh, 3 gelu(erf), 4 exp, 5 sqrt
API void hetu_cpu_unary(int op, const float* x, float* y, int64_t n) {
#pragma omp parallel for simd schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) {
    const float v = x[i];
    float r;
    switch (op) {
      case 0: r = v > 0.f ? v : 0.f; break;
      case 1: r = 1.f / (1.f + expf(-v)); break;
      case 2: r = tanhf(v); break;
      case 3: r = 0.5f * v * (1.f + erff(v * 0.70710678f)); break;
      case 4: r = expf(v); break;
      default: r = sqrtf(v); break;
    }
    y[i] = r;
  }
}

// relu'(x) * g
API void hetu_cpu_relu_grad(const float* x, const float* g, float* y, int64_t n) {
#pragma omp parallel for simd schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) y[i] = x[i] > 0.f ? g[i] : 0.f;
}

// y[c] = scale * sum_r x[r, c]
API void hetu_cpu_reduce_rows(const float* x, float* y, int64_t R, int64_t C, float scale) {
  const int nt = omp_get_max_threads();
  std::vector<double> part((size_t)nt * C, 0.0);
#pragma omp parallel if(R * C >= (1 << 16))
  {
    double* p = part.data() + (size_t)omp_get_thread_num() * C;
#pragma omp for schedule(static)
    for (int64_t r = 0; r < R; ++r)
      for (int64_t c = 0; c < C; ++c) p[c] += x[r * C + c];
  }
  for (int64_t c = 0; c < C; ++c) {
    double s = 0.0;
    for (int t = 0; t < nt; ++t) s += part[(size_t)t * C + c];
    y[c] = (float)(s * scale);
  }
}

// out[i, :] = table[ids[i], :] (out-of-range ids -> 0)
API void hetu_cpu_gather_rows(const float* table, const int64_t* ids, float* out, int64_t n, int64_t dim,
                              int64_t rows) {
#pragma omp parallel for schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) {
    const int64_t id = ids[i];
    if (id >= 0 && id < rows)
      memcpy(out + i * dim, table + id * dim, dim * sizeof(float));
    else
      memset(out + i * dim, 0, dim * sizeof(float));
  }
}

// flat optimizers (same modes / semantics as optimizer.hip): 0 sgd 1 momentum
// 2 nesterov 3 adagrad 4 adam 5 adamw
API void hetu_cpu_optimizer(int mode, float* p, const float* g, float* s1, float* s2, int64_t n, float lr, float l2,
                            float mu, float b1, float b2, float b1t, float b2t, float eps, float wd, float gscale) {
#pragma omp parallel for simd schedule(static) if((int64_t)(n) >= (1 << 16))
  for (int64_t i = 0; i < n; ++i) {
    const float gr = g[i] * gscale + l2 * p[i];
    switch (mode) {
      case 0: p[i] -= lr * gr; break;
      case 1: s1[i] = mu * s1[i] - lr * gr; p[i] += s1[i]; break;
      case 2: {
        const float t = lr * gr;
        s1[i] = (s1[i] - t) * mu;
        p[i] += s1[i] - t;
        break;
      }
      case 3: s1[i] += gr * gr; p[i] -= lr * gr / (sqrtf(s1[i]) + eps); break;
      default: {
        s1[i] = b1 * s1[i] + (1.f - b1) * gr;
        s2[i] = b2 * s2[i] + (1.f - b2) * gr * gr;
        const float u = (s1[i] / (1.f - b1t)) / (sqrtf(s2[i] / (1.f - b2t)) + eps);
        p[i] -= lr * (mode == 5 ? u + wd * p[i] : u);
      }
    }
  }
}

API int hetu_cpu_num_threads() { return omp_get_max_threads(); }

// ---- convolution (NCHW fp32) ------------------------------------------------------------
// The reference's DNNL convolution (src/dnnl_ops/Conv2d.cpp): here im2col of one image
// into a [C*KH*KW][OH*OW] panel and the packed GEMM above, images in sequence (the GEMM
// is OpenMP-parallel over its output blocks); the data gradient is the transposed GEMM
// followed by col2im, the filter gradient accumulates dy[n] @ col[n]^T over images.
namespace {

struct ConvShape {
  int64_t N, C, H, W, K, KH, KW, sh, sw, ph, pw, OH, OW;
  int64_t ckk() const { return C * KH * KW; }
  int64_t ohw() const { return OH * OW; }
};

void im2col(const ConvShape& s, const float* x, float* col) {
#pragma omp parallel for collapse(2) schedule(static) if(s.ckk() * s.ohw() >= (1 << 16))
  for (int64_t c = 0; c < s.C; ++c)
    for (int64_t kh = 0; kh < s.KH; ++kh)
      for (int64_t kw = 0; kw < s.KW; ++kw) {
        float* dst = col + ((c * s.KH + kh) * s.KW + kw) * s.ohw();
        for (int64_t oh = 0; oh < s.OH; ++oh) {
          const int64_t ih = oh * s.sh - s.ph + kh;
          for (int64_t ow = 0; ow < s.OW; ++ow) {
            const int64_t iw = ow * s.sw - s.pw + kw;
            dst[oh * s.OW + ow] = (ih >= 0 && ih < s.H && iw >= 0 && iw < s.W) ? x[(c * s.H + ih) * s.W + iw] : 0.f;
          }
        }
      }
}

// dx[c] += col scattered back (each channel owned by one thread: no races)
void col2im(const ConvShape& s, const float* col, float* dx) {
#pragma omp parallel for schedule(static) if(s.ckk() * s.ohw() >= (1 << 16))
  for (int64_t c = 0; c < s.C; ++c)
    for (int64_t kh = 0; kh < s.KH; ++kh)
      for (int64_t kw = 0; kw < s.KW; ++kw) {
        const float* src = col + ((c * s.KH + kh) * s.KW + kw) * s.ohw();
        for (int64_t oh = 0; oh < s.OH; ++oh) {
          const int64_t ih = oh * s.sh - s.ph + kh;
          if (ih < 0 || ih >= s.H) continue;
          for (int64_t ow = 0; ow < s.OW; ++ow) {
            const int64_t iw = ow * s.sw - s.pw + kw;
            if (iw >= 0 && iw < s.W) dx[(c * s.H + ih) * s.W + iw] += src[oh * s.OW + ow];
          }
        }
      }
}

ConvShape conv_shape(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t KH, int64_t KW, int64_t sh,
                     int64_t sw, int64_t ph, int64_t pw) {
  ConvShape s{N, C, H, W, K, KH, KW, sh, sw, ph, pw, 0, 0};
  s.OH = (H + 2 * ph - KH) / sh + 1;
  s.OW = (W + 2 * pw - KW) / sw + 1;
  return s;
}

}  // namespace

// y[N][K][OH][OW] = conv(x[N][C][H][W], w[K][C][KH][KW]) (+ bias[K])
API void hetu_cpu_conv2d(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C,
                         int64_t H, int64_t W, int64_t K, int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t ph,
                         int64_t pw) {
  const ConvShape s = conv_shape(N, C, H, W, K, KH, KW, sh, sw, ph, pw);
  std::vector<float> col((size_t)s.ckk() * s.ohw());
  for (int64_t n = 0; n < N; ++n) {
    im2col(s, x + n * C * H * W, col.data());
    float* yn = y + n * K * s.ohw();
    hetu_cpu_gemm(w, col.data(), yn, nullptr, K, s.ohw(), s.ckk(), s.ckk(), s.ohw(), s.ohw(), 0, 0, 1.f, 0.f);
    if (bias) {
#pragma omp parallel for schedule(static) if(K * s.ohw() >= (1 << 16))
      for (int64_t k = 0; k < K; ++k)
        for (int64_t i = 0; i < s.ohw(); ++i) yn[k * s.ohw() + i] += bias[k];
    }
  }
}

// dx[N][C][H][W] = conv^T(dy, w)
API void hetu_cpu_conv2d_bwd_data(const float* dy, const float* w, float* dx, int64_t N, int64_t C, int64_t H,
                                  int64_t W, int64_t K, int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t ph,
                                  int64_t pw) {
  const ConvShape s = conv_shape(N, C, H, W, K, KH, KW, sh, sw, ph, pw);
  std::vector<float> col((size_t)s.ckk() * s.ohw());
  memset(dx, 0, sizeof(float) * N * C * H * W);
  for (int64_t n = 0; n < N; ++n) {
    // col[ckk][ohw] = w^T [ckk][K] @ dy[n] [K][ohw]
    hetu_cpu_gemm(w, dy + n * K * s.ohw(), col.data(), nullptr, s.ckk(), s.ohw(), K, s.ckk(), s.ohw(), s.ohw(), 1,
                  0, 1.f, 0.f);
    col2im(s, col.data(), dx + n * C * H * W);
  }
}

// dw[K][C][KH][KW] = sum_n dy[n] @ im2col(x[n])^T; db[K] = sum dy (nullable)
API void hetu_cpu_conv2d_bwd_filter(const float* dy, const float* x, float* dw, float* db, int64_t N, int64_t C,
                                    int64_t H, int64_t W, int64_t K, int64_t KH, int64_t KW, int64_t sh, int64_t sw,
                                    int64_t ph, int64_t pw) {
  const ConvShape s = conv_shape(N, C, H, W, K, KH, KW, sh, sw, ph, pw);
  std::vector<float> col((size_t)s.ckk() * s.ohw());
  for (int64_t n = 0; n < N; ++n) {
    im2col(s, x + n * C * H * W, col.data());
    hetu_cpu_gemm(dy + n * K * s.ohw(), col.data(), dw, nullptr, K, s.ckk(), s.ohw(), s.ohw(), s.ohw(), s.ckk(), 0,
                  1, 1.f, n == 0 ? 0.f : 1.f);
  }
  if (db) {
#pragma omp parallel for schedule(static) if(N * K * s.ohw() >= (1 << 16))
    for (int64_t k = 0; k < K; ++k) {
      double a = 0.0;
      for (int64_t n = 0; n < N; ++n)
        for (int64_t i = 0; i < s.ohw(); ++i) a += dy[(n * K + k) * s.ohw() + i];
      db[k] = (float)a;
    }
  }
}

// ---- pooling (NCHW fp32; reference src/dnnl_ops/MaxPool.cpp, AvgPool.cpp) ----------------
// max: idx[N*C*OH*OW] keeps the argmax input offset inside the plane for the backward
API void hetu_cpu_maxpool2d(const float* x, float* y, int32_t* idx, int64_t NC, int64_t H, int64_t W, int64_t KH,
                            int64_t KW, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t OH, int64_t OW) {
#pragma omp parallel for schedule(static) if((int64_t)(NC) * (H * W) >= (1 << 16))
  for (int64_t p = 0; p < NC; ++p) {
    const float* xp = x + p * H * W;
    for (int64_t oh = 0; oh < OH; ++oh)
      for (int64_t ow = 0; ow < OW; ++ow) {
        float m = -INFINITY;
        int32_t mi = -1;
        for (int64_t kh = 0; kh < KH; ++kh) {
          const int64_t ih = oh * sh - ph + kh;
          if (ih < 0 || ih >= H) continue;
          for (int64_t kw = 0; kw < KW; ++kw) {
            const int64_t iw = ow * sw - pw + kw;
            if (iw < 0 || iw >= W) continue;
            const float v = xp[ih * W + iw];
            if (v > m || mi < 0) { m = v; mi = (int32_t)(ih * W + iw); }
          }
        }
        y[(p * OH + oh) * OW + ow] = m;
        idx[(p * OH + oh) * OW + ow] = mi;
      }
  }
}

API void hetu_cpu_maxpool2d_bwd(const float* dy, const int32_t* idx, float* dx, int64_t NC, int64_t H, int64_t W,
                                int64_t OH, int64_t OW) {
#pragma omp parallel for schedule(static) if((int64_t)(NC) * (H * W) >= (1 << 16))
  for (int64_t p = 0; p < NC; ++p) {
    float* dp = dx + p * H * W;
    memset(dp, 0, sizeof(float) * H * W);
    for (int64_t o = 0; o < OH * OW; ++o) {
      const int32_t i = idx[p * OH * OW + o];
      if (i >= 0) dp[i] += dy[p * OH * OW + o];
    }
  }
}

// average over the window including padding (count_include_pad, the reference's cuDNN mode)
API void hetu_cpu_avgpool2d(const float* x, float* y, int64_t NC, int64_t H, int64_t W, int64_t KH, int64_t KW,
                            int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t OH, int64_t OW) {
  const float inv = 1.f / (float)(KH * KW);
#pragma omp parallel for schedule(static) if((int64_t)(NC) * (H * W) >= (1 << 16))
  for (int64_t p = 0; p < NC; ++p) {
    const float* xp = x + p * H * W;
    for (int64_t oh = 0; oh < OH; ++oh)
      for (int64_t ow = 0; ow < OW; ++ow) {
        float a = 0.f;
        for (int64_t kh = 0; kh < KH; ++kh) {
          const int64_t ih = oh * sh - ph + kh;
          if (ih < 0 || ih >= H) continue;
          for (int64_t kw = 0; kw < KW; ++kw) {
            const int64_t iw = ow * sw - pw + kw;
            if (iw >= 0 && iw < W) a += xp[ih * W + iw];
          }
        }
        y[(p * OH + oh) * OW + ow] = a * inv;
      }
  }
}

API void hetu_cpu_avgpool2d_bwd(const float* dy, float* dx, int64_t NC, int64_t H, int64_t W, int64_t KH, int64_t KW,
                                int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t OH, int64_t OW) {
  const float inv = 1.f / (float)(KH * KW);
#pragma omp parallel for schedule(static) if((int64_t)(NC) * (H * W) >= (1 << 16))
  for (int64_t p = 0; p < NC; ++p) {
    float* dp = dx + p * H * W;
    memset(dp, 0, sizeof(float) * H * W);
    for (int64_t oh = 0; oh < OH; ++oh)
      for (int64_t ow = 0; ow < OW; ++ow) {
        const float g = dy[(p * OH + oh) * OW + ow] * inv;
        for (int64_t kh = 0; kh < KH; ++kh) {
          const int64_t ih = oh * sh - ph + kh;
          if (ih < 0 || ih >= H) continue;
          for (int64_t kw = 0; kw < KW; ++kw) {
            const int64_t iw = ow * sw - pw + kw;
            if (iw >= 0 && iw < W) dp[ih * W + iw] += g;
          }
        }
      }
  }
}

// ---- batch normalisation (NCHW fp32; reference src/dnnl_ops/BatchNorm.cpp) -------------
// training: batch statistics (biased variance for the normalisation), running stats
// updated with `momentum` (unbiased variance, the PyTorch convention); saves mean / rstd
API void hetu_cpu_batchnorm(const float* x, const float* gamma, const float* beta, float* y, float* run_mean,
                            float* run_var, float* save_mean, float* save_rstd, int64_t N, int64_t C, int64_t HW,
                            float momentum, float eps, int training) {
#pragma omp parallel for schedule(static) if((int64_t)(C) * (N * HW) >= (1 << 16))
  for (int64_t c = 0; c < C; ++c) {
    float mean, rstd;
    if (training) {
      double s = 0.0, q = 0.0;
      for (int64_t n = 0; n < N; ++n) {
        const float* xp = x + (n * C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) { s += xp[i]; q += (double)xp[i] * xp[i]; }
      }
      const double cnt = (double)N * HW;
      const double m = s / cnt;
      const double var = std::max(0.0, q / cnt - m * m);
      mean = (float)m;
      rstd = (float)(1.0 / sqrt(var + eps));
      if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
      if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)(var * cnt / std::max(1.0, cnt - 1));
    } else {
      mean = run_mean[c];
      rstd = 1.f / sqrtf(run_var[c] + eps);
    }
    if (save_mean) save_mean[c] = mean;
    if (save_rstd) save_rstd[c] = rstd;
    const float a = gamma[c] * rstd, b = beta[c] - mean * a;
    for (int64_t n = 0; n < N; ++n) {
      const float* xp = x + (n * C + c) * HW;
      float* yp = y + (n * C + c) * HW;
      for (int64_t i = 0; i < HW; ++i) yp[i] = xp[i] * a + b;
    }
  }
}

// dx = gamma*rstd/M * (M*dy - sum(dy) - xhat*sum(dy*xhat)); dgamma = sum(dy*xhat); dbeta = sum(dy)
API void hetu_cpu_batchnorm_bwd(const float* dy, const float* x, const float* gamma, const float* save_mean,
                                const float* save_rstd, float* dx, float* dgamma, float* dbeta, int64_t N, int64_t C,
                                int64_t HW) {
#pragma omp parallel for schedule(static) if((int64_t)(C) * (N * HW) >= (1 << 16))
  for (int64_t c = 0; c < C; ++c) {
    const float mean = save_mean[c], rstd = save_rstd[c];
    double sg = 0.0, sgx = 0.0;
    for (int64_t n = 0; n < N; ++n) {
      const float* xp = x + (n * C + c) * HW;
      const float* gp = dy + (n * C + c) * HW;
      for (int64_t i = 0; i < HW; ++i) { sg += gp[i]; sgx += (double)gp[i] * (xp[i] - mean) * rstd; }
    }
    dgamma[c] = (float)sgx;
    dbeta[c] = (float)sg;
    const double M = (double)N * HW;
    const float k = gamma[c] * rstd;
    const float mg = (float)(sg / M), mgx = (float)(sgx / M);
    for (int64_t n = 0; n < N; ++n) {
      const float* xp = x + (n * C + c) * HW;
      const float* gp = dy + (n * C + c) * HW;
      float* dp = dx + (n * C + c) * HW;
      for (int64_t i = 0; i < HW; ++i) dp[i] = k * (gp[i] - mg - (xp[i] - mean) * rstd * mgx);
    }
  }
}
