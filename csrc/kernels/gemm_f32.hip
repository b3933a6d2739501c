// fp32 MFMA GEMM and implicit-GEMM convolution for gfx950 (CDNA4) -- the parity
// (fp32) path of the reference, whose every GEMM / convolution is fp32
// (src/common/c_runtime_api.cc:79-81; cuBLAS Sgemm in src/ops/MatrixMult.cu:22-26,
// cuDNN in src/ops/CudnnConv2d.cu:54-245).  gfx950 has no TF32/xf32: the exact-fp32
// matrix instruction v_mfma_f32_16x16x4_f32 runs at the fp32 vector rate (64 FLOP /
// clk / SIMD, MI355X_MICROARCH.md "Matrix cores"), so this kernel is MFMA-bound and
// its LDS / staging side is kept simple.
//
// Tile 128 x 128 x 16 (fp32), 256 threads = 4 waves (2 M x 2 N), each wave 64 x 64 =
// 4 x 4 MFMA 16x16x4 tiles.  Three LDS stages of 16 KiB (A and B images), filled by
// global_load_lds (16 B = 4 floats per lane), two K-tiles in flight behind a counted
// vmcnt and a raw s_barrier (a __syncthreads() would drain the DMA).
// The K index inside a 16-deep tile is permuted so that one lane's 4 MFMA steps read
// 4 CONSECUTIVE k of its row: step s, lane l uses k = 4 (l >> 4) + s -- one ds_read_b128
// per fragment set on K-contiguous images, 4 ds_read_b32 on MN-contiguous ones.
//
// Operand roles as in gemm_core.h: the MFMA's first operand is the N side, so a lane
// holds 4 consecutive output columns (16-byte stores).
#include "gemm_core.h"

namespace hetu {
namespace gemmf {

using gemm::FastDiv;
using gemm::ConvGeom;
using gemm::DgradClass;

typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 128, BN = 128, BK = 16, NT = 256, STAGES = 3;
constexpr int IMG = 128 * BK * 4;            // 8 KiB per operand image
constexpr int STAGE_BYTES = 2 * IMG;

static __device__ __attribute__((aligned(64))) float g_zero4[16];

__device__ __forceinline__ void glds16(const float* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

// ---- LDS images ------------------------------------------------------------------------
// K-major [128 rows][16 k] fp32, 64-B rows; chunk c (4 k) of row r at ((c ^ ((r >> 2) & 3)) << 4)
__device__ __forceinline__ int offk(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }
// MN-major [16 k][128 cols] fp32, 512-B rows (plain)
__device__ __forceinline__ int offmn(int k, int col) { return k * 512 + col * 4; }

// Staging slots: 2 glds per wave per operand per K-tile (8 per operand).
//  K-major : instruction i of wave w, lane l -> row 32w + 16i + (l >> 2), physical chunk
//            l & 3, logical chunk (l & 3) ^ ((row >> 2) & 3)
//  MN-major: k = 4w + 2i + (l >> 5), cols 4 (l & 31) .. +3
__device__ __forceinline__ int kslot_row(int w, int i, int l) { return 32 * w + 16 * i + (l >> 2); }
__device__ __forceinline__ int kslot_chunk(int w, int i, int l) {
  return (l & 3) ^ ((kslot_row(w, i, l) >> 2) & 3);
}
__device__ __forceinline__ int mnslot_k(int w, int i, int l) { return 4 * w + 2 * i + (l >> 5); }

#define HETU_F32_LINEAR_ROWS                                        \
  __device__ int64_t rows_eff(int64_t M_) const { return M_; }       \
  __device__ int64_t k_eff(int64_t K_) const { return K_; }          \
  __device__ int64_t out_row(int64_t m_) const { return m_; }

// plain row-major operand, K contiguous: (r, k) at base[r*ld + k]; K % 4 == 0
struct F32K {
  HETU_F32_LINEAR_ROWS
  static constexpr bool KMAJ = true;
  const float* base; int64_t ld, rows, K, bstride;
  int64_t roff[2]; bool rok[2]; int kc[2];
  __device__ void init(int64_t r0, int w, int l, int64_t batch) {
    base += batch * bstride;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = r0 + kslot_row(w, i, l);
      rok[i] = r < rows;
      roff[i] = r * ld;
      kc[i] = 4 * kslot_chunk(w, i, l);
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const int64_t k = k0 + kc[i];
    return (rok[i] && k < K) ? base + roff[i] + k : g_zero4;
  }
};

// plain operand stored [K][rows]: (r, k) at base[k*ld + r]; rows % 4 == 0
struct F32MN {
  HETU_F32_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const float* base; int64_t ld, rows, K, bstride;
  int64_t col[2]; bool cok[2]; int kk[2];
  __device__ void init(int64_t r0, int w, int l, int64_t batch) {
    base += batch * bstride;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      kk[i] = mnslot_k(w, i, l);
      col[i] = r0 + 4 * (l & 31);
      cok[i] = col[i] < rows;
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const int64_t k = k0 + kk[i];
    return (cok[i] && k < K) ? base + k * ld + col[i] : g_zero4;
  }
};

// convolution forward, M side: rows = output pixels, k = (kh, kw, ci), ci fastest; C % 4 == 0
struct F32ConvFwdA {
  HETU_F32_LINEAR_ROWS
  static constexpr bool KMAJ = true;
  const float* x; ConvGeom g; int64_t Ktot, rows;
  int nb[2], ih0[2], iw0[2], kc[2]; bool rok[2];
  __device__ void init(int64_t r0, int w, int l, int64_t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = r0 + kslot_row(w, i, l);
      rok[i] = r < rows;
      const uint32_t rr = rok[i] ? (uint32_t)r : 0;
      const uint32_t t = g.fOW.div(rr);
      const int ow = (int)(rr - t * g.OW);
      const uint32_t n = g.fOH.div(t);
      const int oh = (int)(t - n * g.OH);
      nb[i] = (int)n * g.H;
      ih0[i] = oh * g.sh - g.ph;
      iw0[i] = ow * g.sw - g.pw;
      kc[i] = 4 * kslot_chunk(w, i, l);
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const uint32_t k = (uint32_t)k0 + kc[i];
    const uint32_t tap = g.fC.div(k);
    const int ci = (int)(k - tap * g.C);
    const uint32_t kh = g.fKW.div(tap);
    const int kw = (int)(tap - kh * g.KW);
    const int ih = ih0[i] + (int)kh, iw = iw0[i] + kw;
    const bool ok = k < Ktot && rok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    return ok ? x + ((int64_t)(nb[i] + ih) * g.W + iw) * g.C + ci : g_zero4;
  }
};

// data gradient, M side over one stride class (blockIdx.y): rows = class pixels,
// k = (tap in class, co); K % 4 == 0
struct F32ConvDgradA {
  static constexpr bool KMAJ = true;
  const float* dy; ConvGeom g; DgradClass c;
  int nb[2], ii[2], jj[2], kc[2]; bool rok[2];
  int64_t mrows, kdim;
  __device__ int64_t rows_eff(int64_t) const { return mrows; }
  __device__ int64_t k_eff(int64_t) const { return kdim; }
  __device__ int64_t out_row(int64_t m) const {
    const uint32_t t = c.fWc.div((uint32_t)m);
    const int j = (int)((uint32_t)m - t * c.Wc);
    const uint32_t n = c.fHc.div(t);
    const int i = (int)(t - n * c.Hc);
    return ((int64_t)n * g.H + c.a + g.sh * i) * g.W + c.b + g.sw * j;
  }
  __device__ void init(int64_t r0, int w, int l, int64_t cls) {
    c.make(g, (int)cls);
    mrows = (int64_t)g.N * c.Hc * c.Wc;
    kdim = (int64_t)c.nth * c.ntw * g.K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = r0 + kslot_row(w, i, l);
      rok[i] = r < mrows;
      const uint32_t rr = rok[i] ? (uint32_t)r : 0;
      const uint32_t t = c.fWc.div(rr);
      const int j = (int)(rr - t * c.Wc);
      const uint32_t n = c.fHc.div(t);
      ii[i] = (int)(t - n * c.Hc) + c.cbh;
      jj[i] = j + c.cbw;
      nb[i] = (int)n * g.OH;
      kc[i] = 4 * kslot_chunk(w, i, l);
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const uint32_t k = (uint32_t)k0 + kc[i];
    const uint32_t tap = g.fK.div(k);
    const uint32_t co = k - tap * g.K;
    const uint32_t th = c.fntw.div(tap);
    const int tw = (int)(tap - th * c.ntw);
    const int oh = ii[i] - (int)th, ow = jj[i] - tw;
    const bool ok = (int64_t)k < kdim && rok[i] && (unsigned)oh < (unsigned)g.OH && (unsigned)ow < (unsigned)g.OW;
    return ok ? dy + ((int64_t)(nb[i] + oh) * g.OW + ow) * g.K + co : g_zero4;
  }
};

// data gradient, N side: cols = ci, k rows = (tap in class, co): w[co][kh][kw][ci]; C % 4 == 0
struct F32ConvDgradB {
  HETU_F32_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const float* w; ConvGeom g; DgradClass c;
  int64_t kdim; int col[2], kk[2]; bool cok[2];
  __device__ void init(int64_t r0, int wv, int l, int64_t cls) {
    c.make(g, (int)cls);
    kdim = (int64_t)c.nth * c.ntw * g.K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      kk[i] = mnslot_k(wv, i, l);
      col[i] = (int)r0 + 4 * (l & 31);
      cok[i] = col[i] < g.C;
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const uint32_t k = (uint32_t)k0 + kk[i];
    const uint32_t tap = g.fK.div(k);
    const int co = (int)(k - tap * g.K);
    const uint32_t th = c.fntw.div(tap);
    const int tw = (int)(tap - th * c.ntw);
    const int kh = c.kh0 + g.sh * (int)th, kw = c.kw0 + g.sw * tw;
    return (cok[i] && (int64_t)k < kdim) ? w + ((int64_t)co * (g.KH * g.KW) + kh * g.KW + kw) * g.C + col[i]
                                         : g_zero4;
  }
};

// weight gradient, N side: cols = (kh, kw, ci), k rows = output pixels; C % 4 == 0
struct F32ConvWgradB {
  HETU_F32_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const float* x; ConvGeom g; int64_t P;
  int kh[2], kw[2], ci[2], kk[2]; bool cok[2];
  __device__ void init(int64_t r0, int w, int l, int64_t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      kk[i] = mnslot_k(w, i, l);
      const int col = (int)r0 + 4 * (l & 31);
      cok[i] = col < g.KH * g.KW * g.C;
      const int tap = col / g.C;
      ci[i] = col - tap * g.C;
      kh[i] = tap / g.KW;
      kw[i] = tap - kh[i] * g.KW;
    }
  }
  __device__ const float* src(int64_t k0, int i) const {
    const uint32_t p = (uint32_t)k0 + kk[i];
    const uint32_t t = g.fOW.div(p);
    const int ow = (int)(p - t * g.OW);
    const uint32_t n = g.fOH.div(t);
    const int oh = (int)(t - n * g.OH);
    const int ih = oh * g.sh - g.ph + kh[i], iw = ow * g.sw - g.pw + kw[i];
    const bool ok = cok[i] && (int64_t)p < P && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
    return ok ? x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + ci[i] : g_zero4;
  }
};

struct EpiF {
  float* C; const float* Cin; const float* bias;
  int64_t ldc, ldcin, sC, sCin;
  float alpha, beta;
  int act, atomic, bias_on_m;
};

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return 0.5f * v * (1.f + erff(v * 0.70710678118f));
  return v;
}

// 4 MFMA steps' worth of one 16-row fragment: lane (row = 16 rb + (l & 15)) holds
// k = 4 (l >> 4) + s, s = 0..3
template <bool KMAJ>
__device__ __forceinline__ v4f frag(const char* img, int rb, int lane) {
  const int r = rb * 16 + (lane & 15), q = lane >> 4;
  if constexpr (KMAJ) {
    return *reinterpret_cast<const v4f*>(img + offk(r, q));
  } else {
    const float* p = reinterpret_cast<const float*>(img + offmn(4 * q, r));
    return v4f{p[0], p[128], p[256], p[384]};
  }
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <class LA, class LB>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(LA la, LB lb, EpiF ep, int64_t M, int64_t N, int64_t K,
                                                      int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  // XCD-aware bijective remap, then groups of 8 tiles along M (gemm_core.h)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = 8 * tiles_n;
  const int first_m = (wg / per_group) * 8;
  const int gsz = min(tiles_m - first_m, 8);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  const int64_t batch = blockIdx.y;
  la.init((int64_t)tm * BM, wave, lane, batch);
  lb.init((int64_t)tn * BN, wave, lane, batch);
  const int64_t Mb = la.rows_eff(M);
  if ((int64_t)tm * BM >= Mb) return;  // block-uniform, before any barrier
  K = la.k_eff(K);
  const int nk = (int)((K + BK - 1) / BK);

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt) {
    char* A = smem + (kt % STAGES) * STAGE_BYTES + 2048 * wave;
    char* B = A + IMG;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(la.src(k0, i), A + 1024 * i);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(lb.src(k0, i), B + 1024 * i);
  };

  if (nk > 0) stage(0);
  if (nk > 1) stage(1);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's DMA of K-tile kt has landed (kt+1's 4 may still fly), then every
    // wave's has (barrier); every wave also finished reading tile kt-1, whose buffer
    // the stage of kt+2 reuses
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    if (kt + 2 < nk) stage(kt + 2);
    const char* A = smem + (kt % STAGES) * STAGE_BYTES;
    const char* B = A + IMG;
    v4f mf[4], nf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) mf[i] = frag<LA::KMAJ>(A, wm * 4 + i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) nf[j] = frag<LB::KMAJ>(B, wn * 4 + j, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(nf[j][s], mf[i][s], acc[i][j], 0, 0, 0);
  }

  // epilogue: lane holds C[m][n .. n+3], m = 16-row block + (lane & 15)
  float* Cb = ep.C + batch * ep.sC;
  const float* Cinb = ep.Cin ? ep.Cin + batch * ep.sCin : nullptr;
  const bool vec = (ep.ldc & 3) == 0 && (((uintptr_t)Cb) & 15) == 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = (int64_t)tm * BM + wm * 64 + i * 16 + (lane & 15);
    if (m >= Mb) continue;
    const int64_t orow = la.out_row(m);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = (int64_t)tn * BN + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      float v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float x = acc[i][j][t] * ep.alpha;
        if (ep.bias) x += ep.bias_on_m ? ep.bias[m] : (n + t < N ? ep.bias[n + t] : 0.f);
        if (Cinb && n + t < N) x += ep.beta * Cinb[orow * ep.ldcin + n + t];
        v[t] = act_f(x, ep.act);
      }
      float* d = Cb + orow * ep.ldc + n;
      if (ep.atomic) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (n + t < N) unsafeAtomicAdd(d + t, v[t]);
      } else if (vec && n + 3 < N) {
        *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        for (int t = 0; t < 4; ++t)
          if (n + t < N) d[t] = v[t];
      }
    }
  }
}

template <class LA, class LB>
static int launch(const LA& la, const LB& lb, const EpiF& ep, int64_t M, int64_t N, int64_t K, int batch,
                  hipStream_t st) {
  const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_f32_kernel<LA, LB>), dim3(tiles_m * tiles_n, batch), dim3(NT), 0, st, la, lb, ep, M,
                     N, K, tiles_m, tiles_n);
  return (int)hipGetLastError();
}

}  // namespace gemmf
}  // namespace hetu

using namespace hetu;
using namespace hetu::gemmf;

// C[b] = alpha * op(A[b]) @ op(B[b]) (+ beta * Cin[b]) (+ bias) -> act, all fp32.
// a_kmaj: A stored [M][K] (else [K][M]); b_kmaj: B stored [N][K] (else [K][N]).
// The contiguous extent and leading dimension of each operand are multiples of 4,
// bases 16-byte aligned (checked by the caller).  accumulate: C += result (atomic).
HETU_API int hetu_gemm_f32(const float* A, const float* B, float* C, const float* Cin, const float* bias, int64_t M,
                           int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldcin, int a_kmaj,
                           int b_kmaj, int batch, int64_t sA, int64_t sB, int64_t sC, int64_t sCin, float alpha,
                           float beta, int act, int bias_on_m, int accumulate, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  EpiF ep{C, beta != 0.f ? Cin : nullptr, bias, ldc, ldcin, sC, sCin, alpha, beta, act, accumulate, bias_on_m};
  if (a_kmaj && b_kmaj)
    return launch(F32K{A, lda, M, K, sA}, F32K{B, ldb, N, K, sB}, ep, M, N, K, batch, st);
  if (a_kmaj)
    return launch(F32K{A, lda, M, K, sA}, F32MN{B, ldb, N, K, sB}, ep, M, N, K, batch, st);
  if (b_kmaj)
    return launch(F32MN{A, lda, M, K, sA}, F32K{B, ldb, N, K, sB}, ep, M, N, K, batch, st);
  return launch(F32MN{A, lda, M, K, sA}, F32MN{B, ldb, N, K, sB}, ep, M, N, K, batch, st);
}

// y[N,OH,OW,K] = conv(x[N,H,W,C], w[K,KH,KW,C]) (+bias) -> act; NHWC fp32, C % 4 == 0
HETU_API int hetu_conv_fwd_f32(const float* x, const float* w, float* y, const float* bias, int N, int H, int W,
                               int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, int act,
                               hipStream_t st) {
  ConvGeom g = gemm::geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  const int64_t M = (int64_t)N * g.OH * g.OW, Kt = (int64_t)KH * KW * C;
  EpiF ep{y, nullptr, bias, K, 0, 0, 0, 1.f, 0.f, act, 0, 0};
  if (KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0)
    return launch(F32K{x, C, M, C, 0}, F32K{w, C, K, C, 0}, ep, M, K, C, 1, st);
  F32ConvFwdA la{};
  la.x = x;
  la.g = g;
  la.Ktot = Kt;
  la.rows = M;
  return launch(la, F32K{w, Kt, K, Kt, 0}, ep, M, K, Kt, 1, st);
}

// dx[N,H,W,C] (+)= conv_transpose(dy[N,OH,OW,K], w[K,KH,KW,C]); K % 4 == 0, C % 4 == 0.
// acc (optional, may alias dx) is added in the epilogue.
HETU_API int hetu_conv_dgrad_f32(const float* dy, const float* w, float* dx, const float* acc, int N, int H, int W,
                                 int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, hipStream_t st) {
  ConvGeom g = gemm::geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  EpiF ep{dx, acc, nullptr, C, C, 0, 0, 1.f, acc ? 1.f : 0.f, 0, 0, 0};
  if (KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0) {
    const int64_t M = (int64_t)N * H * W;
    return launch(F32K{dy, K, M, K, 0}, F32MN{w, C, C, K, 0}, ep, M, C, K, 1, st);
  }
  const int64_t Mmax = (int64_t)N * ((H + sh - 1) / sh) * ((W + sw - 1) / sw);
  const int64_t Kmax = (int64_t)((KH + sh - 1) / sh) * ((KW + sw - 1) / sw) * K;
  F32ConvDgradA la{};
  la.dy = dy;
  la.g = g;
  F32ConvDgradB lb{};
  lb.w = w;
  lb.g = g;
  // the sh*sw stride classes partition the input pixels: every dx element is stored
  return launch(la, lb, ep, Mmax, C, Kmax, sh * sw, st);
}

// dw[K, KH*KW*C] (+)= sum over output pixels dy^T x_im2col (fp32); accumulate adds into dw
HETU_API int hetu_conv_wgrad_f32(const float* dy, const float* x, float* dw, int N, int H, int W, int C, int K,
                                 int KH, int KW, int sh, int sw, int ph, int pw, int accumulate, hipStream_t st) {
  ConvGeom g = gemm::geom(N, H, W, C, K, KH, KW, sh, sw, ph, pw);
  const int64_t P = (int64_t)N * g.OH * g.OW, Nc = (int64_t)KH * KW * C;
  EpiF ep{dw, accumulate ? dw : nullptr, nullptr, Nc, Nc, 0, 0, 1.f, accumulate ? 1.f : 0.f, 0, 0, 0};
  F32MN la{dy, K, K, P, 0};
  if (KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0)
    return launch(la, F32MN{x, C, C, P, 0}, ep, K, Nc, P, 1, st);
  F32ConvWgradB lb{};
  lb.x = x;
  lb.g = g;
  lb.P = P;
  return launch(la, lb, ep, K, Nc, P, 1, st);
}
