// bf16 MFMA GEMM for gfx950 (CDNA4): the plain-operand C API (all four transpose
// modes, batched, beta / bias / activation epilogues, split-K) over the kernels of
// gemm_core.h, and the split-K slab reducers.
//
// Replaces the reference's cuBLAS Sgemm / SgemmStridedBatched call sites
// (src/ops/MatrixMult.cu:22-26, BatchMatrixMult.cu:31-36, Linear.cu:50-55,
// Addmm.cu:29, Baddbmm.cu:37), SURVEY.md §2.7.  This unit instantiates the
// K % 64 == 0 kernels; gemm_ktail.hip the ragged-K ones.
#include "gemm_core.h"

namespace hetu {
namespace gemm {
template int launch_buf<true>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t, const Epi&,
                              int64_t, int64_t, int64_t, int, int, hipStream_t, int);
}  // namespace gemm
}  // namespace hetu

using namespace hetu;
using namespace hetu::gemm;

// C[b] = alpha * op(A[b]) @ op(B[b]) (+ beta * Cin[b]) (+ bias) -> act.
// a_kmaj: A stored [M][K] (else [K][M]); b_kmaj: B stored [N][K] (else [K][N]).
// Requirements (checked by the caller): the contiguous dim of each operand and its
// leading dimension are multiples of 8 elements, 16-byte aligned bases.
static int gemm_bf16_impl(const void* A, const void* B, void* C, const void* Cin,
                          const float* bias, int64_t M, int64_t N, int64_t K, int64_t lda,
                          int64_t ldb, int64_t ldc, int64_t ldcin, int a_kmaj, int b_kmaj,
                          int batch, int64_t sA, int64_t sB, int64_t sC, int64_t sCin,
                          float alpha, float beta, int act, int out_f32, int cin_f32,
                          int bias_on_m, int splitk, int atomic, float* ws, int tile, void* C2,
                          float drop_keep, uint64_t drop_seed, hipStream_t st, const void* gmask = nullptr,
                          float gmask_scale = 1.f, int gmask_bits = 0, uint8_t* mbits_out = nullptr) {
  Epi ep{C, Cin, bias, ldc, ldcin, sC, sCin, alpha, beta, act, out_f32, cin_f32, atomic,
         bias_on_m, ws, 0};
  ep.C2 = C2;
  ep.drop_keep = drop_keep < 1.f ? drop_keep : 0.f;
  ep.drop_seed = drop_seed;
  ep.drop_off = ep.drop_keep > 0.f ? hetu_rng_offset_ptr() : nullptr;
  ep.gmask = gmask;
  ep.gmask_scale = gmask_scale;
  ep.gmask_bits = gmask ? gmask_bits : 0;
  ep.mbits_out = ep.drop_keep > 0.f ? mbits_out : nullptr;
  if ((ep.gmask_bits || mbits_out) && ldc % 8) return (int)hipErrorInvalidValue;
  if (mbits_out && !ep.mbits_out) return (int)hipErrorInvalidValue;
  if ((C2 || ep.drop_keep > 0.f || gmask) && (splitk > 1 || atomic)) return (int)hipErrorInvalidValue;
  if (gmask && (batch != 1 || out_f32 || ((uintptr_t)gmask & 15))) return (int)hipErrorInvalidValue;
  if (ep.drop_keep > 0.f && (N % 8 || batch != 1)) return (int)hipErrorInvalidValue;
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  if (M <= 0 || N <= 0) return 0;
  // buffer-descriptor loaders address each operand slice with 32-bit offsets (< 2 GiB);
  // a larger K-major A is processed in row chunks (A, C, Cin and a per-row bias advance)
  const int64_t bbytes = (b_kmaj ? (N - 1) * ldb + K : (K - 1) * ldb + N) * 2;
  const int64_t abytes = (a_kmaj ? (M - 1) * lda + K : (K - 1) * lda + M) * 2;
  if (bbytes >= (1ll << 31)) return (int)hipErrorInvalidValue;
  if (abytes >= (1ll << 31)) {
    if (!a_kmaj || batch != 1 || ep.slab || splitk > 1 || ep.drop_keep > 0.f || gmask) return (int)hipErrorInvalidValue;
    const int64_t rows = std::max<int64_t>(BIG, ((((1ll << 30) / (lda * 2)) / BIG) * BIG));
    for (int64_t m0 = 0; m0 < M; m0 += rows) {
      const int64_t mc = std::min(rows, M - m0);
      Epi e = ep;
      e.C = (char*)ep.C + m0 * ep.ldc * (ep.out_f32 ? 4 : 2);
      if (ep.C2) e.C2 = (char*)ep.C2 + m0 * ep.ldc * 2;
      if (ep.Cin) e.Cin = (const char*)ep.Cin + m0 * ep.ldcin * (ep.cin_f32 ? 4 : 2);
      if (ep.bias && ep.bias_on_m) e.bias = ep.bias + m0;
      const int rc = K % BK == 0 ? launch_buf<true>(a + m0 * lda, b, 1, b_kmaj, lda, ldb, 0, sB, e, mc, N, K, 1, 1, st, tile)
                                 : launch_buf<false>(a + m0 * lda, b, 1, b_kmaj, lda, ldb, 0, sB, e, mc, N, K, 1, 1, st, tile);
      if (rc) return rc;
    }
    return 0;
  }
  if (K % BK == 0) return launch_buf<true>(a, b, a_kmaj, b_kmaj, lda, ldb, sA, sB, ep, M, N, K, batch, splitk, st, tile);
  return launch_buf<false>(a, b, a_kmaj, b_kmaj, lda, ldb, sA, sB, ep, M, N, K, batch, splitk, st, tile);
}

HETU_API int hetu_gemm_bf16(const void* A, const void* B, void* C, const void* Cin,
                            const float* bias, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, int64_t ldcin, int a_kmaj, int b_kmaj,
                            int batch, int64_t sA, int64_t sB, int64_t sC, int64_t sCin,
                            float alpha, float beta, int act, int out_f32, int cin_f32,
                            int bias_on_m, int splitk, int atomic, float* ws, int tile, hipStream_t st) {
  return gemm_bf16_impl(A, B, C, Cin, bias, M, N, K, lda, ldb, ldc, ldcin, a_kmaj, b_kmaj, batch, sA, sB, sC, sCin,
                        alpha, beta, act, out_f32, cin_f32, bias_on_m, splitk, atomic, ws, tile, nullptr, 0.f, 0, st);
}

// bf16 C = dropout(act(A @ B + bias)) with the optional pre-activation copy C2 (nullable)
// or the dropout (keep >= 1: none) in the same epilogue -- not both (hipErrorInvalidValue)
HETU_API int hetu_gemm_bf16_ex(const void* A, const void* B, void* C, void* C2, const float* bias, int64_t M,
                               int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmaj, int b_kmaj,
                               int batch, int64_t sA, int64_t sB, int64_t sC, int act, int tile, float keep,
                               int64_t seed, hipStream_t st) {
  return gemm_bf16_impl(A, B, C, nullptr, bias, M, N, K, lda, ldb, ldc, 0, a_kmaj, b_kmaj, batch, sA, sB, sC, 0,
                        1.f, 0.f, act, 0, 0, 0, 1, 0, nullptr, tile, C2, keep, (uint64_t)seed, st);
}

// the same product, also storing the pre-activation (bias added, before `act`) into C2
// (bf16, C's leading dimension and batch stride; C bf16)
HETU_API int hetu_gemm_bf16_pre(const void* A, const void* B, void* C, void* C2, const float* bias, int64_t M,
                                int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmaj, int b_kmaj,
                                int batch, int64_t sA, int64_t sB, int64_t sC, int act, int tile, hipStream_t st) {
  if (!C2) return (int)hipErrorInvalidValue;
  return gemm_bf16_impl(A, B, C, nullptr, bias, M, N, K, lda, ldb, ldc, 0, a_kmaj, b_kmaj, batch, sA, sB, sC, 0,
                        1.f, 0.f, act, 0, 0, 0, 1, 0, nullptr, tile, C2, 0.f, 0, st);
}

// bf16 C = (A @ B) * scale where G > 0, else 0 (G: bf16, C's shape and leading dimension)
// -- the data gradient of a ReLU (+ dropout) output G, masked in the GEMM that produces it
HETU_API int hetu_gemm_bf16_gmask(const void* A, const void* B, void* C, const void* G, float scale, int64_t M,
                                  int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmaj, int b_kmaj,
                                  int tile, hipStream_t st) {
  if (!G) return (int)hipErrorInvalidValue;
  return gemm_bf16_impl(A, B, C, nullptr, nullptr, M, N, K, lda, ldb, ldc, 0, a_kmaj, b_kmaj, 1, 0, 0, 0, 0, 1.f,
                        0.f, 0, 0, 0, 0, 1, 0, nullptr, tile, nullptr, 0.f, 0, st, G, scale);
}

// dropout(act(A @ B)) as hetu_gemm_bf16_ex (keep < 1, batch 1), also writing the keep bits of
// the stored output to `bits` (one byte per 8 elements of C, ldc % 8 == 0): the mask that
// hetu_gemm_bf16_gbits reads in the backward instead of the bf16 output
HETU_API int hetu_gemm_bf16_drop_bits(const void* A, const void* B, void* C, uint8_t* bits, int64_t M, int64_t N,
                                      int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmaj, int b_kmaj,
                                      int act, int tile, float keep, int64_t seed, hipStream_t st) {
  if (!bits || !(keep < 1.f)) return (int)hipErrorInvalidValue;
  return gemm_bf16_impl(A, B, C, nullptr, nullptr, M, N, K, lda, ldb, ldc, 0, a_kmaj, b_kmaj, 1, 0, 0, 0, 0, 1.f,
                        0.f, act, 0, 0, 0, 1, 0, nullptr, tile, nullptr, keep, (uint64_t)seed, st, nullptr, 1.f, 0,
                        bits);
}

// hetu_gemm_bf16_gmask with the mask given as those keep bits
HETU_API int hetu_gemm_bf16_gbits(const void* A, const void* B, void* C, const uint8_t* bits, float scale, int64_t M,
                                  int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmaj, int b_kmaj,
                                  int tile, hipStream_t st) {
  if (!bits) return (int)hipErrorInvalidValue;
  return gemm_bf16_impl(A, B, C, nullptr, nullptr, M, N, K, lda, ldb, ldc, 0, a_kmaj, b_kmaj, 1, 0, 0, 0, 0, 1.f,
                        0.f, 0, 0, 0, 0, 1, 0, nullptr, tile, nullptr, 0.f, 0, st, bits, scale, 1);
}

HETU_API int hetu_gemm_pick_splitk(int64_t M, int64_t N, int64_t K) { return pick_splitk(M, N, K); }


// split count for the 256x256 kernel: about one block per CU, slices of >= 8 K-tiles
HETU_API int hetu_gemm_pick_splitk_big(int64_t M, int64_t N, int64_t K) {
  int64_t tiles = ((M + BIG - 1) / BIG) * ((N + BIG - 1) / BIG);
  int64_t ktiles = (K + BK - 1) / BK;
  int64_t want = (256 + tiles - 1) / tiles;
  int64_t cap = std::max<int64_t>(1, ktiles / 8);
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min(want, cap), 512));
}

// out[i] = sum_z slab[z * n + i] (fp32; the partials of a split-K library GEMM):
// 16-byte vectors, the slabs' loads issued 8 at a time before the adds, grid-stride.
__global__ void __launch_bounds__(256) splitk_sum_vec_k(const float4* __restrict__ slab, int64_t n4, int nz,
                                                         float4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z0 = 0; z0 < nz; z0 += 8) {
      float4 v[8];
#pragma unroll
      for (int z = 0; z < 8; ++z)
        if (z0 + z < nz) v[z] = slab[(z0 + z) * n4 + i];
#pragma unroll
      for (int z = 0; z < 8; ++z)
        if (z0 + z < nz) { acc.x += v[z].x; acc.y += v[z].y; acc.z += v[z].z; acc.w += v[z].w; }
    }
    out[i] = acc;
  }
}

HETU_API int hetu_splitk_sum_f32(const float* slab, int nz, float* out, int64_t n, hipStream_t st) {
  if (nz < 1 || nz > 64 || (n & 3) || (((uintptr_t)slab | (uintptr_t)out) & 15)) return (int)hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int64_t nb = (n4 + 255) / 256;
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(splitk_sum_vec_k, dim3((unsigned)nb), dim3(256), 0, st, (const float4*)slab, n4, nz, (float4*)out);
  return (int)hipGetLastError();
}

