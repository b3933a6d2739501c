// Same-process A/B of the hand-written bf16 MFMA GEMM tiles against hipBLASLt
// (interleaved rounds, random uniform [-1,1) operands, min / median per variant).
//
//   make -C csrc bench   ->  csrc/build/gemm_bench
//   gemm_bench [M N K ta tb]...      (ta: A stored [K][M]; tb: B stored [N][K])
//   VARS="0:1,3:4,1:7"  tile:splitk variants (default: every tile, no split)
//   WGRAD_F32=1         shapes with ta (weight gradients) write fp32 C, as the framework's
//                       flat gradient buffer does (split-K slabs + reduce when splitk > 1)
//
// Every variant's output is checked against hipBLASLt's (relative Frobenius error).
#include "../kernels/gemm_core.h"
#include <hipblaslt/hipblaslt.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#ifndef BENCH_FAST
namespace hetu {
namespace gemm {
template int launch_buf<true>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t, const Epi&,
                              int64_t, int64_t, int64_t, int, int, hipStream_t, int);
template int launch_buf<false>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t, const Epi&,
                               int64_t, int64_t, int64_t, int, int, hipStream_t, int);
}  // namespace gemm
}  // namespace hetu
#endif

using namespace hetu;
using namespace hetu::gemm;

// -DBENCH_FAST: only the 256x256 kernel (tile 1), K % 64 == 0, for quick kernel iteration
static int run_tile(const bf16* a, const bf16* b, int a_kmaj, int b_kmaj, int64_t lda, int64_t ldb, const Epi& ep,
                    int64_t M, int64_t N, int64_t K, hipStream_t st, int tile, int splitk) {
#ifdef BENCH_FAST
  if (K % BK) return (int)hipErrorInvalidValue;
#define HB_CASE(LA, LB, SA, SB)                                                                          \
  if (tile == 1) return launch_big(LA<true>{a, lda, M, K, 0}, LB<true>{b, ldb, N, K, 0}, ep, M, N, K, 1, 1, st);     \
  return (int)hipErrorInvalidValue;
  if (a_kmaj && b_kmaj) { HB_CASE(BufK, BufK, 0, 0) }
  if (a_kmaj) { HB_CASE(BufK, BufMN, 0, 0) }
  if (b_kmaj) { HB_CASE(BufMN, BufK, 0, 0) }
  HB_CASE(BufMN, BufMN, 0, 0)
#else
  return (K % BK == 0) ? launch_buf<true>(a, b, a_kmaj, b_kmaj, lda, ldb, 0, 0, ep, M, N, K, 1, splitk, st, tile)
                       : launch_buf<false>(a, b, a_kmaj, b_kmaj, lda, ldb, 0, 0, ep, M, N, K, 1, splitk, st, tile);
#endif
}

#define CK(x)                                                                          \
  do {                                                                                 \
    auto e_ = (x);                                                                     \
    if ((int)e_ != 0) {                                                                \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)e_);            \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void fill_k(unsigned short* p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float u = (float)(h >> 8) * (1.f / 8388608.f) - 1.f;   // [-1, 1)
    p[i] = f_to_bf16_bits(u);
  }
}

__global__ void relerr_k(const void* a_, const void* b_, int64_t n, float* out, int f32) {
  float d = 0.f, r = 0.f;
  const unsigned short* a = (const unsigned short*)a_;
  const unsigned short* b = (const unsigned short*)b_;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = f32 ? ((const float*)a_)[i] : bf16_bits_to_f(a[i]);
    const float y = f32 ? ((const float*)b_)[i] : bf16_bits_to_f(b[i]);
    d += (x - y) * (x - y);
    r += y * y;
  }
  atomicAdd(out, d);
  atomicAdd(out + 1, r);
}

struct Shape { int64_t M, N, K; int ta, tb; };

struct Blas {
  hipblasLtHandle_t h;
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasLtMatmulHeuristicResult_t res;
  void* ws; size_t wsz = 64 << 20;
  // row-major C[M][N] = op(A) op(B)  <=>  column-major C^T = op(B)^T op(A)^T
  void init(const Shape& s, bool cf32) {
    CK(hipblasLtCreate(&h));
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    // B stored [N][K] (tb) is column-major KxN -> needs T to give N x K
    hipblasOperation_t opB = s.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    hipblasOperation_t opA = s.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opB, sizeof(opB)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opA, sizeof(opA)));
    // first operand (B): stored [N][K] -> col-major K x N (ld K); stored [K][N] -> N x K (ld N)
    if (s.tb) CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, s.K, s.N, s.K));
    else CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, s.N, s.K, s.N));
    // second operand (A): stored [M][K] -> col-major K x M (ld K); stored [K][M] -> M x K (ld M)
    if (s.ta) CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, s.M, s.K, s.M));
    else CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, s.K, s.M, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lc, cf32 ? HIP_R_32F : HIP_R_16BF, s.N, s.M, s.N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    int cnt = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 1, &res, &cnt));
    if (cnt < 1) { fprintf(stderr, "no hipBLASLt algo\n"); exit(1); }
    CK(hipMalloc(&ws, wsz));
  }
  void run(const void* A, const void* B, void* C, hipStream_t st) {
    float one = 1.f, zero = 0.f;
    CK(hipblasLtMatmul(h, desc, &one, B, la, A, lb, &zero, C, lc, C, lc, &res.algo, ws, wsz, st));
  }
};

int main(int argc, char** argv) {
  std::vector<Shape> shapes;
  for (int i = 1; i + 4 < argc; i += 5)
    shapes.push_back({atoll(argv[i]), atoll(argv[i + 1]), atoll(argv[i + 2]), atoi(argv[i + 3]), atoi(argv[i + 4])});
  if (shapes.empty())
    shapes = {{4096, 4096, 4096, 0, 0}, {4096, 4096, 4096, 0, 1}, {8192, 8192, 8192, 0, 1},
              {8192, 3072, 768, 0, 0},  {8192, 768, 3072, 0, 0},  {768, 3072, 8192, 1, 0},
              {8192, 2304, 768, 0, 0},  {50176, 256, 1024, 0, 1}, {50176, 1024, 256, 0, 1},
              {8192, 768, 768, 0, 0},   {8192, 30528, 768, 0, 1}, {8192, 768, 30528, 0, 0}};
  const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 20;
  const int rounds = getenv("ROUNDS") ? atoi(getenv("ROUNDS")) : 5;
  const char* only = getenv("TILES");   // e.g. "0,1,3"
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float* err;
  CK(hipMalloc(&err, 8));
  const bool wgrad_f32 = getenv("WGRAD_F32") && atoi(getenv("WGRAD_F32"));
  struct Var { std::string name; int tile, splitk; };
  std::vector<Var> user_vars;
  if (const char* vs = getenv("VARS")) {
    std::string str(vs);
    size_t p = 0;
    while (p < str.size()) {
      size_t q = str.find(',', p);
      if (q == std::string::npos) q = str.size();
      std::string tok = str.substr(p, q - p);
      const size_t c = tok.find(':');
      const int t = atoi(tok.substr(0, c).c_str());
      const int sk = c == std::string::npos ? 1 : atoi(tok.substr(c + 1).c_str());
      user_vars.push_back({"t" + std::to_string(t) + "s" + std::to_string(sk), t, sk});
      p = q + 1;
    }
  }
  float* ws = nullptr;
  const size_t ws_bytes = (size_t)1 << 30;
  CK(hipMalloc(&ws, ws_bytes));
  for (const Shape& s : shapes) {
    const int64_t na = s.M * s.K, nb = s.N * s.K, nc = s.M * s.N;
    const bool cf32 = wgrad_f32 && s.ta;
    const int esz = cf32 ? 4 : 2;
    unsigned short *A, *B, *C, *R;
    CK(hipMalloc(&A, na * 2)); CK(hipMalloc(&B, nb * 2)); CK(hipMalloc(&C, nc * esz)); CK(hipMalloc(&R, nc * esz));
    fill_k<<<1024, 256, 0, st>>>(A, na, 17u);
    fill_k<<<1024, 256, 0, st>>>(B, nb, 91u);
    Blas blas;
    blas.init(s, cf32);
    blas.run(A, B, R, st);
    const int64_t lda = s.ta ? s.M : s.K;
    const int64_t ldb = s.tb ? s.K : s.N;
    std::vector<Var> vars = {{"blas", -1, 1}};
    if (!user_vars.empty()) {
      for (const Var& v : user_vars) vars.push_back(v);
    } else {
      for (int t : {0, 1, 2, 3, 5}) {
#ifdef BENCH_FAST
        if (t == 0 || t == 2) continue;
#endif
        if (only && !strchr(only, '0' + t)) continue;
        vars.push_back({"tile" + std::to_string(t), t, 1});
      }
    }
    auto run = [&](const Var& v) {
      if (v.tile < 0) { blas.run(A, B, C, st); return; }
      Epi ep{C, nullptr, nullptr, s.N, 0, 0, 0, 1.f, 0.f, 0, cf32 ? 1 : 0, 0, 0, 0, nullptr, 0, nullptr};
      if (v.splitk > 1) {
        if ((size_t)v.splitk * nc * 4 > ws_bytes) { fprintf(stderr, "slab too big\n"); exit(1); }
        ep.slab = ws;
      }
      CK(run_tile((const bf16*)A, (const bf16*)B, !s.ta, s.tb, lda, ldb, ep, s.M, s.N, s.K, st, v.tile, v.splitk));
    };
    std::vector<std::vector<float>> ms(vars.size());
    std::vector<float> errs(vars.size(), 0.f);
    for (size_t v = 0; v < vars.size(); ++v) {   // correctness + warm
      CK(hipMemsetAsync(C, 0, nc * esz, st));
      run(vars[v]);
      CK(hipMemsetAsync(err, 0, 8, st));
      relerr_k<<<1024, 256, 0, st>>>(C, R, nc, err, cf32 ? 1 : 0);
      float h[2];
      CK(hipMemcpyAsync(h, err, 8, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      errs[v] = sqrtf(h[0] / (h[1] + 1e-30f));
    }
    for (int r = 0; r < rounds; ++r)
      for (size_t v = 0; v < vars.size(); ++v) {
        run(vars[v]);
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < reps; ++i) run(vars[v]);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[v].push_back(t / reps);
      }
    const double fl = 2.0 * s.M * s.N * s.K;
    printf("M %6ld N %6ld K %6ld %s%s%s |", (long)s.M, (long)s.N, (long)s.K, s.ta ? "T" : "N", s.tb ? "T" : "N", cf32 ? " f32" : "");
    for (size_t v = 0; v < vars.size(); ++v) {
      std::sort(ms[v].begin(), ms[v].end());
      const float mn = ms[v][0], med = ms[v][ms[v].size() / 2];
      printf(" %s %.4f/%.4f ms %5.0f TF e%.0e |", vars[v].name.c_str(), mn, med, fl / mn * 1e-9, errs[v]);
    }
    printf("\n");
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R));
  }
  return 0;
}
