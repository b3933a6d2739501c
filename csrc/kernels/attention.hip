// Fused multi-head attention (forward + backward) for gfx950, bf16 in/out,
// fp32 softmax, head dim 64, sequence length S = 32*KB (fwd S <= 256, bwd
// S <= 128: BERT / Transformer encoder lengths).
//
// Replaces the reference's materialised chain batch_matmul -> mask add ->
// softmax -> dropout -> batch_matmul (+ transposes, examples/nlp/bert/
// hetu_bert.py:220-270; Softmax.cu / CudnnSoftmax.cu, Dropout.cu,
// BatchMatrixMult.cu) -- 8 kernels and an S x S fp32 score tensor per
// direction -- with one kernel each way that reads Q/K/V straight out of the
// packed QKV projection [B*S, 3H] and writes the context straight into
// [B*S, H] (no head transposes), and the gradients straight into the packed
// dQKV buffer.
//
// Layout (one workgroup per (batch, head), 4 waves, each wave 32 queries):
//   scores are computed *transposed*, S^T = K . Q^T with
//   mfma_f32_32x32x16_bf16 (A = K rows, B = Q rows, both 16-byte global loads),
//   so every lane owns one query and its keys sit in the accumulator registers:
//   the row softmax is lane-local plus one cross-half (lane ^ 32) exchange.
//   P then feeds O^T = V^T . P^T directly as the B operand (accumulator-as-
//   operand, permuted k order) with V^T staged in LDS.
//   Dropout on P regenerates Philox bits from (seed, flat index of P / 4), so
//   the backward needs no mask tensor.
//   Backward recomputes P from the saved log-sum-exp, builds dS in registers,
//   computes dQ the same way as O, and stages P_drop^T / dS^T in LDS so each
//   wave then produces dV / dK for 32 keys over all queries.
#include "common.h"
#include <string.h>

namespace hetu {
namespace attn {

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int HD = 64;
// shorts of padding per LDS row of the transposed images (16 B: rows stay 16-byte aligned
// for the ds_read_b128 fragment reads; with the paired-key stores of stage_t a wave's
// 64 stores of one column land on 64 distinct banks)
constexpr int PAD = 8;
// images read only by lds_perm (8-byte ds_read_b64, lane groups {0-31} / {32-63}: 32 rows x
// 2 dwords): a row stride of S/2 + 2 dwords = 2 x odd puts the 32 rows on 64 distinct banks
// (the 16-byte-aligned S + 8 stride maps row r and r + 16 onto the same pair: 2-way)
constexpr int PAD_P = 4;

struct Args {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  int64_t ldq, ldk, ldv;
  const float* mask;      // additive key mask [B, S] or null
  bf16* o;
  int64_t ldo;
  float* lse;             // [B*NH*S]
  const bf16* dout;
  int64_t lddo;
  bf16* dq;
  bf16* dk;
  bf16* dv;
  int64_t lddq, lddk, lddv;
  int B, NH;
  float scale, keep;
  uint64_t seed;
  const uint64_t* rngo;    // step counter of the graph-safe RNG (common.h rng_seed)
  short* ws;              // split backward: P_drop^T then (scale dS)^T, [B*NH][S][S] bf16 each
};

__device__ __forceinline__ v16f mfma(v8s a, v8s b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ v8s ld8(const bf16* p) { return *reinterpret_cast<const v8s*>(p); }

// B/A fragment of k-step s from an accumulator tile (rows 8s..8s+7 of the regs)
__device__ __forceinline__ v8s pack_acc(const v16f& x, int s, float mul) {
  v8s r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f_to_bf16_bits(x[8 * s + j] * mul);
  return r;
}

// A fragment from an LDS image T[row][col] (row = lane's output row) whose k
// index runs along the columns in the PERMUTED accumulator order of block kb,
// step s: element j <-> column kb*32 + 16s + 8(j>>2) + 4h + (j&3).
__device__ __forceinline__ v8s lds_perm(const short* T, int ldt, int row, int kb, int s, int h) {
  const short* p = T + row * ldt + kb * 32 + 16 * s + 4 * h;
  const v4s lo = *reinterpret_cast<const v4s*>(p);
  const v4s hi = *reinterpret_cast<const v4s*>(p + 8);
  v8s r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// natural-order fragment from LDS: T[row][c0 .. c0+7]
__device__ __forceinline__ v8s lds8(const short* T, int ldt, int row, int c0) {
  return *reinterpret_cast<const v8s*>(T + row * ldt + c0);
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// x op x[lane ^ 32] for both wave halves by one v_permlane32_swap (no LDS round trip)
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// x of lane ^ 1 (DPP quad_perm [1, 0, 3, 2]: no LDS)
__device__ __forceinline__ float xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f_to_bf16_bits(lo) | ((uint32_t)f_to_bf16_bits(hi) << 16);
}

// keep-mask multiplier (0 or 1/keep) for 4 consecutive keys starting at a flat
// P index divisible by 4
__device__ __forceinline__ void drop_mul4(uint64_t seed, uint64_t flat, float keep, float (&m)[4]) {
  const uint4 r = Philox::gen(seed, flat >> 2);
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  const float inv = 1.f / keep;
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = Philox::u01(rr[k]) < keep ? inv : 0.f;
}

// stage X^T (X rows [S][64] with row stride ld) into LDS T[64][S + PAD]: each thread
// loads two consecutive rows x 8 columns and writes 8 dwords (the two rows' values of one
// column), consecutive lanes on consecutive row pairs -- 4-byte stores on 64 distinct
// banks per wave instead of 2-byte stores 8 rows apart
template <int S, int LT = S + PAD, int NTH = 256>
__device__ __forceinline__ void stage_t(const bf16* X, int64_t ld, short* T) {
  constexpr int RP = S / 2;
  for (int idx = threadIdx.x; idx < RP * 8; idx += NTH) {
    const int rp = idx % RP, c = idx / RP;
    const v8s x0 = ld8(X + (int64_t)(2 * rp) * ld + 8 * c);
    const v8s x1 = ld8(X + (int64_t)(2 * rp + 1) * ld + 8 * c);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t pr = (uint32_t)(unsigned short)x0[i] | ((uint32_t)(unsigned short)x1[i] << 16);
      *reinterpret_cast<uint32_t*>(T + (8 * c + i) * LT + 2 * rp) = pr;
    }
  }
}

// -------------------------------------------------------------------------------------
template <int KB>
__global__ void __launch_bounds__(256) attn_fwd_k(Args a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int S = 32 * KB;
  constexpr int LT = S + PAD_P;                 // V^T: lds_perm reads only
  __shared__ __attribute__((aligned(16))) short vt[HD * LT];
  __shared__ __attribute__((aligned(16))) float msk[S];
  const int bh = blockIdx.x;
  const int b = bh / a.NH, hd = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const bf16* Q = a.q + (int64_t)b * S * a.ldq + hd * HD;
  const bf16* K = a.k + (int64_t)b * S * a.ldk + hd * HD;
  const bf16* V = a.v + (int64_t)b * S * a.ldv + hd * HD;
  stage_t<S, LT>(V, a.ldv, vt);
  // the key mask in log2 units: the softmax runs as exp2 of log2 e-scaled scores
  for (int i = threadIdx.x; i < S; i += 256) msk[i] = a.mask ? a.mask[(int64_t)b * S + i] * kLog2e : 0.f;
  __syncthreads();
  const int qb = blockIdx.y * 4 + w;
  if (qb >= KB) return;
  const int q = qb * 32 + r;
  const float sl2 = a.scale * kLog2e;

  v8s qf[4];
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) qf[ds] = ld8(Q + (int64_t)q * a.ldq + 16 * ds + 8 * h);

  v16f acc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    v16f c = {0.f};
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) c = mfma(ld8(K + (int64_t)(kb * 32 + r) * a.ldk + 16 * ds + 8 * h), qf[ds], c);
    acc[kb] = c;
  }
  // scaled scores + key mask (16-byte LDS reads of 4 consecutive keys), lane-local max,
  // one permlane swap with lane ^ 32
  float m = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 mm = *reinterpret_cast<const float4*>(&msk[kb * 32 + 8 * g + 4 * h]);
      const float m4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float sv = fmaf(acc[kb][4 * g + t], sl2, m4[t]);
        acc[kb][4 * g + t] = sv;
        m = fmaxf(m, sv);
      }
    }
  m = xmax32(m);
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = __builtin_amdgcn_exp2f(acc[kb][i] - m);
      acc[kb][i] = e;
      sum += e;
    }
  sum = xsum32(sum);
  const float inv = 1.f / sum;
  if (h == 0) a.lse[(int64_t)bh * S + q] = m * kLn2 + __logf(sum);
  if (a.keep < 1.f) {
    const uint64_t rowflat = ((uint64_t)bh * S + q) * S;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float mul[4];
        drop_mul4(a.seed, rowflat + kb * 32 + 8 * g + 4 * h, a.keep, mul);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[kb][4 * g + t] *= mul[t];
      }
  }
  // O^T[d][q] = sum_key V^T[d][key] P^T[key][q]; the 1 / sum normalisation at the store
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    v16f o = {0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) o = mfma(lds_perm(vt, LT, db * 32 + r, kb, s, h), pack_acc(acc[kb], s, 1.f), o);
    bf16* O = a.o + ((int64_t)b * S + q) * a.ldo + hd * HD + db * 32;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 pk;
      pk.x = pack2(o[4 * g] * inv, o[4 * g + 1] * inv);
      pk.y = pack2(o[4 * g + 2] * inv, o[4 * g + 3] * inv);
      *reinterpret_cast<uint2*>(O + 8 * g + 4 * h) = pk;
    }
  }
}

// -------------------------------------------------------------------------------------
// PH: 0 = both phases in one workgroup (P_drop^T / dS^T in LDS: ~122 KiB at S = 128, one
// workgroup per CU); 1 = phase 1 only, P_drop^T / dS^T to the global workspace (LDS: K^T);
// 2 = phase 2 only, reading them back (LDS: dO^T, Q^T) -- the split form runs several
// workgroups per CU at the cost of the workspace round trip
template <int KB, int PH = 0>
__global__ void __launch_bounds__(256) attn_bwd_k(Args a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int S = 32 * KB;
  constexpr int LT = S + PAD;
  constexpr int LP = PH == 0 ? LT : S;   // row stride of the P_drop^T / dS^T images
  constexpr int LK = S + PAD_P;          // K^T: lds_perm reads only
  extern __shared__ short lds[];
  const int bh = blockIdx.x;
  short* kt = lds;                                          // K^T   [64][LK]  (PH 0, 1)
  short* qt = PH == 2 ? lds : kt + HD * LK + 64;            // Q^T   [64][LT]  (PH 0, 2; 16-byte aligned)
  short* dot = qt + HD * LT;                                // dO^T  [64][LT]  (PH 0, 2)
  short* pt = PH == 0 ? dot + HD * LT : a.ws + (int64_t)bh * S * S;                  // P_drop^T [S][LP]
  // dS^T (the softmax-gradient without the scale, which goes on at the dQ / dK stores);
  // 64 shorts past P_drop^T's end in LDS, so the two images' paired stores use different banks
  short* dst = PH == 0 ? pt + S * LT + 64 : a.ws + ((int64_t)a.B * a.NH + bh) * S * S;
  float* dvec = reinterpret_cast<float*>(PH == 0 ? dst + S * LT : (PH == 1 ? kt + HD * LK + 64 : dot + HD * LT));
  float* msk = dvec + S;
  const int b = bh / a.NH, hd = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)b * S;
  const bf16* Q = a.q + row0 * a.ldq + hd * HD;
  const bf16* K = a.k + row0 * a.ldk + hd * HD;
  const bf16* V = a.v + row0 * a.ldv + hd * HD;
  const bf16* O = a.o + row0 * a.ldo + hd * HD;
  const bf16* dO = a.dout + row0 * a.lddo + hd * HD;

  if (PH != 2) stage_t<S, LK>(K, a.ldk, kt);
  if (PH != 1) {
    stage_t<S>(Q, a.ldq, qt);
    stage_t<S>(dO, a.lddo, dot);
  }
  for (int i = threadIdx.x; i < S; i += 256) msk[i] = a.mask ? a.mask[(int64_t)b * S + i] * kLog2e : 0.f;
  // D[q] = sum_d dO[q][d] * O[q][d]: 8 consecutive threads per query
  for (int idx = threadIdx.x; PH != 2 && idx < S * 8; idx += 256) {
    const int qq = idx >> 3, c = idx & 7;
    const v8s x = ld8(dO + (int64_t)qq * a.lddo + 8 * c);
    const v8s y = ld8(O + (int64_t)qq * a.ldo + 8 * c);
    float p = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) p += bf16_bits_to_f((unsigned short)x[i]) * bf16_bits_to_f((unsigned short)y[i]);
    p += __shfl_xor(p, 1, 64);
    p += __shfl_xor(p, 2, 64);
    p += __shfl_xor(p, 4, 64);
    if (c == 0) dvec[qq] = p;
  }
  __syncthreads();

  const bool drop = a.keep < 1.f;
  // ---- phase 1: per query block: P, dP, dS; dQ; stage P_drop^T and dS^T -----------------
  for (int qb = w; PH != 2 && qb < KB; qb += 4) {
    const int q = qb * 32 + r;
    v8s qf[4], gf[4];
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      qf[ds] = ld8(Q + (int64_t)q * a.ldq + 16 * ds + 8 * h);
      gf[ds] = ld8(dO + (int64_t)q * a.lddo + 16 * ds + 8 * h);
    }
    const float lse2 = a.lse[(int64_t)bh * S + q] * kLog2e;
    const float Dq = dvec[q];
    const float sl2 = a.scale * kLog2e;
    const uint64_t rowflat = ((uint64_t)bh * S + q) * S;
    v16f ds_acc[KB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      v16f sc = {0.f}, dp = {0.f};
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) {
        sc = mfma(ld8(K + (int64_t)(kb * 32 + r) * a.ldk + 16 * ds + 8 * h), qf[ds], sc);
        dp = mfma(ld8(V + (int64_t)(kb * 32 + r) * a.ldv + 16 * ds + 8 * h), gf[ds], dp);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float mul[4] = {1.f, 1.f, 1.f, 1.f};
        if (drop) drop_mul4(a.seed, rowflat + kb * 32 + 8 * g + 4 * h, a.keep, mul);
        const float4 mm = *reinterpret_cast<const float4*>(&msk[kb * 32 + 8 * g + 4 * h]);
        const float m4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int i = 4 * g + t;
          const int key = kb * 32 + 8 * g + 4 * h + t;
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[i], sl2, m4[t] - lse2));
          const float pd = drop ? p * mul[t] : p;
          const float dsv = p * (drop ? fmaf(dp[i], mul[t], -Dq) : dp[i] - Dq);
          // (pairing the 2-byte stores into 4-byte ones across lane pairs by DPP measured
          // slower: +22 % VALU per block in this VALU-bound loop)
          pt[key * LP + q] = (short)f_to_bf16_bits(pd);
          dst[key * LP + q] = (short)f_to_bf16_bits(dsv);
          sc[i] = dsv;
        }
      }
      ds_acc[kb] = sc;
    }
    // dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      v16f o = {0.f};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          o = mfma(lds_perm(kt, LK, db * 32 + r, kb, s, h), pack_acc(ds_acc[kb], s, 1.f), o);
      bf16* dQ = a.dq + (row0 + q) * a.lddq + hd * HD + db * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pk;
        pk.x = pack2(o[4 * g] * a.scale, o[4 * g + 1] * a.scale);
        pk.y = pack2(o[4 * g + 2] * a.scale, o[4 * g + 3] * a.scale);
        *reinterpret_cast<uint2*>(dQ + 8 * g + 4 * h) = pk;
      }
    }
  }
  if (PH == 1) return;
  __syncthreads();
  // ---- phase 2: per key block: dV^T = dO^T P_drop, dK^T = Q^T (scale dS) -------------------
  for (int kb = w; kb < KB; kb += 4) {
    const int key = kb * 32 + r;
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      const short* A = which == 0 ? dot : qt;
      const short* Bm = which == 0 ? pt : dst;
      bf16* out = which == 0 ? a.dv + (row0 + key) * a.lddv : a.dk + (row0 + key) * a.lddk;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        v16f c = {0.f};
#pragma unroll
        for (int t = 0; t < S / 16; ++t) c = mfma(lds8(A, LT, db * 32 + r, 16 * t + 8 * h), lds8(Bm, LP, key, 16 * t + 8 * h), c);
        bf16* dst_row = out + hd * HD + db * 32;
        const float sc_out = which == 0 ? 1.f : a.scale;     // dK = scale * Q^T dS
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 pk;
          pk.x = pack2(c[4 * g] * sc_out, c[4 * g + 1] * sc_out);
          pk.y = pack2(c[4 * g + 2] * sc_out, c[4 * g + 3] * sc_out);
          *reinterpret_cast<uint2*>(dst_row + 8 * g + 4 * h) = pk;
        }
      }
    }
  }
}

// -------------------------------------------------------------------------------------
// 8-wave single-launch backward: the PH 0 schedule at two waves per SIMD.  The ~122 KiB of
// images keep one workgroup per CU, so PH 0 ran one wave per SIMD with nothing to hide the
// global K / V fragment loads and the exp / Philox VALU work behind; the split form (PH 1 + 2)
// buys occupancy with a 2 x S^2 bf16 workspace round trip per head (at BERT-base's shape
// 100 MB per layer).  Here the 16 (query block, key block) tiles of phase 1 go to 8 waves
// (wave w: query block w & 3, key half w >> 2), each key half's partial dQ^T meets its
// partner's through a 32 KiB fp32 LDS exchange, and phase 2's 8 (key block, dV | dK) jobs
// are one per wave.  LDS at S = 128: 155 KiB of gfx950's 160.
template <int KB>
__global__ void __launch_bounds__(512) attn_bwd8_k(Args a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int S = 32 * KB;
  constexpr int LT = S + PAD;
  constexpr int LK = S + PAD_P;
  constexpr int KH = (KB + 1) / 2;        // key blocks per key half
  extern __shared__ short lds[];
  const int bh = blockIdx.x;
  short* kt = lds;                        // K^T      [64][LK]   lds_perm reads (dQ)
  short* qt = kt + HD * LK + 64;          // Q^T      [64][LT]   phase 2 A (dK)
  short* dot = qt + HD * LT;              // dO^T     [64][LT]   phase 2 A (dV)
  short* pt = dot + HD * LT;              // P_drop^T [S][LT]
  short* dst = pt + S * LT + 64;          // dS^T     [S][LT]
  float* dvec = reinterpret_cast<float*>(dst + S * LT);
  float* msk = dvec + S;
  float* red = msk + S;                   // partial dQ^T of key half 1: [4][32][64] fp32
  const int b = bh / a.NH, hd = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)b * S;
  const bf16* Q = a.q + row0 * a.ldq + hd * HD;
  const bf16* K = a.k + row0 * a.ldk + hd * HD;
  const bf16* V = a.v + row0 * a.ldv + hd * HD;
  const bf16* O = a.o + row0 * a.ldo + hd * HD;
  const bf16* dO = a.dout + row0 * a.lddo + hd * HD;

  stage_t<S, LK, 512>(K, a.ldk, kt);
  stage_t<S, LT, 512>(Q, a.ldq, qt);
  stage_t<S, LT, 512>(dO, a.lddo, dot);
  for (int i = threadIdx.x; i < S; i += 512) msk[i] = a.mask ? a.mask[(int64_t)b * S + i] * kLog2e : 0.f;
  for (int idx = threadIdx.x; idx < S * 8; idx += 512) {
    const int qq = idx >> 3, c = idx & 7;
    const v8s x = ld8(dO + (int64_t)qq * a.lddo + 8 * c);
    const v8s y = ld8(O + (int64_t)qq * a.ldo + 8 * c);
    float p = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) p += bf16_bits_to_f((unsigned short)x[i]) * bf16_bits_to_f((unsigned short)y[i]);
    p += __shfl_xor(p, 1, 64);
    p += __shfl_xor(p, 2, 64);
    p += __shfl_xor(p, 4, 64);
    if (c == 0) dvec[qq] = p;
  }
  __syncthreads();

  const bool drop = a.keep < 1.f;
  const int qb = w & 3, kh = w >> 2;
  const int kb0 = kh * KH, kb1 = min(KB, kb0 + KH);
  const bool qact = qb < KB;
  v16f dqp[2] = {v16f{0.f}, v16f{0.f}};   // this key half's dQ^T[d][q] for d blocks 0, 1
  if (qact) {
    const int q = qb * 32 + r;
    v8s qf[4], gf[4];
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      qf[ds] = ld8(Q + (int64_t)q * a.ldq + 16 * ds + 8 * h);
      gf[ds] = ld8(dO + (int64_t)q * a.lddo + 16 * ds + 8 * h);
    }
    const float lse2 = a.lse[(int64_t)bh * S + q] * kLog2e;
    const float Dq = dvec[q];
    const float sl2 = a.scale * kLog2e;
    const uint64_t rowflat = ((uint64_t)bh * S + q) * S;
#pragma unroll
    for (int j = 0; j < KH; ++j) {
      const int kb = kb0 + j;
      if (kb >= kb1) break;
      v16f sc = {0.f}, dp = {0.f};
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) {
        sc = mfma(ld8(K + (int64_t)(kb * 32 + r) * a.ldk + 16 * ds + 8 * h), qf[ds], sc);
        dp = mfma(ld8(V + (int64_t)(kb * 32 + r) * a.ldv + 16 * ds + 8 * h), gf[ds], dp);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float mul[4] = {1.f, 1.f, 1.f, 1.f};
        if (drop) drop_mul4(a.seed, rowflat + kb * 32 + 8 * g + 4 * h, a.keep, mul);
        const float4 mm = *reinterpret_cast<const float4*>(&msk[kb * 32 + 8 * g + 4 * h]);
        const float m4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int i = 4 * g + t;
          const int key = kb * 32 + 8 * g + 4 * h + t;
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[i], sl2, m4[t] - lse2));
          const float pd = drop ? p * mul[t] : p;
          const float dsv = p * (drop ? fmaf(dp[i], mul[t], -Dq) : dp[i] - Dq);
          pt[key * LT + q] = (short)f_to_bf16_bits(pd);
          dst[key * LT + q] = (short)f_to_bf16_bits(dsv);
          sc[i] = dsv;
        }
      }
      // dQ^T[d][q] += sum_{key in kb} K^T[d][key] dS^T[key][q]
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int s = 0; s < 2; ++s) dqp[db] = mfma(lds_perm(kt, LK, db * 32 + r, kb, s, h), pack_acc(sc, s, 1.f), dqp[db]);
    }
    if (kh == 1) {   // lane-major fp32 exchange: conflict-free 4-byte stores / loads
      float* rp = red + qb * 2048;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) rp[(db * 16 + i) * 64 + lane] = dqp[db][i];
    }
  }
  __syncthreads();
  if (qact && kh == 0) {
    const int q = qb * 32 + r;
    const float* rp = red + qb * 2048;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      v16f o = dqp[db];
      if (KB > 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] += rp[(db * 16 + i) * 64 + lane];
      }
      bf16* dQ = a.dq + (row0 + q) * a.lddq + hd * HD + db * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pk;
        pk.x = pack2(o[4 * g] * a.scale, o[4 * g + 1] * a.scale);
        pk.y = pack2(o[4 * g + 2] * a.scale, o[4 * g + 3] * a.scale);
        *reinterpret_cast<uint2*>(dQ + 8 * g + 4 * h) = pk;
      }
    }
  }
  // ---- phase 2: wave w -> key block w & 3, dV (w < 4) or dK (w >= 4) --------------------------
  const int kb = w & 3, which = w >> 2;
  if (kb < KB) {
    const int key = kb * 32 + r;
    const short* A = which == 0 ? dot : qt;
    const short* Bm = which == 0 ? pt : dst;
    bf16* out = which == 0 ? a.dv + (row0 + key) * a.lddv : a.dk + (row0 + key) * a.lddk;
    const float sc_out = which == 0 ? 1.f : a.scale;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      v16f c = {0.f};
#pragma unroll
      for (int t = 0; t < S / 16; ++t) c = mfma(lds8(A, LT, db * 32 + r, 16 * t + 8 * h), lds8(Bm, LT, key, 16 * t + 8 * h), c);
      bf16* dst_row = out + hd * HD + db * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pk;
        pk.x = pack2(c[4 * g] * sc_out, c[4 * g + 1] * sc_out);
        pk.y = pack2(c[4 * g + 2] * sc_out, c[4 * g + 3] * sc_out);
        *reinterpret_cast<uint2*>(dst_row + 8 * g + 4 * h) = pk;
      }
    }
  }
}

template <int KB>
size_t bwd8_lds_bytes() {
  constexpr int S = 32 * KB, LT = S + PAD, LK = S + PAD_P;
  return (size_t)(HD * LK + 64 + 2 * HD * LT + 2 * S * LT + 64) * sizeof(short) + 2 * S * sizeof(float) +
         4 * 2048 * sizeof(float);
}

template <int KB>
void launch_bwd8(dim3 grid, const Args& a, hipStream_t st) {
  static bool attr = false;
  const size_t bytes = bwd8_lds_bytes<KB>();
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd8_k<KB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    attr = true;
  }
  hipLaunchKernelGGL(attn_bwd8_k<KB>, grid, dim3(512), bytes, st, a);
}

template <int KB, int PH = 0>
size_t bwd_lds_bytes() {
  constexpr int S = 32 * KB, LT = S + PAD, LK = S + PAD_P;
  if (PH == 1) return (size_t)(HD * LK + 64) * sizeof(short) + 2 * S * sizeof(float);
  if (PH == 2) return (size_t)2 * HD * LT * sizeof(short) + 2 * S * sizeof(float);
  return (size_t)(HD * LK + 64 + 2 * HD * LT + 2 * S * LT + 64) * sizeof(short) + 2 * S * sizeof(float);
}

// > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU) must be opted into once
template <int KB>
void launch_bwd(dim3 grid, const Args& a, hipStream_t st) {
  if (a.ws) {   // split form: two launches, the images through the workspace
    const size_t b1 = bwd_lds_bytes<KB, 1>(), b2 = bwd_lds_bytes<KB, 2>();
    hipLaunchKernelGGL((attn_bwd_k<KB, 1>), grid, dim3(256), b1, st, a);
    hipLaunchKernelGGL((attn_bwd_k<KB, 2>), grid, dim3(256), b2, st, a);
    return;
  }
  static bool attr = false;
  const size_t bytes = bwd_lds_bytes<KB>();
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_k<KB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    attr = true;
  }
  hipLaunchKernelGGL(attn_bwd_k<KB>, grid, dim3(256), bytes, st, a);
}

}  // namespace attn
}  // namespace hetu

using namespace hetu;
using namespace hetu::attn;

static Args make_args(const void* q, const void* k, const void* v, int64_t ldq, int64_t ldk, int64_t ldv,
                      const float* mask, int B, int NH, float scale, float keep, int64_t seed) {
  Args a;
  memset(&a, 0, sizeof(a));
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv;
  a.mask = mask;
  a.B = B; a.NH = NH;
  a.scale = scale; a.keep = keep; a.seed = (uint64_t)seed; a.rngo = hetu_rng_offset_ptr();
  return a;
}

// q/k/v: bf16 rows of a [B*S, ld] matrix, head h at columns [h*64, h*64+64).
HETU_API int hetu_attn_fwd(const void* q, const void* k, const void* v, int64_t ldq, int64_t ldk, int64_t ldv,
                           const float* mask, void* o, int64_t ldo, float* lse, int B, int NH, int S,
                           float scale, float keep, int64_t seed, hipStream_t st) {
  if (S % 32 || S <= 0 || S > 256 || B <= 0 || NH <= 0) return (int)hipErrorInvalidValue;
  Args a = make_args(q, k, v, ldq, ldk, ldv, mask, B, NH, scale, keep, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = lse;
  const int KB = S / 32;
  dim3 grid((unsigned)(B * NH), (unsigned)((KB + 3) / 4));
  switch (KB) {
    case 1: hipLaunchKernelGGL(attn_fwd_k<1>, grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(attn_fwd_k<2>, grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(attn_fwd_k<3>, grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL(attn_fwd_k<4>, grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL(attn_fwd_k<5>, grid, dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL(attn_fwd_k<6>, grid, dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL(attn_fwd_k<7>, grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL(attn_fwd_k<8>, grid, dim3(256), 0, st, a); break;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

// ws (nullable): 2 * B*NH*S*S bf16 -- the split two-launch form (see attn_bwd_k PH)
HETU_API int hetu_attn_bwd2(const void* q, const void* k, const void* v, int64_t ldq, int64_t ldk, int64_t ldv,
                            const float* mask, const void* o, int64_t ldo, const float* lse, const void* dout,
                            int64_t lddo, void* dq, void* dk, void* dv, int64_t lddq, int64_t lddk, int64_t lddv,
                            int B, int NH, int S, float scale, float keep, int64_t seed, void* ws, hipStream_t st) {
  if (S % 32 || S <= 0 || S > 128 || B <= 0 || NH <= 0 || (((uintptr_t)ws) & 15)) return (int)hipErrorInvalidValue;
  Args a = make_args(q, k, v, ldq, ldk, ldv, mask, B, NH, scale, keep, seed);
  a.ws = (short*)ws;
  a.o = (bf16*)o; a.ldo = ldo; a.lse = (float*)lse;
  a.dout = (const bf16*)dout; a.lddo = lddo;
  a.dq = (bf16*)dq; a.dk = (bf16*)dk; a.dv = (bf16*)dv;
  a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  const int KB = S / 32;
  dim3 grid((unsigned)(B * NH));
  switch (KB) {
    case 1: launch_bwd<1>(grid, a, st); break;
    case 2: launch_bwd<2>(grid, a, st); break;
    case 3: launch_bwd<3>(grid, a, st); break;
    case 4: launch_bwd<4>(grid, a, st); break;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

// the 8-wave single-launch backward (attn_bwd8_k); arguments as hetu_attn_bwd
HETU_API int hetu_attn_bwd8(const void* q, const void* k, const void* v, int64_t ldq, int64_t ldk, int64_t ldv,
                            const float* mask, const void* o, int64_t ldo, const float* lse, const void* dout,
                            int64_t lddo, void* dq, void* dk, void* dv, int64_t lddq, int64_t lddk, int64_t lddv,
                            int B, int NH, int S, float scale, float keep, int64_t seed, hipStream_t st) {
  if (S % 32 || S <= 0 || S > 128 || B <= 0 || NH <= 0) return (int)hipErrorInvalidValue;
  Args a = make_args(q, k, v, ldq, ldk, ldv, mask, B, NH, scale, keep, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = (float*)lse;
  a.dout = (const bf16*)dout; a.lddo = lddo;
  a.dq = (bf16*)dq; a.dk = (bf16*)dk; a.dv = (bf16*)dv;
  a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  dim3 grid((unsigned)(B * NH));
  switch (S / 32) {
    case 1: launch_bwd8<1>(grid, a, st); break;
    case 2: launch_bwd8<2>(grid, a, st); break;
    case 3: launch_bwd8<3>(grid, a, st); break;
    case 4: launch_bwd8<4>(grid, a, st); break;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_attn_bwd(const void* q, const void* k, const void* v, int64_t ldq, int64_t ldk, int64_t ldv,
                           const float* mask, const void* o, int64_t ldo, const float* lse, const void* dout,
                           int64_t lddo, void* dq, void* dk, void* dv, int64_t lddq, int64_t lddk, int64_t lddv,
                           int B, int NH, int S, float scale, float keep, int64_t seed, hipStream_t st) {
  return hetu_attn_bwd2(q, k, v, ldq, ldk, ldv, mask, o, ldo, lse, dout, lddo, dq, dk, dv, lddq, lddk, lddv, B, NH,
                        S, scale, keep, seed, nullptr, st);
}
