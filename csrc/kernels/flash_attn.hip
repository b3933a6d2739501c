// General fused attention (flash-style, online softmax) for gfx950: any query /
// key length, head dim 32 / 64 / 128, causal mode, an additive mask broadcastable
// to [B, NH, Sq, Sk] (strides, 0 on broadcast dims), dropout on P.  bf16 Q/K/V/O
// with arbitrary batch / head / row strides (packed QKV projections and
// [B, NH, S, D] head views are read in place), fp32 softmax statistics.
//
// Replaces the reference's materialised chain batch_matmul -> mask add -> causal
// where -> softmax -> dropout -> batch_matmul (examples/nlp/hetu_transformer.py:
// 99-130, examples/nlp/bert/hetu_bert.py:220-271) for every shape the fixed-length
// kernel of attention.hip (S <= 128, D = 64, no causal) does not take: the
// Transformer's maxlen-100 encoder / causal decoder / cross attention and BERT
// phase 2 at S = 512.
//
// Layout (known from attention.hip): scores are computed transposed,
// S^T = K . Q^T on mfma_f32_32x32x16_bf16 (A = K rows, B = Q rows), so each lane
// owns one query (lane & 31) and 16 of the 32 keys of a key block in its
// accumulator (key = (i & 3) + 8 (i >> 2) + 4 (lane >> 5)); the softmax is
// lane-local plus one exchange with lane ^ 32.  P feeds O^T = V^T . P^T as the B
// operand straight from the accumulator (permuted k order), V^T is staged per
// 32-key block in LDS as [D][36] (pairs of keys per 4-byte store; the 36-short row
// stride puts the 8 d-groups of a wave's store on distinct bank groups).
//
// Kernels: flash_fwd_k (per 128 queries: 4 waves x 32), flash_dq_k (the same walk
// for dQ from recomputed P and dP), flash_dkdv_k (per 128 keys: the transposed
// walk over query blocks, lane = key), flash_dsum_k (D = rowsum(dO * O)).
// Deterministic: no atomics; dropout bits from Philox(seed, row * ceil(Sk / 4) +
// key / 4)[key & 3], identical in the three kernels.
#include "common.h"
#include <string.h>

namespace hetu {
namespace flash {

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int KBLK = 32;     // keys (fwd / dq) or queries (dkdv) per inner block
constexpr int LT = 36;       // LDS row stride (shorts) of the transposed [D][32] images
constexpr int WQ = 128;      // queries (keys) per workgroup: 4 waves x 32

struct FArgs {
  const bf16 *q, *k, *v;
  int64_t qb, qh, qs;        // batch / head / row strides (elements), last dim contiguous
  int64_t kb, kh, ks;
  int64_t vb, vh, vs;
  bf16* o;
  int64_t ob, oh, os;
  float* lse;                // [B * NH * Sq]
  const float* mask;         // additive, element (b, h, i, j) at mb*b + mh*h + mq*i + mk*j; null: none
  int64_t mb, mh, mq, mk;
  const bf16* dout;
  int64_t gb, gh, gs;
  const float* dsum;         // [B * NH * Sq] rowsum(dO * O)
  bf16 *dq, *dk, *dv;
  int64_t dqb, dqh, dqs, dkb, dkh, dks, dvb, dvh, dvs;
  int B, NH, Sq, Sk;
  float scale, keep;
  uint64_t seed;
  const uint64_t* rngo;      // step counter of the graph-safe RNG (common.h rng_seed)
  int causal;
};

__device__ __forceinline__ v16f mfma(v8s a, v8s b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ v8s ld8(const bf16* p) { return *reinterpret_cast<const v8s*>(p); }
__device__ __forceinline__ v8s zero8() { v8s z = {0, 0, 0, 0, 0, 0, 0, 0}; return z; }

__device__ __forceinline__ v8s pack_acc(const v16f& x, int s) {
  v8s r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f_to_bf16_bits(x[8 * s + j]);
  return r;
}

// A fragment from T[row][col] with k along the columns in the permuted accumulator
// order: element j <-> column 16 s + 8 (j >> 2) + 4 h + (j & 3)
__device__ __forceinline__ v8s lds_perm(const short* T, int row, int s, int h) {
  const short* p = T + row * LT + 16 * s + 4 * h;
  const v4s lo = *reinterpret_cast<const v4s*>(p);
  const v4s hi = *reinterpret_cast<const v4s*>(p + 8);
  v8s r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// X^T staging for rows r0 .. r0+31 of X (row stride ld, D columns) into T[D][LT], split
// into a global read into registers (issued a block ahead) and the LDS write; rows at
// or past n are zeros.  Thread t < 2 D moves 2 rows x 8 columns as 8 4-byte stores.
template <int D>
__device__ __forceinline__ void load_t32(const bf16* X, int64_t ld, int r0, int n, v8s& x0, v8s& x1) {
  constexpr int C8 = D / 8;
  const int idx = threadIdx.x;
  x0 = zero8();
  x1 = zero8();
  if (idx < 16 * C8) {
    const int rp = idx & 15, c = idx >> 4;          // row pair, 8-column group
    const int ra = r0 + 2 * rp;
    if (ra < n) x0 = ld8(X + (int64_t)ra * ld + 8 * c);
    if (ra + 1 < n) x1 = ld8(X + (int64_t)(ra + 1) * ld + 8 * c);
  }
}
template <int D>
__device__ __forceinline__ void store_t32(const v8s& x0, const v8s& x1, short* T) {
  constexpr int C8 = D / 8;
  const int idx = threadIdx.x;
  if (idx >= 16 * C8) return;
  const int rp = idx & 15, c = idx >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t pr = (uint32_t)(unsigned short)x0[i] | ((uint32_t)(unsigned short)x1[i] << 16);
    *reinterpret_cast<uint32_t*>(T + (8 * c + i) * LT + 2 * rp) = pr;
  }
}

// dropout multiplier (0 or 1/keep) of P[row][key]
__device__ __forceinline__ float drop1(uint64_t seed, uint64_t row, int key, int sk4, float keep) {
  const uint4 r = Philox::gen(seed, row * (uint64_t)sk4 + (uint64_t)(key >> 2));
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  return Philox::u01(rr[key & 3]) < keep ? 1.f / keep : 0.f;
}
// the 4 multipliers of keys key0 .. key0+3 (key0 % 4 == 0) of one row
__device__ __forceinline__ void drop4(uint64_t seed, uint64_t row, int key0, int sk4, float keep, float (&m)[4]) {
  const uint4 r = Philox::gen(seed, row * (uint64_t)sk4 + (uint64_t)(key0 >> 2));
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  const float inv = 1.f / keep;
#pragma unroll
  for (int t = 0; t < 4; ++t) m[t] = Philox::u01(rr[t]) < keep ? inv : 0.f;
}

__device__ __forceinline__ void store_rows4(bf16* dst, const v16f& o, int g, int h, float mul) {
  uint2 pk;
  pk.x = (unsigned)f_to_bf16_bits(o[4 * g] * mul) | ((unsigned)f_to_bf16_bits(o[4 * g + 1] * mul) << 16);
  pk.y = (unsigned)f_to_bf16_bits(o[4 * g + 2] * mul) | ((unsigned)f_to_bf16_bits(o[4 * g + 3] * mul) << 16);
  *reinterpret_cast<uint2*>(dst + 8 * g + 4 * h) = pk;
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// x op x[lane ^ 32] for both halves of the wave by one v_permlane32_swap (no LDS trip)
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }

// mask modes: none, key-only (the same additive row for every query of a (b, h): staged per
// block in LDS, pre-scaled by log2 e, -inf past Sk), general (per-element global reads)
enum { MK_NONE = 0, MK_KEY = 1, MK_FULL = 2 };

// -------------------------------------------------------------------------------------
// forward: workgroup = (b*NH + h, 128-query tile); wave w: queries q0 + 32 w + (lane & 31).
// Software-pipelined over 32-key blocks: while block j's scores, softmax and P.V run,
// block j+1's K fragments and V rows are in flight into registers; V^T is written to
// the other half of a double-buffered LDS image after the P.V, so one barrier per block.
// The softmax is VALU-bound (16 scores per lane per block against 8 MFMAs), so it runs
// in the log2 domain (scale * log2 e folded into one multiply, bare v_exp_f32), checks
// bounds / causality only on edge blocks, reads the key mask as 16-byte LDS vectors, and
// rescales O lazily: the running max moves only when some row's block max exceeds it by
// more than 8 (P <= 256, exact in fp32 accumulation), which after the first blocks is rare.
template <int D, bool DROP, int MK>
__global__ void __launch_bounds__(256) flash_fwd_k(FArgs a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int DS = D / 16, DB = D / 32;
  __shared__ short vt[2][D * LT];
  __shared__ __attribute__((aligned(16))) float msk[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int qt0 = blockIdx.y * WQ;
  const int qw0 = qt0 + 32 * w;
  const int q = qw0 + r;
  const bool qv = q < a.Sq;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const float* M = MK != MK_NONE ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const float sl2 = a.scale * kLog2e;

  v8s qf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) qf[ds] = qv ? ld8(Q + (int64_t)q * a.qs + 16 * ds + 8 * h) : zero8();
  v16f o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = v16f{0.f};
  float m = -INFINITY, l = 0.f;      // running max (log2 domain) and sum of this lane's half
  const int sk4 = (a.Sk + 3) >> 2;
  const uint64_t qrow = (uint64_t)bh * a.Sq + (qv ? q : 0);
  // causal: keys past the tile's last query contribute nothing
  const int kend = a.causal ? min(a.Sk, min(a.Sq, qt0 + WQ)) : a.Sk;

  auto key_mask = [&](int kb) -> float {
    const int key = kb + (int)threadIdx.x;
    return key < a.Sk ? M[(int64_t)key * a.mk] * kLog2e : -INFINITY;
  };
  // prologue: block 0 staged and its scores issued, block 1's K fragments in registers.
  // The loop computes block j+1's scores (MFMA) ahead of block j's softmax (VALU): the two
  // are independent, so the matrix pipe works while the VALU runs the exp2 / max / sum.
  auto kfrag = [&](int kb, v8s (&f)[DS]) {
    const int kr = kb + r;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) f[ds] = kr < a.Sk ? ld8(K + (int64_t)kr * a.ks + 16 * ds + 8 * h) : zero8();
  };
  v8s kf[DS], x0, x1;
  float mv = 0.f;
  load_t32<D>(V, a.vs, 0, a.Sk, x0, x1);
  if (MK == MK_KEY && threadIdx.x < KBLK) mv = key_mask(0);
  kfrag(0, kf);
  v16f sc_cur = v16f{0.f};
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) sc_cur = mfma(kf[ds], qf[ds], sc_cur);
  if (KBLK < kend) kfrag(KBLK, kf);
  store_t32<D>(x0, x1, vt[0]);
  if (MK == MK_KEY && threadIdx.x < KBLK) msk[0][threadIdx.x] = mv;
  __syncthreads();

  int buf = 0;
  for (int kb0 = 0; kb0 < kend; kb0 += KBLK, buf ^= 1) {
    const int nb = kb0 + KBLK;
    const bool more = nb < kend;
    v8s kn[DS];
    if (more) {
      load_t32<D>(V, a.vs, nb, a.Sk, x0, x1);
      if (MK == MK_KEY && threadIdx.x < KBLK) mv = key_mask(nb);
      if (nb + KBLK < kend) kfrag(nb + KBLK, kn);
    }
    // block j+1's scores, independent of this block's softmax below
    v16f sc_next = v16f{0.f};
    if (more) {
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) sc_next = mfma(kf[ds], qf[ds], sc_next);
    }
    // a causal block wholly above this wave's queries adds nothing (wave-uniform skip)
    if (!(a.causal && kb0 > qw0 + 31)) {
      v16f sc = sc_cur;
      const bool full = MK != MK_FULL && nb <= a.Sk && !(a.causal && kb0 + KBLK - 1 > qw0);
      if (full) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4 mm = make_float4(0.f, 0.f, 0.f, 0.f);
          if (MK == MK_KEY) mm = *reinterpret_cast<const float4*>(&msk[buf][8 * g + 4 * h]);
          sc[4 * g] = fmaf(sc[4 * g], sl2, mm.x);
          sc[4 * g + 1] = fmaf(sc[4 * g + 1], sl2, mm.y);
          sc[4 * g + 2] = fmaf(sc[4 * g + 2], sl2, mm.z);
          sc[4 * g + 3] = fmaf(sc[4 * g + 3], sl2, mm.w);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kl = (i & 3) + 8 * (i >> 2) + 4 * h, key = kb0 + kl;
          float s = sc[i] * sl2;
          if (MK == MK_KEY) s += msk[buf][kl];
          if (MK == MK_FULL) s += key < a.Sk && qv ? M[(int64_t)q * a.mq + (int64_t)key * a.mk] * kLog2e : 0.f;
          if (key >= a.Sk || (a.causal && key > q)) s = -INFINITY;
          sc[i] = s;
        }
      }
      float mb = sc[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mb = fmaxf(mb, sc[i]);
      mb = xmax32(mb);
      if (__ballot(mb > m + 8.f)) {
        const float mn = fmaxf(m, mb);
        const float alpha = mn == -INFINITY ? 1.f : exp2_(m - mn);
#pragma unroll
        for (int db = 0; db < DB; ++db) o[db] *= alpha;
        l *= alpha;
        m = mn;
      }
      const float ms = m == -INFINITY ? 0.f : m;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float mul[4] = {1.f, 1.f, 1.f, 1.f};
        if (DROP) drop4(a.seed, qrow, kb0 + 8 * g + 4 * h, sk4, a.keep, mul);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int i = 4 * g + t;
          const float p = exp2_(sc[i] - ms);
          l += p;
          sc[i] = DROP ? p * mul[t] : p;
        }
      }
      const short* vb = vt[buf];
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int s = 0; s < 2; ++s) o[db] = mfma(lds_perm(vb, db * 32 + r, s, h), pack_acc(sc, s), o[db]);
    }
    if (more) {
      store_t32<D>(x0, x1, vt[buf ^ 1]);
      if (MK == MK_KEY && threadIdx.x < KBLK) msk[buf ^ 1][threadIdx.x] = mv;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) kf[ds] = kn[ds];
    }
    sc_cur = sc_next;
    __syncthreads();
  }
  l = xsum32(l);
  if (!qv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (h == 0) a.lse[(int64_t)bh * a.Sq + q] = l > 0.f ? m * kLn2 + __logf(l) : -INFINITY;
  bf16* O = a.o + b * a.ob + hh * a.oh + (int64_t)q * a.os;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) store_rows4(O + db * 32, o[db], g, h, inv);
}

// -------------------------------------------------------------------------------------
// D[row] = sum_d dO[row][d] * O[row][d] (fp32), 8 lanes per row
template <int D>
__global__ void __launch_bounds__(256) flash_dsum_k(FArgs a, float* dsum) {
  constexpr int C8 = D / 8;
  const int64_t rows = (int64_t)a.B * a.NH * a.Sq;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = idx / 8;
  const int c = (int)(idx & 7);
  float p = 0.f;
  if (row < rows) {
    const int64_t bh = row / a.Sq;
    const int qq = (int)(row - bh * a.Sq);
    const int b = (int)(bh / a.NH), hh = (int)(bh - (int64_t)b * a.NH);
    const bf16* G = a.dout + b * a.gb + hh * a.gh + (int64_t)qq * a.gs;
    const bf16* O = a.o + b * a.ob + hh * a.oh + (int64_t)qq * a.os;
    for (int cc = c; cc < C8; cc += 8) {
      const v8s x = ld8(G + 8 * cc), y = ld8(O + 8 * cc);
#pragma unroll
      for (int i = 0; i < 8; ++i) p += bf16_bits_to_f((unsigned short)x[i]) * bf16_bits_to_f((unsigned short)y[i]);
    }
  }
  p += __shfl_xor(p, 1, 64);
  p += __shfl_xor(p, 2, 64);
  p += __shfl_xor(p, 4, 64);
  if (row < rows && c == 0) dsum[row] = p;
}

// -------------------------------------------------------------------------------------
// dQ: the forward's walk (lane = query) with P from the saved lse and dP^T = V . dO^T,
// pipelined like the forward (next block's K / V fragments and K rows in flight,
// double-buffered K^T image, one barrier per block)
template <int D, bool DROP, int MK>
__global__ void __launch_bounds__(256) flash_dq_k(FArgs a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool PF = D <= 32;     // fragments a block ahead only where registers allow 2 waves / SIMD
  __shared__ short kt[2][D * LT];
  __shared__ __attribute__((aligned(16))) float msk[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int qt0 = blockIdx.y * WQ;
  const int qw0 = qt0 + 32 * w;
  const int q = qw0 + r;
  const bool qv = q < a.Sq;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const bf16* G = a.dout + b * a.gb + hh * a.gh;
  const float* M = MK != MK_NONE ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const float sl2 = a.scale * kLog2e;
  v8s qf[DS], gf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    qf[ds] = qv ? ld8(Q + (int64_t)q * a.qs + 16 * ds + 8 * h) : zero8();
    gf[ds] = qv ? ld8(G + (int64_t)q * a.gs + 16 * ds + 8 * h) : zero8();
  }
  // P = exp2(S log2e - lse log2e); a row with no live key (lse = -inf) or past Sq gets +inf: P = 0
  const float lse0 = qv ? a.lse[(int64_t)bh * a.Sq + q] : -INFINITY;
  const float lse2 = lse0 == -INFINITY ? INFINITY : lse0 * kLog2e;
  const float Dq = qv ? a.dsum[(int64_t)bh * a.Sq + q] : 0.f;
  v16f o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = v16f{0.f};
  const int sk4 = (a.Sk + 3) >> 2;
  const uint64_t qrow = (uint64_t)bh * a.Sq + (qv ? q : 0);
  const int kend = a.causal ? min(a.Sk, min(a.Sq, qt0 + WQ)) : a.Sk;

  v8s kf[DS], vf[DS], x0, x1;
  float mv = 0.f;
  load_t32<D>(K, a.ks, 0, a.Sk, x0, x1);
  auto key_mask = [&](int kb) -> float {
    const int key = kb + (int)threadIdx.x;
    return key < a.Sk ? M[(int64_t)key * a.mk] * kLog2e : -INFINITY;
  };
  if (MK == MK_KEY && threadIdx.x < KBLK) mv = key_mask(0);
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    kf[ds] = r < a.Sk ? ld8(K + (int64_t)r * a.ks + 16 * ds + 8 * h) : zero8();
    vf[ds] = r < a.Sk ? ld8(V + (int64_t)r * a.vs + 16 * ds + 8 * h) : zero8();
  }
  store_t32<D>(x0, x1, kt[0]);
  if (MK == MK_KEY && threadIdx.x < KBLK) msk[0][threadIdx.x] = mv;
  __syncthreads();

  int buf = 0;
  for (int kb0 = 0; kb0 < kend; kb0 += KBLK, buf ^= 1) {
    const int nb = kb0 + KBLK;
    const bool more = nb < kend;
    v8s kn[DS], vn[DS];
    if (!PF && kb0 > 0) {
      const int kr = kb0 + r;
      const bool kv = kr < a.Sk;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        kf[ds] = kv ? ld8(K + (int64_t)kr * a.ks + 16 * ds + 8 * h) : zero8();
        vf[ds] = kv ? ld8(V + (int64_t)kr * a.vs + 16 * ds + 8 * h) : zero8();
      }
    }
    if (more) {
      load_t32<D>(K, a.ks, nb, a.Sk, x0, x1);
      if (MK == MK_KEY && threadIdx.x < KBLK) mv = key_mask(nb);
      if (PF) {
        const int kr = nb + r;
        const bool kv = kr < a.Sk;
#pragma unroll
        for (int ds = 0; ds < DS; ++ds) {
          kn[ds] = kv ? ld8(K + (int64_t)kr * a.ks + 16 * ds + 8 * h) : zero8();
          vn[ds] = kv ? ld8(V + (int64_t)kr * a.vs + 16 * ds + 8 * h) : zero8();
        }
      }
    }
    if (!(a.causal && kb0 > qw0 + 31)) {
      v16f sc = v16f{0.f}, dp = v16f{0.f};
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        sc = mfma(kf[ds], qf[ds], sc);
        dp = mfma(vf[ds], gf[ds], dp);
      }
      const bool full = MK != MK_FULL && nb <= a.Sk && !(a.causal && kb0 + KBLK - 1 > qw0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float mul[4] = {1.f, 1.f, 1.f, 1.f};
        if (DROP) drop4(a.seed, qrow, kb0 + 8 * g + 4 * h, sk4, a.keep, mul);
        float4 mm = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MK == MK_KEY) mm = *reinterpret_cast<const float4*>(&msk[buf][8 * g + 4 * h]);
        const float mk4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int i = 4 * g + t;
          float x = fmaf(sc[i], sl2, mk4[t] - lse2);
          if (!full) {
            const int key = kb0 + 8 * g + 4 * h + t;
            if (MK == MK_FULL) x += key < a.Sk && qv ? M[(int64_t)q * a.mq + (int64_t)key * a.mk] * kLog2e : 0.f;
            if (key >= a.Sk || (a.causal && key > q)) x = -INFINITY;
          }
          const float p = exp2_(x);
          // dS / scale (the scale goes on at the dQ store)
          sc[i] = p * (DROP ? fmaf(dp[i], mul[t], -Dq) : dp[i] - Dq);
        }
      }
      const short* kb = kt[buf];
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int s = 0; s < 2; ++s) o[db] = mfma(lds_perm(kb, db * 32 + r, s, h), pack_acc(sc, s), o[db]);
    }
    if (more) {
      store_t32<D>(x0, x1, kt[buf ^ 1]);
      if (MK == MK_KEY && threadIdx.x < KBLK) msk[buf ^ 1][threadIdx.x] = mv;
      if (PF) {
#pragma unroll
        for (int ds = 0; ds < DS; ++ds) { kf[ds] = kn[ds]; vf[ds] = vn[ds]; }
      }
    }
    __syncthreads();
  }
  if (!qv) return;
  bf16* dQ = a.dq + b * a.dqb + hh * a.dqh + (int64_t)q * a.dqs;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) store_rows4(dQ + db * 32, o[db], g, h, a.scale);
}

// -------------------------------------------------------------------------------------
// dK, dV: workgroup = (b*NH + h, 128-key tile), lane = key; walk over 32-query blocks:
// S = Q . K^T (A = Q rows, B = this lane's K row), dP = dO . V^T, then
// dV^T += dO^T . P_drop and dK^T += Q^T . dS with dO^T / Q^T staged in double-buffered
// LDS from registers loaded a block ahead (the Q / dO fragments too at D = 32; above
// that they would cost the second wave per SIMD).
template <int D, bool DROP, int MK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D <= 64 ? 2 : 1))) flash_dkdv_k(FArgs a) {
  a.seed = rng_seed(a.seed, a.rngo);
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool PF = D <= 32;
  __shared__ short qt[2][D * LT];
  __shared__ short gt[2][D * LT];
  __shared__ __attribute__((aligned(16))) float ls[2][KBLK];
  __shared__ __attribute__((aligned(16))) float dl[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int kt0 = blockIdx.y * WQ;
  const int kw0 = kt0 + 32 * w;
  const int key = kw0 + r;
  const bool kv = key < a.Sk;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const bf16* G = a.dout + b * a.gb + hh * a.gh;
  const float* M = MK != MK_NONE ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const float sl2 = a.scale * kLog2e;
  const float* LSE = a.lse + (int64_t)bh * a.Sq;
  const float* DSUM = a.dsum + (int64_t)bh * a.Sq;
  v8s kf[DS], vf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    kf[ds] = kv ? ld8(K + (int64_t)key * a.ks + 16 * ds + 8 * h) : zero8();
    vf[ds] = kv ? ld8(V + (int64_t)key * a.vs + 16 * ds + 8 * h) : zero8();
  }
  // this lane's key-mask term (log2 domain); a key past Sk gets -inf: P = 0
  const float mkey = !kv ? -INFINITY : (MK == MK_KEY ? M[(int64_t)key * a.mk] * kLog2e : 0.f);
  v16f dvt[DB], dkt[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) { dvt[db] = v16f{0.f}; dkt[db] = v16f{0.f}; }
  const int sk4 = (a.Sk + 3) >> 2;
  // causal: queries before the tile's first key see none of its keys
  const int qstart = a.causal ? (kt0 / KBLK) * KBLK : 0;
  if (qstart >= a.Sq) {
    // no query reaches these keys: zero gradients
    if (!kv) return;
    bf16* dK = a.dk + b * a.dkb + hh * a.dkh + (int64_t)key * a.dks;
    bf16* dV = a.dv + b * a.dvb + hh * a.dvh + (int64_t)key * a.dvs;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        store_rows4(dK + db * 32, dkt[db], g, h, 1.f);
        store_rows4(dV + db * 32, dvt[db], g, h, 1.f);
      }
    return;
  }

  v8s x0, x1, y0, y1, qf[DS], gf[DS];
  float lv = INFINITY, dv = 0.f;
  auto fetch = [&](int qb0) {
    load_t32<D>(Q, a.qs, qb0, a.Sq, x0, x1);
    load_t32<D>(G, a.gs, qb0, a.Sq, y0, y1);
    if (threadIdx.x < KBLK) {
      // lse in log2 units; +inf (P = 0) for rows past Sq and rows with no live key
      const int qq = qb0 + threadIdx.x;
      const float x = qq < a.Sq ? LSE[qq] : -INFINITY;
      lv = x == -INFINITY ? INFINITY : x * kLog2e;
      dv = qq < a.Sq ? DSUM[qq] : 0.f;
    }
  };
  auto frags = [&](int qb0) {
    const int qr = qb0 + r;
    const bool qrv = qr < a.Sq;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      qf[ds] = qrv ? ld8(Q + (int64_t)qr * a.qs + 16 * ds + 8 * h) : zero8();
      gf[ds] = qrv ? ld8(G + (int64_t)qr * a.gs + 16 * ds + 8 * h) : zero8();
    }
  };
  auto put = [&](int bf) {
    store_t32<D>(x0, x1, qt[bf]);
    store_t32<D>(y0, y1, gt[bf]);
    if (threadIdx.x < KBLK) { ls[bf][threadIdx.x] = lv; dl[bf][threadIdx.x] = dv; }
  };
  fetch(qstart);
  if (PF) frags(qstart);
  put(0);
  __syncthreads();

  int buf = 0;
  for (int qb0 = qstart; qb0 < a.Sq; qb0 += KBLK, buf ^= 1) {
    const int nb = qb0 + KBLK;
    const bool more = nb < a.Sq;
    v8s qa[DS], ga[DS];
    if (PF) {
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) { qa[ds] = qf[ds]; ga[ds] = gf[ds]; }
    } else {
      frags(qb0);
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) { qa[ds] = qf[ds]; ga[ds] = gf[ds]; }
    }
    if (more) {
      fetch(nb);
      if (PF) frags(nb);
    }
    // causal: a query block wholly before this wave's keys sees none of them
    if (!(a.causal && kw0 > qb0 + 31)) {
      v16f sc = v16f{0.f}, dp = v16f{0.f};
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        sc = mfma(qa[ds], kf[ds], sc);
        dp = mfma(ga[ds], vf[ds], dp);
      }
      const bool full = MK != MK_FULL && !(a.causal && kw0 + 31 > qb0);
      v16f pd;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(&ls[buf][8 * g + 4 * h]);
        const float4 d4 = *reinterpret_cast<const float4*>(&dl[buf][8 * g + 4 * h]);
        const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int i = 4 * g + t, qq = qb0 + 8 * g + 4 * h + t;
          float x = fmaf(sc[i], sl2, mkey - lq[t]);
          if (!full) {
            if (MK == MK_FULL) x += kv && qq < a.Sq ? M[(int64_t)qq * a.mq + (int64_t)key * a.mk] * kLog2e : 0.f;
            if (a.causal && key > qq) x = -INFINITY;
          }
          const float p = exp2_(x);
          const float mul = DROP ? drop1(a.seed, (uint64_t)bh * a.Sq + qq, key, sk4, a.keep) : 1.f;
          pd[i] = DROP ? p * mul : p;
          // dS / scale (the scale goes on at the dK store)
          sc[i] = p * (DROP ? fmaf(dp[i], mul, -dq4[t]) : dp[i] - dq4[t]);
        }
      }
      const short* gb = gt[buf];
      const short* qb = qt[buf];
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dvt[db] = mfma(lds_perm(gb, db * 32 + r, s, h), pack_acc(pd, s), dvt[db]);
          dkt[db] = mfma(lds_perm(qb, db * 32 + r, s, h), pack_acc(sc, s), dkt[db]);
        }
    }
    if (more) put(buf ^ 1);
    __syncthreads();
  }
  if (!kv) return;
  bf16* dK = a.dk + b * a.dkb + hh * a.dkh + (int64_t)key * a.dks;
  bf16* dV = a.dv + b * a.dvb + hh * a.dvh + (int64_t)key * a.dvs;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store_rows4(dK + db * 32, dkt[db], g, h, a.scale);
      store_rows4(dV + db * 32, dvt[db], g, h, 1.f);
    }
}

static int mask_mode(const FArgs& a) { return a.mask == nullptr ? MK_NONE : (a.mq == 0 ? MK_KEY : MK_FULL); }

template <int D, int MK>
static void fwd_dm(const FArgs& a, hipStream_t st) {
  dim3 grid((unsigned)(a.B * a.NH), (unsigned)((a.Sq + WQ - 1) / WQ));
  if (a.keep < 1.f) hipLaunchKernelGGL((flash_fwd_k<D, true, MK>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((flash_fwd_k<D, false, MK>), grid, dim3(256), 0, st, a);
}

template <int D>
static int fwd_d(const FArgs& a, hipStream_t st) {
  switch (mask_mode(a)) {
    case MK_NONE: fwd_dm<D, MK_NONE>(a, st); break;
    case MK_KEY: fwd_dm<D, MK_KEY>(a, st); break;
    default: fwd_dm<D, MK_FULL>(a, st); break;
  }
  return (int)hipGetLastError();
}

template <int D, int MK>
static void bwd_dm(const FArgs& b, hipStream_t st) {
  dim3 gq((unsigned)(b.B * b.NH), (unsigned)((b.Sq + WQ - 1) / WQ));
  dim3 gk((unsigned)(b.B * b.NH), (unsigned)((b.Sk + WQ - 1) / WQ));
  if (b.keep < 1.f) {
    hipLaunchKernelGGL((flash_dq_k<D, true, MK>), gq, dim3(256), 0, st, b);
    hipLaunchKernelGGL((flash_dkdv_k<D, true, MK>), gk, dim3(256), 0, st, b);
  } else {
    hipLaunchKernelGGL((flash_dq_k<D, false, MK>), gq, dim3(256), 0, st, b);
    hipLaunchKernelGGL((flash_dkdv_k<D, false, MK>), gk, dim3(256), 0, st, b);
  }
}

template <int D>
static int bwd_d(const FArgs& a, float* dsum, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.NH * a.Sq;
  hipLaunchKernelGGL((flash_dsum_k<D>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, st, a, dsum);
  FArgs b = a;
  b.dsum = dsum;
  switch (mask_mode(a)) {
    case MK_NONE: bwd_dm<D, MK_NONE>(b, st); break;
    case MK_KEY: bwd_dm<D, MK_KEY>(b, st); break;
    default: bwd_dm<D, MK_FULL>(b, st); break;
  }
  return (int)hipGetLastError();
}

// ring attention (parallel/ring_attention.py): merge one key block's (o_b, lse_b) into the
// running fp32 (o, lse) by the log-sum-exp rule; one thread per (b, s, h) row of D values.
// o: [B, S, NH, D] fp32; ob: [B, S, NH, D] bf16; lse / lb: [B, NH, S].
__global__ void __launch_bounds__(256) lse_merge_k(float* __restrict__ o, float* __restrict__ lse,
                                                   const bf16* __restrict__ ob, const float* __restrict__ lb,
                                                   int B, int S, int NH, int D) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * S * NH) return;
  const int hh = (int)(t % NH);
  const int64_t bs = t / NH;
  const int ss = (int)(bs % S), b = (int)(bs / S);
  const int64_t li = ((int64_t)b * NH + hh) * S + ss;
  const float la = lse[li], lbb = lb[li];
  const float m = fmaxf(la, lbb);
  if (m == -INFINITY) return;
  const float nw = m + __logf(__expf(la - m) + __expf(lbb - m));
  const float wa = __expf(la - nw), wb = __expf(lbb - nw);
  float* orow = o + t * D;
  const bf16* brow = ob + t * D;
  for (int c = 0; c < D; c += 8) {
    const v8s x = ld8(brow + c);
    float4* p = reinterpret_cast<float4*>(orow + c);
    float4 u = p[0], v = p[1];
    u.x = u.x * wa + bf16_bits_to_f((unsigned short)x[0]) * wb;
    u.y = u.y * wa + bf16_bits_to_f((unsigned short)x[1]) * wb;
    u.z = u.z * wa + bf16_bits_to_f((unsigned short)x[2]) * wb;
    u.w = u.w * wa + bf16_bits_to_f((unsigned short)x[3]) * wb;
    v.x = v.x * wa + bf16_bits_to_f((unsigned short)x[4]) * wb;
    v.y = v.y * wa + bf16_bits_to_f((unsigned short)x[5]) * wb;
    v.z = v.z * wa + bf16_bits_to_f((unsigned short)x[6]) * wb;
    v.w = v.w * wa + bf16_bits_to_f((unsigned short)x[7]) * wb;
    p[0] = u;
    p[1] = v;
  }
  lse[li] = nw;
}

// acc[r][c] += x[r][c] (fp32 += bf16) over rows x cols (cols % 8 == 0), row strides lda / ldx
__global__ void __launch_bounds__(256) acc_rows_k(float* __restrict__ acc, int64_t lda, const bf16* __restrict__ x,
                                                  int64_t ldx, int64_t rows, int cols) {
  const int c8 = cols / 8;
  const int64_t n = rows * c8;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / c8;
    const int c = (int)(t - r * c8) * 8;
    const v8s v = ld8(x + r * ldx + c);
    float4* p = reinterpret_cast<float4*>(acc + r * lda + c);
    float4 u = p[0], w = p[1];
    u.x += bf16_bits_to_f((unsigned short)v[0]); u.y += bf16_bits_to_f((unsigned short)v[1]);
    u.z += bf16_bits_to_f((unsigned short)v[2]); u.w += bf16_bits_to_f((unsigned short)v[3]);
    w.x += bf16_bits_to_f((unsigned short)v[4]); w.y += bf16_bits_to_f((unsigned short)v[5]);
    w.z += bf16_bits_to_f((unsigned short)v[6]); w.w += bf16_bits_to_f((unsigned short)v[7]);
    p[0] = u;
    p[1] = w;
  }
}

}  // namespace flash
}  // namespace hetu

using namespace hetu;
using namespace hetu::flash;

// strides: [b, h, s] per tensor (elements); the head dim is contiguous and 16-byte aligned.
// mask: fp32 additive, strides [b, h, q, k] (0 on broadcast dims), or null.
HETU_API int hetu_flash_fwd(const void* q, const void* k, const void* v, const int64_t* qst, const int64_t* kst,
                            const int64_t* vst, void* o, const int64_t* ost, float* lse, const float* mask,
                            const int64_t* mst, int B, int NH, int Sq, int Sk, int D, int causal, float scale,
                            float keep, int64_t seed, hipStream_t st) {
  if (B <= 0 || NH <= 0 || Sq <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  if (D != 32 && D != 64 && D != 128) return (int)hipErrorInvalidValue;
  FArgs a;
  memset(&a, 0, sizeof(a));
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v;
  a.qb = qst[0]; a.qh = qst[1]; a.qs = qst[2];
  a.kb = kst[0]; a.kh = kst[1]; a.ks = kst[2];
  a.vb = vst[0]; a.vh = vst[1]; a.vs = vst[2];
  a.o = (bf16*)o; a.ob = ost[0]; a.oh = ost[1]; a.os = ost[2];
  a.lse = lse;
  a.mask = mask;
  if (mask) { a.mb = mst[0]; a.mh = mst[1]; a.mq = mst[2]; a.mk = mst[3]; }
  a.B = B; a.NH = NH; a.Sq = Sq; a.Sk = Sk;
  a.scale = scale; a.keep = keep; a.seed = (uint64_t)seed; a.rngo = hetu_rng_offset_ptr(); a.causal = causal;
  if (D == 32) return fwd_d<32>(a, st);
  if (D == 64) return fwd_d<64>(a, st);
  return fwd_d<128>(a, st);
}

// dsum: [B * NH * Sq] fp32 workspace
HETU_API int hetu_flash_bwd(const void* q, const void* k, const void* v, const int64_t* qst, const int64_t* kst,
                            const int64_t* vst, const void* o, const int64_t* ost, const float* lse,
                            const void* dout, const int64_t* gst, void* dq, const int64_t* dqst, void* dk,
                            const int64_t* dkst, void* dv, const int64_t* dvst, const float* mask,
                            const int64_t* mst, float* dsum, int B, int NH, int Sq, int Sk, int D, int causal,
                            float scale, float keep, int64_t seed, hipStream_t st) {
  if (B <= 0 || NH <= 0 || Sq <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  if (D != 32 && D != 64 && D != 128) return (int)hipErrorInvalidValue;
  FArgs a;
  memset(&a, 0, sizeof(a));
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v;
  a.qb = qst[0]; a.qh = qst[1]; a.qs = qst[2];
  a.kb = kst[0]; a.kh = kst[1]; a.ks = kst[2];
  a.vb = vst[0]; a.vh = vst[1]; a.vs = vst[2];
  a.o = (bf16*)o; a.ob = ost[0]; a.oh = ost[1]; a.os = ost[2];
  a.lse = (float*)lse;
  a.dout = (const bf16*)dout; a.gb = gst[0]; a.gh = gst[1]; a.gs = gst[2];
  a.dq = (bf16*)dq; a.dqb = dqst[0]; a.dqh = dqst[1]; a.dqs = dqst[2];
  a.dk = (bf16*)dk; a.dkb = dkst[0]; a.dkh = dkst[1]; a.dks = dkst[2];
  a.dv = (bf16*)dv; a.dvb = dvst[0]; a.dvh = dvst[1]; a.dvs = dvst[2];
  a.mask = mask;
  if (mask) { a.mb = mst[0]; a.mh = mst[1]; a.mq = mst[2]; a.mk = mst[3]; }
  a.B = B; a.NH = NH; a.Sq = Sq; a.Sk = Sk;
  a.scale = scale; a.keep = keep; a.seed = (uint64_t)seed; a.rngo = hetu_rng_offset_ptr(); a.causal = causal;
  if (D == 32) return bwd_d<32>(a, dsum, st);
  if (D == 64) return bwd_d<64>(a, dsum, st);
  return bwd_d<128>(a, dsum, st);
}

HETU_API int hetu_flash_lse_merge(float* o, float* lse, const void* ob, const float* lb, int B, int S, int NH, int D,
                                  hipStream_t st) {
  if (D % 8) return (int)hipErrorInvalidValue;
  const int64_t rows = (int64_t)B * S * NH;
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(lse_merge_k, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, o, lse, (const bf16*)ob, lb,
                     B, S, NH, D);
  return (int)hipGetLastError();
}

HETU_API int hetu_acc_rows_bf16(float* acc, int64_t lda, const void* x, int64_t ldx, int64_t rows, int cols,
                                hipStream_t st) {
  if (cols % 8 || lda % 4 || ldx % 8) return (int)hipErrorInvalidValue;
  if (rows <= 0 || cols <= 0) return 0;
  const int g = stream_grid(rows * (cols / 8), 256, 4);
  hipLaunchKernelGGL(acc_rows_k, dim3(g), dim3(256), 0, st, acc, lda, (const bf16*)x, ldx, rows, cols);
  return (int)hipGetLastError();
}
