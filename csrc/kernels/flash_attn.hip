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

// -------------------------------------------------------------------------------------
// forward: workgroup = (b*NH + h, 128-query tile); wave w: queries q0 + 32 w + (lane & 31).
// Software-pipelined over 32-key blocks: while block j's scores, softmax and P.V run,
// block j+1's K fragments and V rows are in flight into registers; V^T is written to
// the other half of a double-buffered LDS image after the P.V, so one barrier per block.
template <int D, bool DROP>
__global__ void __launch_bounds__(256) flash_fwd_k(FArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  __shared__ short vt[2][D * LT];
  __shared__ float msk[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int qt0 = blockIdx.y * WQ;
  const int q = qt0 + 32 * w + r;
  const bool qv = q < a.Sq;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const float* M = a.mask ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const bool mrow = M != nullptr && a.mq == 0;     // key-only mask: staged per block

  v8s qf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) qf[ds] = qv ? ld8(Q + (int64_t)q * a.qs + 16 * ds + 8 * h) : zero8();
  v16f o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = v16f{0.f};
  float m = -INFINITY, l = 0.f;
  const int sk4 = (a.Sk + 3) >> 2;
  const uint64_t qrow = (uint64_t)bh * a.Sq + (qv ? q : 0);
  // causal: keys past the tile's last query contribute nothing
  const int kend = a.causal ? min(a.Sk, min(a.Sq, qt0 + WQ)) : a.Sk;

  // prologue: block 0 staged, its K fragments in registers
  v8s kf[DS], x0, x1;
  float mv = 0.f;
  load_t32<D>(V, a.vs, 0, a.Sk, x0, x1);
  if (mrow && threadIdx.x < KBLK) mv = threadIdx.x < a.Sk ? M[(int64_t)threadIdx.x * a.mk] : 0.f;
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) kf[ds] = r < a.Sk ? ld8(K + (int64_t)r * a.ks + 16 * ds + 8 * h) : zero8();
  store_t32<D>(x0, x1, vt[0]);
  if (mrow && threadIdx.x < KBLK) msk[0][threadIdx.x] = mv;
  __syncthreads();

  int buf = 0;
  for (int kb0 = 0; kb0 < kend; kb0 += KBLK, buf ^= 1) {
    const int nb = kb0 + KBLK;
    const bool more = nb < kend;
    v8s kn[DS];
    if (more) {
      load_t32<D>(V, a.vs, nb, a.Sk, x0, x1);
      if (mrow && threadIdx.x < KBLK) mv = nb + threadIdx.x < a.Sk ? M[(int64_t)(nb + threadIdx.x) * a.mk] : 0.f;
      const int kr = nb + r;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) kn[ds] = kr < a.Sk ? ld8(K + (int64_t)kr * a.ks + 16 * ds + 8 * h) : zero8();
    }
    v16f sc = v16f{0.f};
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) sc = mfma(kf[ds], qf[ds], sc);
    float mb = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kl = (i & 3) + 8 * (i >> 2) + 4 * h, key = kb0 + kl;
      float s = sc[i] * a.scale;
      if (M != nullptr) s += mrow ? msk[buf][kl] : (key < a.Sk && qv ? M[(int64_t)q * a.mq + (int64_t)key * a.mk] : 0.f);
      if (key >= a.Sk || (a.causal && key > q)) s = -INFINITY;
      sc[i] = s;
      mb = fmaxf(mb, s);
    }
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float mn = fmaxf(m, mb);
    const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
#pragma unroll
    for (int db = 0; db < DB; ++db) o[db] *= alpha;
    l *= alpha;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float mul[4] = {1.f, 1.f, 1.f, 1.f};
      if (DROP) drop4(a.seed, qrow, kb0 + 8 * g + 4 * h, sk4, a.keep, mul);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = 4 * g + t;
        const float p = mn == -INFINITY ? 0.f : __expf(sc[i] - mn);
        l += p;
        sc[i] = p * mul[t];
      }
    }
    m = mn;
    const short* vb = vt[buf];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int s = 0; s < 2; ++s) o[db] = mfma(lds_perm(vb, db * 32 + r, s, h), pack_acc(sc, s), o[db]);
    if (more) {
      store_t32<D>(x0, x1, vt[buf ^ 1]);
      if (mrow && threadIdx.x < KBLK) msk[buf ^ 1][threadIdx.x] = mv;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) kf[ds] = kn[ds];
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (h == 0) a.lse[(int64_t)bh * a.Sq + q] = l > 0.f ? m + __logf(l) : -INFINITY;
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
template <int D, bool DROP>
__global__ void __launch_bounds__(256) flash_dq_k(FArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool PF = D <= 32;     // fragments a block ahead only where registers allow 2 waves / SIMD
  __shared__ short kt[2][D * LT];
  __shared__ float msk[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int qt0 = blockIdx.y * WQ;
  const int q = qt0 + 32 * w + r;
  const bool qv = q < a.Sq;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const bf16* G = a.dout + b * a.gb + hh * a.gh;
  const float* M = a.mask ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const bool mrow = M != nullptr && a.mq == 0;
  v8s qf[DS], gf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    qf[ds] = qv ? ld8(Q + (int64_t)q * a.qs + 16 * ds + 8 * h) : zero8();
    gf[ds] = qv ? ld8(G + (int64_t)q * a.gs + 16 * ds + 8 * h) : zero8();
  }
  const float lse = qv ? a.lse[(int64_t)bh * a.Sq + q] : 0.f;
  const float Dq = qv ? a.dsum[(int64_t)bh * a.Sq + q] : 0.f;
  const bool live = qv && lse != -INFINITY;
  v16f o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = v16f{0.f};
  const int sk4 = (a.Sk + 3) >> 2;
  const uint64_t qrow = (uint64_t)bh * a.Sq + (qv ? q : 0);
  const int kend = a.causal ? min(a.Sk, min(a.Sq, qt0 + WQ)) : a.Sk;

  v8s kf[DS], vf[DS], x0, x1;
  float mv = 0.f;
  load_t32<D>(K, a.ks, 0, a.Sk, x0, x1);
  if (mrow && threadIdx.x < KBLK) mv = threadIdx.x < a.Sk ? M[(int64_t)threadIdx.x * a.mk] : 0.f;
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    kf[ds] = r < a.Sk ? ld8(K + (int64_t)r * a.ks + 16 * ds + 8 * h) : zero8();
    vf[ds] = r < a.Sk ? ld8(V + (int64_t)r * a.vs + 16 * ds + 8 * h) : zero8();
  }
  store_t32<D>(x0, x1, kt[0]);
  if (mrow && threadIdx.x < KBLK) msk[0][threadIdx.x] = mv;
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
      if (mrow && threadIdx.x < KBLK) mv = nb + threadIdx.x < a.Sk ? M[(int64_t)(nb + threadIdx.x) * a.mk] : 0.f;
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
    v16f sc = v16f{0.f}, dp = v16f{0.f};
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      sc = mfma(kf[ds], qf[ds], sc);
      dp = mfma(vf[ds], gf[ds], dp);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float mul[4] = {1.f, 1.f, 1.f, 1.f};
      if (DROP) drop4(a.seed, qrow, kb0 + 8 * g + 4 * h, sk4, a.keep, mul);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = 4 * g + t;
        const int kl = 8 * g + 4 * h + t, key = kb0 + kl;
        float s = sc[i] * a.scale;
        if (M != nullptr) s += mrow ? msk[buf][kl] : (key < a.Sk && qv ? M[(int64_t)q * a.mq + (int64_t)key * a.mk] : 0.f);
        const bool ok = live && key < a.Sk && !(a.causal && key > q);
        const float p = ok ? __expf(s - lse) : 0.f;
        sc[i] = p * (dp[i] * mul[t] - Dq) * a.scale;
      }
    }
    const short* kb = kt[buf];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int s = 0; s < 2; ++s) o[db] = mfma(lds_perm(kb, db * 32 + r, s, h), pack_acc(sc, s), o[db]);
    if (more) {
      store_t32<D>(x0, x1, kt[buf ^ 1]);
      if (mrow && threadIdx.x < KBLK) msk[buf ^ 1][threadIdx.x] = mv;
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
    for (int g = 0; g < 4; ++g) store_rows4(dQ + db * 32, o[db], g, h, 1.f);
}

// -------------------------------------------------------------------------------------
// dK, dV: workgroup = (b*NH + h, 128-key tile), lane = key; walk over 32-query blocks:
// S = Q . K^T (A = Q rows, B = this lane's K row), dP = dO . V^T, then
// dV^T += dO^T . P_drop and dK^T += Q^T . dS with dO^T / Q^T staged in double-buffered
// LDS from registers loaded a block ahead (the Q / dO fragments too at D = 32; above
// that they would cost the second wave per SIMD).
template <int D, bool DROP>
__global__ void __launch_bounds__(256) flash_dkdv_k(FArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool PF = D <= 32;
  __shared__ short qt[2][D * LT];
  __shared__ short gt[2][D * LT];
  __shared__ float ls[2][KBLK], dl[2][KBLK];
  const int bh = blockIdx.x, b = bh / a.NH, hh = bh - b * a.NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int kt0 = blockIdx.y * WQ;
  const int key = kt0 + 32 * w + r;
  const bool kv = key < a.Sk;
  const bf16* Q = a.q + b * a.qb + hh * a.qh;
  const bf16* K = a.k + b * a.kb + hh * a.kh;
  const bf16* V = a.v + b * a.vb + hh * a.vh;
  const bf16* G = a.dout + b * a.gb + hh * a.gh;
  const float* M = a.mask ? a.mask + b * a.mb + hh * a.mh : nullptr;
  const float* LSE = a.lse + (int64_t)bh * a.Sq;
  const float* DSUM = a.dsum + (int64_t)bh * a.Sq;
  v8s kf[DS], vf[DS];
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    kf[ds] = kv ? ld8(K + (int64_t)key * a.ks + 16 * ds + 8 * h) : zero8();
    vf[ds] = kv ? ld8(V + (int64_t)key * a.vs + 16 * ds + 8 * h) : zero8();
  }
  const float mkey = (M != nullptr && a.mq == 0 && kv) ? M[(int64_t)key * a.mk] : 0.f;
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
  float lv = -INFINITY, dv = 0.f;
  auto fetch = [&](int qb0) {
    load_t32<D>(Q, a.qs, qb0, a.Sq, x0, x1);
    load_t32<D>(G, a.gs, qb0, a.Sq, y0, y1);
    if (threadIdx.x < KBLK) {
      const int qq = qb0 + threadIdx.x;
      const bool ok = qq < a.Sq;
      lv = ok ? LSE[qq] : -INFINITY;
      dv = ok ? DSUM[qq] : 0.f;
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
    v16f sc = v16f{0.f}, dp = v16f{0.f};
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      sc = mfma(qa[ds], kf[ds], sc);
      dp = mfma(ga[ds], vf[ds], dp);
    }
    v16f pd;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ql = (i & 3) + 8 * (i >> 2) + 4 * h, qq = qb0 + ql;
      const float lq = ls[buf][ql];
      float s = sc[i] * a.scale;
      if (M != nullptr) s += a.mq == 0 ? mkey : (kv && qq < a.Sq ? M[(int64_t)qq * a.mq + (int64_t)key * a.mk] : 0.f);
      const bool ok = kv && qq < a.Sq && lq != -INFINITY && !(a.causal && key > qq);
      const float p = ok ? __expf(s - lq) : 0.f;
      const float mul = (DROP && ok) ? drop1(a.seed, (uint64_t)bh * a.Sq + qq, key, sk4, a.keep) : 1.f;
      pd[i] = p * mul;
      sc[i] = p * (dp[i] * mul - dl[buf][ql]) * a.scale;
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
      store_rows4(dK + db * 32, dkt[db], g, h, 1.f);
      store_rows4(dV + db * 32, dvt[db], g, h, 1.f);
    }
}

template <int D>
static int fwd_d(const FArgs& a, hipStream_t st) {
  dim3 grid((unsigned)(a.B * a.NH), (unsigned)((a.Sq + WQ - 1) / WQ));
  if (a.keep < 1.f) hipLaunchKernelGGL((flash_fwd_k<D, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((flash_fwd_k<D, false>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <int D>
static int bwd_d(const FArgs& a, float* dsum, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.NH * a.Sq;
  hipLaunchKernelGGL((flash_dsum_k<D>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, st, a, dsum);
  FArgs b = a;
  b.dsum = dsum;
  dim3 gq((unsigned)(a.B * a.NH), (unsigned)((a.Sq + WQ - 1) / WQ));
  dim3 gk((unsigned)(a.B * a.NH), (unsigned)((a.Sk + WQ - 1) / WQ));
  if (a.keep < 1.f) {
    hipLaunchKernelGGL((flash_dq_k<D, true>), gq, dim3(256), 0, st, b);
    hipLaunchKernelGGL((flash_dkdv_k<D, true>), gk, dim3(256), 0, st, b);
  } else {
    hipLaunchKernelGGL((flash_dq_k<D, false>), gq, dim3(256), 0, st, b);
    hipLaunchKernelGGL((flash_dkdv_k<D, false>), gk, dim3(256), 0, st, b);
  }
  return (int)hipGetLastError();
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
  a.scale = scale; a.keep = keep; a.seed = (uint64_t)seed; a.causal = causal;
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
  a.scale = scale; a.keep = keep; a.seed = (uint64_t)seed; a.causal = causal;
  if (D == 32) return bwd_d<32>(a, dsum, st);
  if (D == 64) return bwd_d<64>(a, dsum, st);
  return bwd_d<128>(a, dsum, st);
}
