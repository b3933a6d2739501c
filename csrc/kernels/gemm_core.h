// bf16 MFMA GEMM and implicit-GEMM convolution for gfx950 (CDNA4).
//
// Replaces the reference's cuBLAS Sgemm / SgemmStridedBatched call sites
// (src/ops/MatrixMult.cu:22-26, BatchMatrixMult.cu:31-36, Linear.cu:50-55,
// Addmm.cu:29, Baddbmm.cu:37) and cuDNN convolution (CudnnConv2d.cu:54-245,
// CudnnConv2dAddBias.cu:93), SURVEY.md §2.7.
//
// One kernel template, operand "loaders" as policies:
//   C[M,N] = alpha * sum_k  Am[m,k] * Bn[n,k]  (+ beta*Cin) (+ bias) -> act
// Each operand is either K-contiguous ("KMAJ", LDS image [rows][64] with a
// 16-byte-chunk XOR swizzle, fragments via ds_read_b128) or MN-contiguous
// (LDS image [64 k][128 rows], 256-byte rows with the T10 XOR, fragments via
// ds_read_b64_tr_b16 -- the hardware transpose read), so all four transpose
// modes and the three conv passes use the same main loop with no transpose
// pass over memory.
//
// Geometry: 128x128x64 block tile, 256 threads = 4 waves (2 M x 2 N), each wave
// 64x64 = 4x4 mfma_f32_16x16x32_bf16 tiles; LDS double buffer (2 x 32 KiB)
// filled by global_load_lds (16 B/lane, swizzle applied on the source address),
// tile k+1 in flight during the MFMAs of tile k, one barrier per K-tile.  Operand roles are swapped (A_op = N side, B_op = M side) so the
// accumulator holds 4 consecutive N columns per lane -> 8/16-byte stores.
// Block ids are remapped so that consecutive tiles share an XCD's L2, then
// grouped 8 tiles along M for operand reuse.  Split-K over gridDim.z with
// fp32 atomics for the long-K weight-gradient GEMMs.
#pragma once
#include "common.h"
#include "lds_tr.h"
#include <algorithm>
#include <type_traits>

namespace hetu {
namespace gemm {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * BK * 2;  // 16 KiB per operand tile

// n / d for 0 <= n < 2^31 by multiply-high (Granlund-Montgomery): the implicit-GEMM
// loaders decompose pixel / tap indices per lane per K-tile, where a hardware-less
// 32-bit integer division would cost ~40 VALU ops each.
struct FastDiv {
  uint32_t d, m, l;
  __host__ __device__ FastDiv() : d(1), m(1), l(0) {}
  __host__ __device__ explicit FastDiv(uint32_t dv) : d(dv < 1 ? 1 : dv) {
    l = 0;
    while (l < 31 && (1u << l) < d) ++l;
    m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> l; }
};

// Default per-block problem view: the whole M x K problem, rows stored linearly.
// Loaders that split the problem into classes over blockIdx.y (strided dgrad)
// override rows_eff / k_eff / out_row.
#define HETU_LINEAR_ROWS                                             \
  __device__ int64_t rows_eff(int64_t M_) const { return M_; }        \
  __device__ int64_t k_eff(int64_t K_) const { return K_; }           \
  __device__ int64_t out_row(int64_t m_) const { return m_; }




// ---- LDS images -------------------------------------------------------------------------
// K-major: [128 rows][64 k] bf16, 128-B rows, chunk c (0..7) of row r at ((c ^ (r&7)) << 4)
__device__ __forceinline__ int offk(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }
// MN-major: [64 k][128 cols] bf16, 256-B rows, chunk c (0..15), T10 image (b)
__device__ __forceinline__ int offmn(int k, int c) {
  return k * 256 + ((c ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4);
}

// Zero chunk that out-of-range / padding lanes stage from (global_load_lds has no
// per-lane predicate: the lane still writes its LDS slot, so it reads zeros).
static __device__ __attribute__((aligned(64))) bf16 g_zero_chunk[32];

__device__ __forceinline__ void glds16(const bf16* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// ASM: the MN-major reads as ds_tr16 (lds_tr.h), which leave an in-flight operand DMA
// alone (the intrinsic makes the compiler wait for it); the caller then calls frag_wait()
// before its MFMAs.  Used by the double-buffered K loops (ST 2 / 3), whose next K-tile is
// in flight while a tile's fragments are read.  The single-stage loop (nothing in flight)
// and the 256x256 kernel keep the intrinsic: their compiler-scheduled partial lgkmcnt
// waits interleave reads and MFMAs, and measured faster that way.

// fragment of 16 rows (row block rb) x 32 k (k-step s): lane holds row (lane&15),
// k = 32s + 8(lane>>4) + j, j = 0..7
template <bool KMAJ, bool ASM = false>
__device__ __forceinline__ v8s lds_frag(const char* lds, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    int r = rb * 16 + (lane & 15);
    int c = s * 4 + (lane >> 4);
    return *reinterpret_cast<const v8s*>(lds + offk(r, c));
  } else {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int c = rb * 2 + (p >> 1);
    int k1 = s * 32 + 8 * g + q;
    const char* a1 = lds + offmn(k1, c) + 8 * (p & 1);
    const char* a2 = lds + offmn(k1 + 4, c) + 8 * (p & 1);
    v4s x, y;
    if constexpr (ASM) {
      x = ds_tr16(a1);
      y = ds_tr16(a2);
    } else {
      x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a1));
      y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a2));
    }
    return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// ---- operand loaders ------------------------------------------------------------------
// The 128x64 tile is staged by 16 global_load_lds instructions (4 per wave), each
// filling 1 KiB of LDS lane-linearly: instruction i of wave w covers LDS bytes
// [4096w + 1024i, +1024).  The swizzle is applied on the SOURCE side: lane l of
// that instruction fetches the logical chunk that belongs at its physical slot.
//   KMAJ: row r = 32w + 8i + (l>>3), physical chunk l&7, logical c = (l&7) ^ (l>>3)
//   MN  : k   = 16w + 4i + (l>>4), physical chunk l&15, logical
//         c = (l&15) ^ (((l>>4)&3)<<2 | i)
// Loaders return, per instruction i, the global address of that chunk (or the
// zero chunk).

__device__ __forceinline__ const bf16* zchunk() { return g_zero_chunk; }

// Which slot of the staged tile load i of wave w, lane l fills.  `map`:
//  0  128x128 kernel (4 waves): one 128-row image per operand, 4 loads per wave.
//  1  256x256 kernel, A operand (2 wave rows x 128 rows, sub-tiles of 64 rows)
//  2  256x256 kernel, B operand (4 wave columns x 64, sub-tiles of 32)
//  For 1/2 each operand is staged as two 128-row "half-tile" images (2 loads per wave
//  each); half h holds the rows every wave reads in ITS h-th sub-tile, so a half can be
//  restaged as soon as the phase that reads it has passed (gemm_big_kernel).
__device__ __forceinline__ int half_to_rel(int map, int h, int x) {
  return map == 1 ? (x >> 6) * 128 + h * 64 + (x & 63) : (x >> 5) * 64 + h * 32 + (x & 31);
}
// K-major: returns the operand row (relative to the tile) of the lane's 16-B chunk.
__device__ __forceinline__ int kmaj_row(int map, int w, int i, int l) {
  if (map == 0) return 32 * w + 8 * i + (l >> 3);
  if (map == 3) return 64 * w + 8 * i + (l >> 3);   // 256-row image, 4 waves x 8 loads
  return half_to_rel(map, i >> 1, 16 * w + 8 * (i & 1) + (l >> 3));
}
// MN-major: k row of the image and operand column (relative) of the lane's chunk.
__device__ __forceinline__ void mn_slot(int map, int w, int i, int l, int& k, int& col) {
  if (map == 3) {   // two 128-column images [64 k][128], waves 2h, 2h+1 fill half h
    k = 32 * (w & 1) + 4 * i + (l >> 4);
    const int c = (l & 15) ^ (((k & 3) << 2) | ((k >> 2) & 3));
    col = (w >> 1) * 128 + 8 * c;
    return;
  }
  k = map ? 8 * w + 4 * (i & 1) + (l >> 4) : 16 * w + 4 * i + (l >> 4);
  const int c = (l & 15) ^ (((k & 3) << 2) | ((k >> 2) & 3));  // T10 image, logical chunk
  col = map ? half_to_rel(map, i >> 1, 8 * c) : 8 * c;
}

// plain row-major operand with contiguous K: element (r, k) at base[r*ld + k]
struct PlainK {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = true;
  const bf16* base; int64_t ld, rows, K, bstride;
  int64_t roff[4]; bool rok[4]; int ch;
  __device__ void init(int64_t r0, int w, int l, int64_t batch, int big) {
    base += batch * bstride;
    ch = (l & 7) ^ (l >> 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t r = r0 + kmaj_row(big, w, i, l);
      rok[i] = r < rows;
      roff[i] = r * ld;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    int64_t k = k0 + ch * 8;
    return (rok[i] && k < K) ? base + roff[i] + k : zchunk();
  }
};

// plain operand stored [K][rows]: element (r, k) at base[k*ld + r]
struct PlainMN {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const bf16* base; int64_t ld, rows, K, bstride;
  int64_t col[4]; bool cok[4]; int kk[4];
  __device__ void init(int64_t r0, int w, int l, int64_t batch, int big) {
    base += batch * bstride;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c;
      mn_slot(big, w, i, l, kk[i], c);
      col[i] = r0 + c;
      cok[i] = col[i] < rows;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    int64_t k = k0 + kk[i];
    return (cok[i] && k < K) ? base + k * ld + col[i] : zchunk();
  }
};

// ---- buffer-descriptor loaders (plain GEMM operands) ------------------------------------
// The staging DMA goes through a 128-bit buffer descriptor of the operand slice:
// buffer_load_dwordx4 ... lds with a per-lane 32-bit voffset fixed at init and the
// K-tile advance in the SCALAR soffset, so a K-tile costs no per-lane address
// arithmetic and no 64-bit selects.  Out-of-range rows (and, when K is not a multiple
// of the 64-wide K-tile, out-of-range k in the last tile) point past num_records and
// the hardware range check returns zeros.  Host side guarantees the slice is
// < 2 GiB (hetu_gemm_bf16 falls back to the pointer loaders otherwise).
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

template <bool KF, int NS = 4>
struct BufK {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = true, BUF = true;
  static constexpr int SLOTS = NS;
  const bf16* base; int64_t ld, rows, K, bstride;
  __amdgpu_buffer_rsrc_t rs; uint32_t vo[NS], oob; int ch;
  __device__ void init(int64_t r0, int w, int l, int64_t batch, int big) {
    oob = (uint32_t)(((rows - 1) * ld + K) * 2);
    rs = make_rsrc(base + batch * bstride, oob);
    ch = (l & 7) ^ (l >> 3);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int64_t r = r0 + kmaj_row(big, w, i, l);
      vo[i] = r < rows ? (uint32_t)((r * ld + ch * 8) * 2) : oob;
    }
  }
  __device__ __forceinline__ void dma(int64_t k0, int i, char* dst) const {
    uint32_t v = vo[i];
    if (!KF && k0 + BK > K && k0 + ch * 8 >= K) v = oob;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, v, (uint32_t)(k0 * 2), 0, 0);
  }
};

template <bool KF, int NS = 4>
struct BufMN {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = false, BUF = true;
  static constexpr int SLOTS = NS;
  const bf16* base; int64_t ld, rows, K, bstride;
  __amdgpu_buffer_rsrc_t rs; uint32_t vo[NS], oob; int kk[NS];
  __device__ void init(int64_t r0, int w, int l, int64_t batch, int big) {
    oob = (uint32_t)(((K - 1) * ld + rows) * 2);
    rs = make_rsrc(base + batch * bstride, oob);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      int c;
      mn_slot(big, w, i, l, kk[i], c);
      const int64_t col = r0 + c;
      vo[i] = col < rows ? (uint32_t)((kk[i] * ld + col) * 2) : oob;
    }
  }
  __device__ __forceinline__ void dma(int64_t k0, int i, char* dst) const {
    uint32_t v = vo[i];
    if (!KF && k0 + BK > K && k0 + kk[i] >= K) v = oob;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, v, (uint32_t)(k0 * ld * 2), 0, 0);
  }
};

// one staging DMA of loader slot i: buffer form, or global_load_lds from the
// loader's per-lane pointer (implicit-GEMM convolution loaders)
template <class L, class = void> struct is_buf : std::false_type {};
template <class L> struct is_buf<L, std::void_t<decltype(L::BUF)>> : std::true_type {};

// staging slots per wave a loader carries (the 4-wave 256-row kernel needs 8)
template <class L, class = void> struct slots_of { static constexpr int value = 4; };
template <class L> struct slots_of<L, std::void_t<decltype(L::SLOTS)>> { static constexpr int value = L::SLOTS; };

template <class L>
__device__ __forceinline__ void stage_dma(const L& l, int64_t k0, int i, char* dst) {
  if constexpr (is_buf<L>::value) {
    l.dma(k0, i, dst);
  } else {
    glds16(l.src(k0, i), dst);
  }
}

struct ConvGeom {
  int N, H, W, C, K, KH, KW, sh, sw, ph, pw, OH, OW;  // C = in channels, K = out channels
  FastDiv fOW, fOH, fC, fK, fKW;
  // reduction channels (C forward, K data-gradient) a multiple of the 64-wide
  // K-tile: every K-tile lies inside ONE filter tap, so the tap decomposition is
  // wave-uniform (scalar ALU, once per tile) and each lane only adds offsets
  int ctap;
};

// forward, M side: rows = output pixels, k = (kh, kw, ci), ci fastest
struct ConvFwdA {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = true;
  const bf16* x; ConvGeom g; int64_t Ktot, rows;
  int nb[4]; int ih0[4], iw0[4]; bool rok[4]; int ch;
  int64_t pix[4];  // element offset of (n, ih0, iw0, 0); dereferenced only in bounds
  __device__ void init(int64_t r0, int w, int l, int64_t, int big) {
    ch = (l & 7) ^ (l >> 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t r = r0 + kmaj_row(big, w, i, l);
      rok[i] = r < rows;
      uint32_t rr = rok[i] ? (uint32_t)r : 0;
      uint32_t t = g.fOW.div(rr);
      int ow = (int)(rr - t * g.OW);
      uint32_t n = g.fOH.div(t);
      int oh = (int)(t - n * g.OH);
      nb[i] = (int)n * g.H;
      ih0[i] = oh * g.sh - g.ph;
      iw0[i] = ow * g.sw - g.pw;
      pix[i] = ((int64_t)(nb[i] + ih0[i]) * g.W + iw0[i]) * g.C;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    if (g.ctap) {
      // tap, kh, kw uniform over the tile (k0 is wave-uniform)
      const uint32_t tap = g.fC.div((uint32_t)k0);
      const int ci = (int)((uint32_t)k0 - tap * g.C) + ch * 8;
      const uint32_t kh = g.fKW.div(tap);
      const int kw = (int)(tap - kh * g.KW);
      const int ih = ih0[i] + (int)kh, iw = iw0[i] + kw;
      const bool ok = k0 < Ktot && rok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      return ok ? x + pix[i] + ((int64_t)kh * g.W + kw) * g.C + ci : zchunk();
    }
    uint32_t k = (uint32_t)k0 + ch * 8;
    uint32_t tap = g.fC.div(k);
    int ci = (int)(k - tap * g.C);
    uint32_t kh = g.fKW.div(tap);
    int kw = (int)(tap - kh * g.KW);
    int ih = ih0[i] + (int)kh, iw = iw0[i] + kw;
    bool ok = k < Ktot && rok[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
    return ok ? x + ((int64_t)(nb[i] + ih) * g.W + iw) * g.C + ci : zchunk();
  }
};

// Data gradient, split into sh*sw stride classes over blockIdx.y.  Class (a, b)
// holds the input pixels with ih % sh == a, iw % sw == b; only the taps with
// kh == (a + ph) mod sh (step sh), kw likewise, reach an output pixel, so each
// class is a dense implicit GEMM over exactly its useful taps (no zero-filled
// K-tiles, no divisibility tests).  Stride 1 is the single class (0, 0).
struct DgradClass {
  int a, b, kh0, kw0, nth, ntw, Hc, Wc, cbh, cbw;
  FastDiv fWc, fHc, fntw;
  __device__ void make(const ConvGeom& g, int cls) {
    a = cls / g.sw;
    b = cls - a * g.sw;
    Hc = a < g.H ? (g.H - a + g.sh - 1) / g.sh : 0;
    Wc = b < g.W ? (g.W - b + g.sw - 1) / g.sw : 0;
    kh0 = (a + g.ph) % g.sh;
    kw0 = (b + g.pw) % g.sw;
    nth = kh0 < g.KH ? (g.KH - kh0 + g.sh - 1) / g.sh : 0;
    ntw = kw0 < g.KW ? (g.KW - kw0 + g.sw - 1) / g.sw : 0;
    // (a + ph - kh0) is a multiple of sh: output row of class row i and class tap th
    // is oh = i + cbh - th exactly (no per-lane division by the stride)
    cbh = (a + g.ph) / g.sh;
    cbw = (b + g.pw) / g.sw;
    fWc = FastDiv((uint32_t)Wc);
    fHc = FastDiv((uint32_t)Hc);
    fntw = FastDiv((uint32_t)ntw);
  }
};

// data gradient, M side: rows = class pixels (n, i, j), k = (tap in class, co)
struct ConvDgradA {
  static constexpr bool KMAJ = true;
  const bf16* dy; ConvGeom g;
  DgradClass c;
  int nb[4]; int ii[4], jj[4]; bool rok[4]; int ch;
  int64_t mrows, kdim;
  __device__ int64_t rows_eff(int64_t) const { return mrows; }
  __device__ int64_t k_eff(int64_t) const { return kdim; }
  __device__ int64_t out_row(int64_t m) const {
    uint32_t t = c.fWc.div((uint32_t)m);
    int j = (int)((uint32_t)m - t * c.Wc);
    uint32_t n = c.fHc.div(t);
    int i = (int)(t - n * c.Hc);
    return ((int64_t)n * g.H + c.a + g.sh * i) * g.W + c.b + g.sw * j;
  }
  __device__ void init(int64_t r0, int w, int l, int64_t cls, int big) {
    c.make(g, (int)cls);
    mrows = (int64_t)g.N * c.Hc * c.Wc;
    kdim = (int64_t)c.nth * c.ntw * g.K;
    ch = (l & 7) ^ (l >> 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t r = r0 + kmaj_row(big, w, i, l);
      rok[i] = r < mrows;
      uint32_t rr = rok[i] ? (uint32_t)r : 0;
      uint32_t t = c.fWc.div(rr);
      int j = (int)(rr - t * c.Wc);
      uint32_t n = c.fHc.div(t);
      ii[i] = (int)(t - n * c.Hc) + c.cbh;
      jj[i] = j + c.cbw;
      nb[i] = (int)n * g.OH;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    uint32_t tap, co;
    if (g.ctap) {                     // K % 64 == 0: one tap per K-tile (scalar)
      tap = g.fK.div((uint32_t)k0);
      co = (uint32_t)k0 - tap * g.K + ch * 8;
    } else {
      uint32_t k = (uint32_t)k0 + ch * 8;
      tap = g.fK.div(k);
      co = k - tap * g.K;
    }
    uint32_t th = c.fntw.div(tap);
    int tw = (int)(tap - th * c.ntw);
    int oh = ii[i] - (int)th, ow = jj[i] - tw;
    bool ok = (int64_t)k0 + (g.ctap ? 0 : ch * 8) < kdim && rok[i] && (unsigned)oh < (unsigned)g.OH &&
              (unsigned)ow < (unsigned)g.OW;
    return ok ? dy + ((int64_t)(nb[i] + oh) * g.OW + ow) * g.K + co : zchunk();
  }
};

// data gradient, N side: cols = ci, k rows = (tap in class, co): w[co][kh][kw][ci]
struct ConvDgradB {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const bf16* w; ConvGeom g;
  DgradClass c;
  int64_t kdim;
  int col[4]; bool cok[4]; int kk[4];
  __device__ void init(int64_t r0, int wv, int l, int64_t cls, int big) {
    c.make(g, (int)cls);
    kdim = (int64_t)c.nth * c.ntw * g.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int cc;
      mn_slot(big, wv, i, l, kk[i], cc);
      col[i] = (int)r0 + cc;
      cok[i] = col[i] < g.C;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    uint32_t k = (uint32_t)k0 + kk[i];
    uint32_t tap;
    int co;
    if (g.ctap) {                     // tap uniform over the K-tile
      tap = g.fK.div((uint32_t)k0);
      co = (int)(k - tap * g.K);
    } else {
      tap = g.fK.div(k);
      co = (int)(k - tap * g.K);
    }
    uint32_t th = c.fntw.div(tap);
    int tw = (int)(tap - th * c.ntw);
    int kh = c.kh0 + g.sh * (int)th, kw = c.kw0 + g.sw * tw;
    return (cok[i] && (int64_t)k < kdim)
               ? w + ((int64_t)co * (g.KH * g.KW) + kh * g.KW + kw) * g.C + col[i]
               : zchunk();
  }
};

// weight gradient, N side: cols = (kh, kw, ci), k rows = output pixels
struct ConvWgradB {
  HETU_LINEAR_ROWS
  static constexpr bool KMAJ = false;
  const bf16* x; ConvGeom g; int64_t P;  // P = N*OH*OW
  int kh[4], kw[4], ci[4]; bool cok[4]; int kk[4];
  __device__ void init(int64_t r0, int w, int l, int64_t, int big) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c;
      mn_slot(big, w, i, l, kk[i], c);
      int col = (int)r0 + c;
      cok[i] = col < g.KH * g.KW * g.C;
      int tap = col / g.C;
      ci[i] = col - tap * g.C;
      kh[i] = tap / g.KW;
      kw[i] = tap - kh[i] * g.KW;
    }
  }
  __device__ const bf16* src(int64_t k0, int i) const {
    uint32_t p = (uint32_t)k0 + kk[i];
    uint32_t t = g.fOW.div(p);
    int ow = (int)(p - t * g.OW);
    uint32_t n = g.fOH.div(t);
    int oh = (int)(t - n * g.OH);
    int ih = oh * g.sh - g.ph + kh[i], iw = ow * g.sw - g.pw + kw[i];
    bool ok = cok[i] && (int64_t)p < P && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
    return ok ? x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + ci[i] : zchunk();
  }
};

// ---- epilogue ------------------------------------------------------------------------
struct Epi {
  void* C; const void* Cin; const float* bias;
  int64_t ldc, ldcin, sC, sCin;
  float alpha, beta;
  int act;        // 0 none, 1 relu, 2 gelu(erf)
  int out_f32;    // C dtype
  int cin_f32;    // Cin dtype
  int atomic;     // fp32 atomicAdd into C (split-K / accumulate)
  int bias_on_m;  // bias indexed by m instead of n
  float* slab;    // split-K: fp32 partial tiles, slab z at slab + z*slab_stride (ld = N)
  int64_t slab_stride;
  // per-column sum / sum of squares of the stored outputs (fp32 atomics into
  // colstats[0..N) and colstats[N..2N), pre-zeroed): the BatchNorm statistics of a
  // convolution output, fused into the epilogue that already holds the values
  float* colstats;
  // BatchNorm-backward form of colstats (C is the gradient dy of a BN output, bf16,
  // ldc % 8 == 0): colstats receives sum(dy') and sum(dy' * x), dy' = dy masked by the
  // forward's ReLU keep-bits (bnmask, one byte per 8 channels, null: no ReLU) and x the
  // BN input (bnx, C's layout) -- the BN backward's reduction pass, fused here
  const bf16* bnx;
  const uint8_t* bnmask;
  int bnstore;    // store dy' (dy masked by bnmask) instead of dy: the BN backward and the
                  // residual branch then read the masked gradient as it is
  // Cin on the stride-2 subgrid (cin_h, cin_w = the output's H, W; 0 = off): output row
  // (n, h, w) adds Cin row (n, h/2, w/2) when h and w are even, nothing otherwise -- the
  // gradient of a 1x1 stride-2 downsample convolution joined without scattering it first
  int cin_h, cin_w;
  // colstats replicas ([cs_rep][2N], 0/1 = one): block b adds into replica b % cs_rep -- a
  // few thousand blocks adding into the same 2N addresses serialise on them (the
  // consumer folds the replicas)
  int cs_rep;
  // pre-activation copy (bf16, C's layout; null: none): the epilogue stores the value
  // before the activation here and the activated value in C -- a training GELU layer
  // keeps its pre-activation for the backward without a separate activation pass
  void* C2;
  // dropout after the activation (0 = off): element (m, n) kept with probability drop_keep
  // and scaled by 1 / drop_keep, bits from Philox(drop_seed, (m * N + n) / 4)[(m * N + n) % 4]
  // -- the standalone dropout kernel's counters over the [M, N] output (host: N % 8 == 0)
  float drop_keep;
  uint64_t drop_seed;
  // gradient mask (bf16, C's layout, batch 1; null: none): out = value * gmask_scale where
  // gmask > 0, else 0 -- the backward of ReLU (+ dropout) applied to the data-gradient GEMM
  // that produces its input, from the forward's output alone
  const void* gmask;
  float gmask_scale;
  // gmask_bits: gmask holds keep bits instead (one byte per 8 consecutive elements of C's
  // layout, bit t = element n + t; ldc % 8 == 0) -- 1/16 of the bf16 mask's bytes
  int gmask_bits;
  // keep-bit output of the epilogue dropout (EX bit 1; null: none): the byte for elements
  // n..n+7 of a row gets bit t set where the stored value is positive, in gmask_bits' layout
  // -- the forward writes the mask its backward GEMM reads
  uint8_t* mbits_out;
  // step counter of the graph-safe RNG (common.h rng_seed) for the epilogue dropout
  const uint64_t* drop_off;
};

// column statistics of one epilogue: each thread holds sums of its 8 columns over
// its rows; threads sharing columns are folded by lane shuffles (lanes l ^ 16k within
// a wave), then across waves through LDS, one atomic per column per block.
//   groups: threads per row (16 for the 128-wide tile, 32 for the 256-wide tile)
template <int GROUPS, int NWAVES>
__device__ __forceinline__ void epilogue_colstats(float (&cs)[8], float (&cq)[8], float* lds, int tid,
                                                  int64_t n0, int64_t N, float* colstats) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int o = GROUPS; o < 64; o <<= 1) {
      cs[t] += __shfl_xor(cs[t], o, 64);
      cq[t] += __shfl_xor(cq[t], o, 64);
    }
  }
  __syncthreads();   // the staging area is free again
  if (lane < GROUPS) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      lds[(wave * GROUPS + lane) * 8 + t] = cs[t];
      lds[NWAVES * GROUPS * 8 + (wave * GROUPS + lane) * 8 + t] = cq[t];
    }
  }
  __syncthreads();
  if (tid < GROUPS * 8) {
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) {
      S += lds[w * GROUPS * 8 + tid];
      Q += lds[NWAVES * GROUPS * 8 + w * GROUPS * 8 + tid];
    }
    const int64_t n = n0 + tid;
    if (n < N) {
      unsafeAtomicAdd(colstats + n, S);
      unsafeAtomicAdd(colstats + N + n, Q);
    }
  }
}

// erf to 1.5e-7 absolute (Abramowitz & Stegun 7.1.26): one v_exp + one v_rcp and a
// 5-term polynomial instead of erff's two-branch rational form -- the GELU epilogue
// costs ~1/3 of the VALU, far below bf16 resolution
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t +
                   0.254829592f) * t;
  return copysignf(1.f - p * __expf(-ax * ax), x);
}

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return 0.5f * v * (1.f + erf_fast(v * 0.70710678118f));
  return v;
}

// Row-coalesced epilogue of one thread: 8 consecutive columns n..n+7 of row m.
// The bias columns are loaded once per thread (bcol; the column set of a thread is
// fixed over all its rows) -- per-element bias loads behind the C stores (possible
// aliasing) serialised the epilogue.
struct EpiOut {
  char* Cb;
  char* C2b;
  const char* Cinb;
  bool cvec, ivec;
  bool cvec2;   // bf16 C with an even (not 8-multiple) ldc: 4-byte stores of column pairs
  float bcol[8];
};

__device__ __forceinline__ void epi_init(const Epi& ep, EpiOut& o, int64_t batch, int64_t n, int64_t N) {
  o.Cb = (char*)ep.C + batch * ep.sC * (ep.out_f32 ? 4 : 2);
  o.C2b = ep.C2 ? (char*)ep.C2 + batch * ep.sC * 2 : nullptr;
  o.Cinb = ep.Cin ? (const char*)ep.Cin + batch * ep.sCin * (ep.cin_f32 ? 4 : 2) : nullptr;
  o.cvec = ep.out_f32 ? ((ep.ldc & 3) == 0 && ((uintptr_t)o.Cb & 15) == 0)
                      : ((ep.ldc & 7) == 0 && ((uintptr_t)o.Cb & 15) == 0);
  o.cvec2 = !ep.out_f32 && !o.cvec && (ep.ldc & 1) == 0 && ((uintptr_t)o.Cb & 3) == 0;
  o.ivec = o.Cinb && (ep.cin_f32 ? ((ep.ldcin & 3) == 0 && ((uintptr_t)o.Cinb & 15) == 0)
                                 : ((ep.ldcin & 7) == 0 && ((uintptr_t)o.Cinb & 15) == 0));
#pragma unroll
  for (int t = 0; t < 8; ++t) o.bcol[t] = 0.f;
  if (ep.bias && !ep.bias_on_m) {
    if (n + 7 < N && ((uintptr_t)(ep.bias + n) & 15) == 0) {
      const float4 b0 = *reinterpret_cast<const float4*>(ep.bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(ep.bias + n + 4);
      o.bcol[0] = b0.x; o.bcol[1] = b0.y; o.bcol[2] = b0.z; o.bcol[3] = b0.w;
      o.bcol[4] = b1.x; o.bcol[5] = b1.y; o.bcol[6] = b1.z; o.bcol[7] = b1.w;
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) o.bcol[t] = n + t < N ? ep.bias[n + t] : 0.f;
    }
  }
}

// EX: bit 0 compiles in the pre-activation copy (Epi::C2), bit 1 the epilogue dropout,
// bit 2 the gradient mask (Epi::gmask)
// (plain GEMM loaders only: they cost registers every other epilogue would carry; one
// feature per build -- with both, the 4-blocks-per-CU tile ran out of scalar registers
// and spilled in the epilogue).
// BNX: the BatchNorm-backward / subgrid-Cin extensions (Epi::bnx, bnmask, bnstore, cin_w)
// are compiled in; the plain epilogue (forward convolutions, GEMMs) keeps its register
// budget -- the 4-blocks-per-CU tile has 128 registers and spilled with them inlined
template <bool BNX = true, int EX = 0>
__device__ __forceinline__ void epi_row8(const Epi& ep, const EpiOut& o, float (&v)[8], int64_t m, int64_t n,
                                         int64_t N, int64_t orow, float (&cs)[8], float (&cq)[8],
                                         bool has_pre = false, uint4 pre = uint4{}, bool has_gm = false,
                                         uint4 gmv = uint4{}) {
  // pre: this row piece of Cin, already loaded (by value: a selected pointer into the
  // caller's prefetch array would keep that array in scratch memory)
  const bool full = n + 7 < N;
  if (ep.bias) {
    const float bm = ep.bias_on_m ? ep.bias[m] : 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] += ep.bias_on_m ? bm : o.bcol[t];
  }
  // BN-backward operands of this row piece (x and the ReLU keep-bits): requested first, so
  // they are in flight together with the Cin load below instead of one round trip each
  // after the store
  const int64_t off = orow * ep.ldc + n;
  const bool bnv = BNX && ep.colstats && ep.bnx;
  uint4 bxr = make_uint4(0, 0, 0, 0);
  if (bnv && o.cvec && full) bxr = *reinterpret_cast<const uint4*>(ep.bnx + off);
  const unsigned bnmk = (bnv && ep.bnmask) ? (unsigned)ep.bnmask[off >> 3] : 0xffu;
  int64_t crow = orow;
  if (BNX && o.Cinb && ep.cin_w) {   // stride-2 subgrid Cin: even (h, w) only
    const uint32_t hw = (uint32_t)(ep.cin_h * ep.cin_w), o32 = (uint32_t)orow;   // rows < 2^31 (host check)
    const uint32_t img = o32 / hw, r = o32 - img * hw;
    const uint32_t h = r / (uint32_t)ep.cin_w, w = r - h * (uint32_t)ep.cin_w;
    crow = ((h | w) & 1u) ? -1 : ((int64_t)img * (ep.cin_h >> 1) + (h >> 1)) * (ep.cin_w >> 1) + (w >> 1);
  }
  if (o.Cinb && crow >= 0) {
    const int64_t coff = crow * ep.ldcin + n;
    float cv[8];
    if (has_pre && o.ivec && full && !ep.cin_f32) {
      const uint32_t w[4] = {pre.x, pre.y, pre.z, pre.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        cv[2 * t] = bf16_bits_to_f((unsigned short)(w[t] & 0xffffu));
        cv[2 * t + 1] = bf16_bits_to_f((unsigned short)(w[t] >> 16));
      }
    } else if (o.ivec && full) {
      if (ep.cin_f32) {
        float4 c0 = *reinterpret_cast<const float4*>((const float*)o.Cinb + coff);
        float4 c1 = *reinterpret_cast<const float4*>((const float*)o.Cinb + coff + 4);
        cv[0] = c0.x; cv[1] = c0.y; cv[2] = c0.z; cv[3] = c0.w;
        cv[4] = c1.x; cv[5] = c1.y; cv[6] = c1.z; cv[7] = c1.w;
      } else {
        load_vec<bf16>((const bf16*)o.Cinb + coff, cv);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        cv[t] = n + t < N ? (ep.cin_f32 ? ((const float*)o.Cinb)[coff + t] : to_f(((const bf16*)o.Cinb)[coff + t]))
                          : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] += ep.beta * cv[t];
  }
  if ((EX & 4) && ep.gmask && ep.gmask_bits) {   // the same from the forward's keep bits
    const unsigned kb = has_gm ? gmv.x : (unsigned)((const uint8_t*)ep.gmask)[off >> 3];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = (kb >> t) & 1u ? v[t] * ep.gmask_scale : 0.f;
  } else if ((EX & 4) && ep.gmask) {   // ReLU / dropout backward: keep where the forward output is positive
    const bf16* G = (const bf16*)ep.gmask + off;
    float gv[8];
    if (has_gm && full) {   // prefetched by the caller (this row piece, C's alignment)
      const uint32_t w[4] = {gmv.x, gmv.y, gmv.z, gmv.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        gv[2 * t] = bf16_bits_to_f((unsigned short)(w[t] & 0xffffu));
        gv[2 * t + 1] = bf16_bits_to_f((unsigned short)(w[t] >> 16));
      }
    } else if (o.cvec && full) {
      load_vec<bf16>(G, gv);
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) gv[t] = n + t < N ? to_f(G[t]) : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = gv[t] > 0.f ? v[t] * ep.gmask_scale : 0.f;
  }
  if ((EX & 1) && o.C2b) {   // the pre-activation, bf16 in C's layout
    bf16* P = (bf16*)o.C2b + off;
    if (o.cvec && full) {
      store_vec<bf16>(P, v);
    } else {
      for (int t = 0; t < 8; ++t)
        if (n + t < N) ((unsigned short*)P)[t] = f_to_bf16_bits(v[t]);
    }
  }
  if (ep.act) {
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = act_f(v[t], ep.act);
  }
  if (BNX && ep.bnstore) {
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = (bnmk >> t) & 1u ? v[t] : 0.f;
  }
  if ((EX & 2) && ep.drop_keep > 0.f) {
    const uint64_t ctr = ((uint64_t)m * (uint64_t)N + (uint64_t)n) >> 2;
    const uint64_t sd = rng_seed(ep.drop_seed, ep.drop_off);
    const uint4 r0 = Philox::gen(sd, ctr);
    const uint4 r1 = Philox::gen(sd, ctr + 1);
    const uint32_t q[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    const float inv = 1.f / ep.drop_keep;
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = Philox::u01(q[t]) < ep.drop_keep ? v[t] * inv : 0.f;
    if (ep.mbits_out) {
      unsigned kb = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) kb |= (v[t] > 0.f ? 1u : 0u) << t;
      ep.mbits_out[off >> 3] = (uint8_t)kb;
    }
  }
  if (ep.out_f32) {
    float* Cf = (float*)o.Cb + off;
    if (o.cvec && full) {
      *reinterpret_cast<float4*>(Cf) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(Cf + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int t = 0; t < 8; ++t)
        if (n + t < N) Cf[t] = v[t];
    }
  } else {
    bf16* Ch = (bf16*)o.Cb + off;
    if (o.cvec && full) {
      store_vec<bf16>(Ch, v);
    } else if (o.cvec2 && full) {   // row offset and n even: 4-byte aligned pairs (the 30522-wide MLM head)
      uint32_t* C2 = reinterpret_cast<uint32_t*>(Ch);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        C2[t] = (uint32_t)f_to_bf16_bits(v[2 * t]) | ((uint32_t)f_to_bf16_bits(v[2 * t + 1]) << 16);
    } else {
      for (int t = 0; t < 8; ++t)
        if (n + t < N) ((unsigned short*)Ch)[t] = f_to_bf16_bits(v[t]);
    }
  }
  if (bnv) {   // BN backward sums of the stored dy
    float xv[8];
    if (o.cvec && full) {
      const uint32_t xw[4] = {bxr.x, bxr.y, bxr.z, bxr.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xv[2 * t] = bf16_bits_to_f((unsigned short)(xw[t] & 0xffffu));
        xv[2 * t + 1] = bf16_bits_to_f((unsigned short)(xw[t] >> 16));
      }
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) xv[t] = n + t < N ? to_f(ep.bnx[off + t]) : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float g = (bnmk >> t) & 1u ? bf16_bits_to_f(f_to_bf16_bits(v[t])) : 0.f;
      cs[t] += g;
      cq[t] += g * xv[t];
    }
  } else if (ep.colstats) {   // statistics of the values as stored
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float sv = ep.out_f32 ? v[t] : bf16_bits_to_f(f_to_bf16_bits(v[t]));
      cs[t] += sv;
      cq[t] += sv * sv;
    }
  }
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ST: LDS stages.  1: one 32 KiB buffer when every block owns a single K-tile (short-K
// 1x1 convolutions: more resident blocks per CU); 2: double buffer, vmcnt(0) +
// barrier per K-tile (2 blocks per CU); 3: the same two buffers restaged two K-tiles
// ahead (fragments read to registers before the restage; counted vmcnt).  (A 3-stage variant at 1 block per CU measured
// 0.5-0.8x of ST 2 on every bench_tiles shape: occupancy, not prefetch depth, hides the
// DMA latency here.)
// WN: 16-column MFMA blocks per wave along N.  4: 128x128 tile (waves 64x64);
// 2: 128x64 tile (waves 64x32) for the 64-channel convolutions, where half of a 128-wide
// tile's MFMAs would multiply zero columns.  The B image keeps its 128-row staging map
// (rows past the tile are in-range neighbours or range-checked zeros, never read).
// ST == 1 is also the high-occupancy form for short-K, memory-bound shapes (1x1 convolutions,
// their gradient joins): one 32 KiB LDS buffer restaged per K-tile behind a barrier and at most
// 128 VGPRs, so 4 blocks share a CU and hide each other's DMA / epilogue latency.
// HETU_BNX_PRE1 (build flag, default on): the single-stage BN-backward tile also prefetches
// its gradient-join rows before the epilogue staging, at 3 blocks per CU -- ResNet-50
// 10 898 / 10 859 vs 10 808 / 10 812 img/s interleaved (profiles/bnx_prefetch_ab_r6.txt)
#ifndef HETU_BNX_PRE1
#define HETU_BNX_PRE1 1
#endif
template <class LA, class LB, int ST, int WN = 4, bool BNX = false, int EX = 0>
__global__ __launch_bounds__(NT, (ST == 1 && !BNX ? 4 : (ST == 1 && HETU_BNX_PRE1 ? 3 : 2))) void gemm_kernel(LA la, LB lb, Epi ep, int64_t M, int64_t N,
                                                                     int64_t K, int tiles_m, int tiles_n, int ktps) {
  constexpr bool DB = ST >= 2;
  constexpr int TBN = 32 * WN;                 // block tile columns
  constexpr int TPR = TBN / 8;                 // epilogue threads per row (8 columns each)
  constexpr int RPP = NT / TPR;                // epilogue rows per pass (21 for the 96-wide tile)
  constexpr int NPASS = (64 + RPP - 1) / RPP;  // passes per 64-row half
  __shared__ __attribute__((aligned(16))) char smem_raw[DB ? 4 * TILE_BYTES : 64 * (BN + 4) * 4];
  constexpr int buf_stride = DB ? 2 * TILE_BYTES : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  // XCD-aware bijective remap, then group-of-8 along M for L2 reuse
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int gid = wg / per_group, first_m = gid * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  const int64_t batch = blockIdx.y;
  la.init((int64_t)tm * BM, wave, lane, batch, 0);
  lb.init((int64_t)tn * TBN, wave, lane, batch, 0);
  // per-block problem view (a stride class of a strided dgrad may be smaller)
  const int64_t Mb = la.rows_eff(M);
  if ((int64_t)tm * BM >= Mb) return;  // block-uniform, before any barrier
  K = la.k_eff(K);

  const int nkt = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.z * ktps;
  const int kt1 = min(kt0 + ktps, nkt);

  const int ec = (tid % TPR) * 8;
  const bool erow = tid < RPP * TPR;           // threads past the last full row pass idle
  EpiOut eo;
  epi_init(ep, eo, batch, (int64_t)tn * TBN + ec, N);   // bias columns in flight during the K loop

  v4f acc[4][WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // stage K-tile kt into LDS buffer b: 4 + 4 global_load_lds per wave
  auto stage = [&](int kt, int b) {
    char* As = smem_raw + b * buf_stride + 4096 * wave;
    char* Bs = As + TILE_BYTES;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) stage_dma(la, k0, i, As + 1024 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) stage_dma(lb, k0, i, Bs + 1024 * i);
  };

  if constexpr (ST == 3) {
    // Two K-tiles ahead in the same two buffers: a K-tile's fragments (both k-steps) are
    // read into registers first, and once every wave has read them the buffer is restaged
    // with K-tile kt+2 BEFORE this tile's MFMAs -- the DMA has two tiles of MFMA time to
    // land instead of one, at the same LDS footprint and 2 blocks per CU.  The waits are
    // counted (vmcnt 8 = the younger tile's 8 DMAs stay in flight) and the barriers raw:
    // __syncthreads() would drain the prefetch.
    if (kt0 < kt1) stage(kt0, 0);
    if (kt0 + 1 < kt1) {
      stage(kt0 + 1, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const char* As = smem_raw + cur * buf_stride;
      const char* Bs = As + TILE_BYTES;
      v8s mf[2][4], nf[2][WN];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) mf[s][i] = lds_frag<LA::KMAJ, true>(As, wm * 4 + i, s, lane);
#pragma unroll
        for (int j = 0; j < WN; ++j) nf[s][j] = lds_frag<LB::KMAJ, true>(Bs, wn * WN + j, s, lane);
      }
      frag_wait();
      lds_barrier();
      const bool more = kt + 2 < kt1;
      if (more) stage(kt + 2, cur);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nf[s][j], mf[s][i], acc[i][j], 0, 0, 0);
      if (kt + 1 < kt1) {
        if (more) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
  if (kt0 < kt1) stage(kt0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = DB ? (kt - kt0) & 1 : 0;
    if (DB && kt + 1 < kt1) stage(kt + 1, cur ^ 1);  // in flight during this tile's MFMAs
    const char* As = smem_raw + cur * buf_stride;
    const char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v8s mf[4], nf[WN];
#pragma unroll
      for (int i = 0; i < 4; ++i) mf[i] = lds_frag<LA::KMAJ, DB>(As, wm * 4 + i, s, lane);
#pragma unroll
      for (int j = 0; j < WN; ++j) nf[j] = lds_frag<LB::KMAJ, DB>(Bs, wn * WN + j, s, lane);
      if constexpr (DB) frag_wait();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nf[j], mf[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!DB && kt + 1 < kt1) {   // single buffer: restage once every wave has read it
      stage(kt + 1, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  }

  // bf16 Cin (residual / gradient join, beta): this thread's Cin row pieces of the first
  // 64-row half are requested at once before the LDS staging of the epilogue -- one memory
  // latency instead of one per 16-row pass (the short-K 1x1 data-gradient joins were all
  // epilogue latency) -- and each second-half piece is requested as soon as its first-half
  // register is consumed: 16 registers instead of 32, so the 4-blocks-per-CU tile does not
  // spill them.  Issuing them before the K loop instead measured slower: they queue ahead
  // of the operand DMA that the first K-tile waits for.
  // (not in the single-stage 4-blocks-per-CU build: at 128 registers the prefetch spills,
  // and its neighbours on the CU hide the epilogue latency instead)
  uint4 cpre[NPASS];
  const bool use_pre = (ST == 2 || (HETU_BNX_PRE1 && ST == 1 && BNX)) && eo.Cinb && !ep.cin_f32 && !ep.atomic && !ep.slab && eo.ivec && !(BNX && ep.cin_w);
  const int64_t pre_n = (int64_t)tn * TBN + ec;
  auto pre_load = [&](int h, int pss) {
    const int rr = pss * RPP + tid / TPR;
    const int64_t m = (int64_t)tm * BM + h * 64 + rr;
    cpre[pss] = (erow && rr < 64 && m < Mb && pre_n + 7 < N)
                    ? *reinterpret_cast<const uint4*>((const bf16*)eo.Cinb + la.out_row(m) * ep.ldcin + pre_n)
                    : make_uint4(0, 0, 0, 0);
  };
  if (use_pre) {
#pragma unroll
    for (int pss = 0; pss < NPASS; ++pss) pre_load(0, pss);
  }
  // keep bits of the gradient mask (Epi::gmask_bits): all of this thread's row pieces,
  // one byte each, requested together before the staging (NPASS <= 4: one word per half)
  uint32_t gbw[2] = {0u, 0u};
  const bool use_gb = (EX & 4) && ep.gmask && ep.gmask_bits;
  if constexpr ((EX & 4) != 0) {
    if (use_gb) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int pss = 0; pss < NPASS; ++pss) {
          const int rr = pss * RPP + tid / TPR;
          const int64_t m = (int64_t)tm * BM + h * 64 + rr;
          const uint32_t b = (erow && rr < 64 && m < Mb && pre_n < N)
                                 ? (uint32_t)((const uint8_t*)ep.gmask)[(la.out_row(m) * ep.ldc + pre_n) >> 3]
                                 : 0u;
          gbw[h] |= b << (8 * pss);
        }
    }
  }

  // epilogue: lane holds C[m][n..n+3]
  if (ep.slab) {  // split-K partial: plain fp32 stores into this slice's slab
    float* S = ep.slab + blockIdx.z * ep.slab_stride;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = (int64_t)tm * BM + wm * 64 + i * 16 + (lane & 15);
      if (m >= Mb) continue;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int64_t n = (int64_t)tn * TBN + wn * 16 * WN + j * 16 + 4 * (lane >> 4);
        if (n >= N) continue;
        float* d = S + m * N + n;
        if (n + 3 < N && (N & 3) == 0) {
          *reinterpret_cast<float4*>(d) =
              make_float4(acc[i][j][0] * ep.alpha, acc[i][j][1] * ep.alpha, acc[i][j][2] * ep.alpha,
                          acc[i][j][3] * ep.alpha);
        } else {
          for (int t = 0; t < 4; ++t)
            if (n + t < N) d[t] = acc[i][j][t] * ep.alpha;
        }
      }
    }
    return;
  }
  if (!ep.atomic) {
    float cs[8], cq[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { cs[t] = 0.f; cq[t] = 0.f; }
    // Row-coalesced epilogue: the tile goes through LDS in two 64-row halves
    // (fp32, rows padded by 4 floats so the 16-row MFMA write pattern spreads
    // over the banks), then TPR lanes cover one row with 8 elements each: full
    // bf16 rows per instruction instead of scattered 32-byte pieces, and the same
    // for the Cin (residual / beta) read.
    constexpr int SROW = TBN + 4;
    float* stg = reinterpret_cast<float*>(smem_raw);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (wm == half) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            const int rr = i * 16 + (lane & 15), cc = wn * 16 * WN + j * 16 + 4 * (lane >> 4);
            *reinterpret_cast<v4f*>(stg + rr * SROW + cc) = acc[i][j];
          }
      }
      __syncthreads();
#pragma unroll
      for (int pss = 0; pss < NPASS; ++pss) {
        const int rr = pss * RPP + tid / TPR;
        const int64_t m = (int64_t)tm * BM + half * 64 + rr;
        const int64_t n = (int64_t)tn * TBN + ec;
        if (erow && rr < 64 && m < Mb && n < N) {
          float v[8];
          v4f a0 = *reinterpret_cast<const v4f*>(stg + rr * SROW + ec);
          v4f a1 = *reinterpret_cast<const v4f*>(stg + rr * SROW + ec + 4);
#pragma unroll
          for (int t = 0; t < 4; ++t) { v[t] = a0[t] * ep.alpha; v[4 + t] = a1[t] * ep.alpha; }
          if constexpr ((EX & 4) != 0)
            epi_row8<BNX, EX>(ep, eo, v, m, n, N, la.out_row(m), cs, cq, use_pre, cpre[pss], use_gb,
                              make_uint4((gbw[half] >> (8 * pss)) & 0xffu, 0u, 0u, 0u));
          else
            epi_row8<BNX, EX>(ep, eo, v, m, n, N, la.out_row(m), cs, cq, use_pre, cpre[pss]);
        }
        if (use_pre && half == 0) pre_load(1, pss);
      }
      __syncthreads();
    }
    if (ep.colstats)
      epilogue_colstats<TPR, 4>(cs, cq, stg, tid, (int64_t)tn * TBN, N,
                                ep.colstats + (ep.cs_rep > 1 ? (int64_t)(blockIdx.x % ep.cs_rep) * 2 * N : 0));
    return;
  }
  // fp32 atomic accumulation (split-K without a slab / accumulate into C)
  float* Cf = (float*)((char*)ep.C + batch * ep.sC * 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = (int64_t)tm * BM + wm * 64 + i * 16 + (lane & 15);
    if (m >= Mb) continue;
    const int64_t orow = la.out_row(m);
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int64_t n = (int64_t)tn * TBN + wn * 16 * WN + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      const int64_t o = orow * ep.ldc + n;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (n + t >= N) continue;
        float x = acc[i][j][t] * ep.alpha;
        if (ep.bias && blockIdx.z == 0) x += ep.bias_on_m ? ep.bias[m] : ep.bias[n + t];
        unsafeAtomicAdd(Cf + o + t, x);
      }
    }
  }
}

// ---- 256x256 tile, 8 waves, phase-interleaved K loop -----------------------------------
// Block tile 256x256x64, 512 threads = 8 waves as 2 (M) x 4 (N); wave tile 128x64 =
// 8 x 4 mfma_f32_16x16x32_bf16 tiles (128 fp32 accumulators per lane).  LDS = 2 K-tile
// buffers x 4 half-tile images of 16 KiB (A rows / B columns each wave reads in its
// sub-tile 0 or 1; kmaj_row / mn_slot) = 128 KiB, one block per CU, 2 waves per SIMD.
// Every K-tile runs as 4 phases; each phase reads one register sub-tile from LDS,
// stages ONE half-tile (2 global_load_lds per thread) 7 half-tiles ahead, and runs the
// 16 MFMAs of one 64x32 quadrant of the wave tile between two raw s_barriers.  The DMA
// stays in flight across the barriers (counted vmcnt, never 0 in the loop): the
// buffer for K-tile t+1 is retired by the wait in the last phase of K-tile t.
//   phase 0: read A-sub0 + B-sub0, MMA (A0,B0)     restage (K-tile t+2, same buffer):
//   phase 1: read B-sub1,          MMA (A0,B1)       A-half0 in phase 1, B-half1 in 2,
//   phase 2: read A-sub1,          MMA (A1,B1)       A-half1 in 3, B-half0 in phase 0
//   phase 3: read B-sub0,          MMA (A1,B0)       of t+1: one phase after last read
constexpr int BIG = 256, BIG_NT = 512;
constexpr int HALF_BYTES = 128 * BK * 2;       // 16 KiB
constexpr int BUF_BYTES = 4 * HALF_BYTES;       // A-h0, A-h1, B-h0, B-h1

__device__ __forceinline__ void vm_wait_halves(int n) {
  // wait until at most n half-tiles (2 DMA each) of this wave are still in flight
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}


template <class LA, class LB, int EX = 0>
__global__ __launch_bounds__(BIG_NT, 1) void gemm_big_kernel(LA la, LB lb, Epi ep, int64_t M, int64_t N,
                                                             int64_t K, int tiles_m, int tiles_n, int ktps) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int gid = wg / per_group, first_m = gid * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  const int64_t batch = blockIdx.y;
  la.init((int64_t)tm * BIG, wave, lane, batch, 1);
  lb.init((int64_t)tn * BIG, wave, lane, batch, 2);
  const int64_t Mb = la.rows_eff(M);
  if ((int64_t)tm * BIG >= Mb) return;  // block-uniform, before any barrier
  K = la.k_eff(K);
  const int nkt = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.z * ktps;
  const int nk = max(0, min(kt0 + ktps, nkt) - kt0);
  const int nh = 4 * nk;                 // half-tiles to stage

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // half-tile j: K-tile j>>2, staging order A-h0, B-h1, A-h1, B-h0 (the order the
  // phases of the previous use of the buffer finish reading them, see below)
  auto issue = [&](int j) {
    if (j >= nh) return;
    const int t = j >> 2, which = j & 3;
    const int64_t k0 = (int64_t)(kt0 + t) * BK;
    char* buf = smem + (t & 1) * BUF_BYTES;
    const bool isA = (which & 1) == 0;
    const int h = isA ? (which >> 1) : (which == 1 ? 1 : 0);
    char* dst = buf + (isA ? 0 : 2 * HALF_BYTES) + h * HALF_BYTES + 2048 * wave;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      if (isA) stage_dma(la, k0, 2 * h + ii, dst + 1024 * ii);
      else stage_dma(lb, k0, 2 * h + ii, dst + 1024 * ii);
    }
  };
  // half-tiles issued after the last half of K-tile t (at most 3 in flight)
  auto younger_than_tile = [&](int t, int issued) { return max(0, min(3, issued - 4 * (t + 1))); };

#pragma clang loop unroll(full)
  for (int j = 0; j < 7; ++j) issue(j);   // unrolled: loader arrays stay in registers
  int issued = min(7, nh);
  vm_wait_halves(younger_than_tile(0, issued));
  raw_barrier();
  // Ping-pong: the wave-row-1 group runs one barrier behind the wave-row-0 group, so on
  // every SIMD (one wave of each group) one wave's 16 MFMAs overlap the other wave's
  // LDS reads / DMA issue / waits.  Each phase ends its reads with lgkmcnt(0) BEFORE its
  // first barrier, so a half is restaged one phase after the phase that last read it.
  if (wr == 1) raw_barrier();

  v8s fa[2][4][2], fb[2][2][2];   // [sub][row/col block][k-step]
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF_BYTES;
    const char* Ah[2] = {buf, buf + HALF_BYTES};
    const char* Bh[2] = {buf + 2 * HALF_BYTES, buf + 3 * HALF_BYTES};
#pragma clang loop unroll(full)
    for (int p = 0; p < 4; ++p) {
      // phase p reads: 0: B-sub0 + A-sub0, 1: B-sub1, 2: A-sub1, 3: nothing
      if (p == 0) {   // B-sub0 stays in registers through phase 3
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) fb[0][jj][s2] = lds_frag<LB::KMAJ>(Bh[0], wc * 2 + jj, s2, lane);
      }
      if (p == 0) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) fa[0][ii][s2] = lds_frag<LA::KMAJ>(Ah[0], wr * 4 + ii, s2, lane);
      } else if (p == 1) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) fb[1][jj][s2] = lds_frag<LB::KMAJ>(Bh[1], wc * 2 + jj, s2, lane);
      } else if (p == 2) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) fa[1][ii][s2] = lds_frag<LA::KMAJ>(Ah[1], wr * 4 + ii, s2, lane);
      }
      issue(4 * t + p + 7);
      if (p == 3) {
        issued = min(4 * t + 11, nh);
        vm_wait_halves(younger_than_tile(t + 1, issued));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
      const int sa = (p < 2) ? 0 : 1;
      const int sb = (p == 0 || p == 3) ? 0 : 1;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            acc[sa * 4 + ii][sb * 2 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fb[sb][jj][s2], fa[sa][ii][s2], acc[sa * 4 + ii][sb * 2 + jj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      raw_barrier();
    }
  }
  if (wr == 0) raw_barrier();   // re-align the two groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: lane holds C[m][n..n+3] of acc[i][j],
  //   m = tm*256 + wr*128 + 16i + (lane&15), n = tn*256 + wc*64 + 16j + 4(lane>>4)
  if (ep.slab || ep.atomic) {
    float* S = ep.slab ? ep.slab + blockIdx.z * ep.slab_stride : nullptr;
    char* Cb = (char*)ep.C + batch * ep.sC * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t m = (int64_t)tm * BIG + wr * 128 + i * 16 + (lane & 15);
      if (m >= Mb) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = (int64_t)tn * BIG + wc * 64 + j * 16 + 4 * (lane >> 4);
        if (n >= N) continue;
        if (S) {
          float* d = S + m * N + n;
          if (n + 3 < N && (N & 3) == 0) {
            *reinterpret_cast<float4*>(d) = make_float4(acc[i][j][0] * ep.alpha, acc[i][j][1] * ep.alpha,
                                                        acc[i][j][2] * ep.alpha, acc[i][j][3] * ep.alpha);
          } else {
            for (int t = 0; t < 4; ++t)
              if (n + t < N) d[t] = acc[i][j][t] * ep.alpha;
          }
        } else {
          float* Cf = (float*)Cb + la.out_row(m) * ep.ldc + n;
          for (int t = 0; t < 4; ++t)
            if (n + t < N) unsafeAtomicAdd(Cf + t, acc[i][j][t] * ep.alpha);
        }
      }
    }
    return;
  }
  constexpr int SROW = BIG + 4;
  float* stg = reinterpret_cast<float*>(smem);
  float cs[8], cq[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) { cs[t] = 0.f; cq[t] = 0.f; }
  const int c = (tid & 31) * 8;
  EpiOut eo;
  epi_init(ep, eo, batch, (int64_t)tn * BIG + c, N);
  // 4 passes of 64 rows through LDS (64 x 260 fp32 = 66.5 KiB), full-row stores
  // gradient-mask build: a pass's 4 mask row pieces are requested before its LDS staging,
  // one memory latency per pass instead of one per row piece
  const bool use_gm = (EX & 4) && ep.gmask && eo.cvec;
  uint4 gpre[4];
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    if constexpr ((EX & 4) != 0) {
      if (use_gm) {
#pragma unroll
        for (int sp = 0; sp < 4; ++sp) {
          const int64_t m = (int64_t)tm * BIG + pass * 64 + sp * 16 + (tid >> 5);
          const int64_t n = (int64_t)tn * BIG + c;
          if (ep.gmask_bits)
            gpre[sp] = make_uint4(m < Mb && n < N ? ((const uint8_t*)ep.gmask)[(la.out_row(m) * ep.ldc + n) >> 3] : 0u,
                                  0u, 0u, 0u);
          else
            gpre[sp] = (m < Mb && n + 7 < N)
                           ? *reinterpret_cast<const uint4*>((const bf16*)ep.gmask + la.out_row(m) * ep.ldc + n)
                           : make_uint4(0, 0, 0, 0);
        }
      }
    }
    if (wr == (pass >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = (pass & 1) * 4 + ii;
          const int rr = ii * 16 + (lane & 15), cc = wc * 64 + j * 16 + 4 * (lane >> 4);
          *reinterpret_cast<v4f*>(stg + rr * SROW + cc) = acc[i][j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int sp = 0; sp < 4; ++sp) {
      const int rr = sp * 16 + (tid >> 5);
      const int64_t m = (int64_t)tm * BIG + pass * 64 + rr;
      const int64_t n = (int64_t)tn * BIG + c;
      if (m >= Mb || n >= N) continue;
      float v[8];
      {
        v4f a0 = *reinterpret_cast<const v4f*>(stg + rr * SROW + c);
        v4f a1 = *reinterpret_cast<const v4f*>(stg + rr * SROW + c + 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) { v[t] = a0[t] * ep.alpha; v[4 + t] = a1[t] * ep.alpha; }
      }
      if constexpr ((EX & 4) != 0)
        epi_row8<true, EX>(ep, eo, v, m, n, N, la.out_row(m), cs, cq, false, uint4{}, use_gm, gpre[sp]);
      else
        epi_row8<true, EX>(ep, eo, v, m, n, N, la.out_row(m), cs, cq);
    }
    __syncthreads();
  }
  if (ep.colstats)
    epilogue_colstats<32, 8>(cs, cq, stg, tid, (int64_t)tn * BIG, N,
                             ep.colstats + (ep.cs_rep > 1 ? (int64_t)(blockIdx.x % ep.cs_rep) * 2 * N : 0));
}

// dst[m][n] (ld ldd, fp32 or bf16) (+)= sum_z slab[z][m][n]
static __global__ void splitk_reduce_k(const float* __restrict__ slab, int64_t stride, int nz,
                                void* dst, int64_t M, int64_t N, int64_t ldd, int out_f32,
                                int accumulate) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < nz; ++z) v += slab[z * stride + i];
    const int64_t m = i / N, n = i - m * N;
    const int64_t o = m * ldd + n;
    if (out_f32) {
      float* d = (float*)dst;
      d[o] = accumulate ? d[o] + v : v;
    } else {
      unsigned short* d = (unsigned short*)dst;
      d[o] = f_to_bf16_bits(accumulate ? bf16_bits_to_f(d[o]) + v : v);
    }
  }
}

// Vector form of splitk_reduce_k for fp32 outputs with N % 4 == 0, ldd % 4 == 0
// and 16-byte aligned slab / dst: 4 columns per lane, the slices' loads in flight.
static __global__ void __launch_bounds__(256) splitk_reduce_vec_k(const float* __restrict__ slab, int64_t stride, int nz,
                                                            float* __restrict__ dst, int64_t M, int64_t N,
                                                            int64_t ldd, int accumulate) {
  const int64_t n4 = N / 4, total4 = M * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / n4, c = (i - m * n4) * 4;
    float4 acc = *reinterpret_cast<const float4*>(slab + m * N + c);
    int z = 1;
    for (; z + 1 < nz; z += 2) {
      const float4 a = *reinterpret_cast<const float4*>(slab + z * stride + m * N + c);
      const float4 b = *reinterpret_cast<const float4*>(slab + (z + 1) * stride + m * N + c);
      acc.x += a.x + b.x; acc.y += a.y + b.y; acc.z += a.z + b.z; acc.w += a.w + b.w;
    }
    if (z < nz) {
      const float4 a = *reinterpret_cast<const float4*>(slab + z * stride + m * N + c);
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    float4* d = reinterpret_cast<float4*>(dst + m * ldd + c);
    if (accumulate) {
      const float4 o = *d;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    }
    *d = acc;
  }
}

// Many slabs over a small output (weight gradients: thousands of outputs, 16-64 splits):
// 8 thread groups per block take every 8th slab for 32 float4 outputs, so a thread has a
// few independent loads instead of a chain of nz, and 8x more threads are in flight;
// the 8 partials are folded through LDS.
static __global__ void __launch_bounds__(256) splitk_reduce_grp_k(const float* __restrict__ slab, int64_t stride,
                                                                 int nz, float* __restrict__ dst, int64_t M,
                                                                 int64_t N, int64_t ldd, int accumulate) {
  __shared__ float4 part[8][32];
  const int o = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t n4 = N / 4, total4 = M * n4;
  const int64_t i = (int64_t)blockIdx.x * 32 + o;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t m = 0, c = 0;
  if (i < total4) {
    m = i / n4;
    c = (i - m * n4) * 4;
    const float* base = slab + m * N + c;
#pragma unroll 4
    for (int z = g; z < nz; z += 8) {
      const float4 a = *reinterpret_cast<const float4*>(base + z * stride);
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
  }
  part[g][o] = acc;
  __syncthreads();
  if (g == 0 && i < total4) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float4 a = part[k][o];
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    float4* d = reinterpret_cast<float4*>(dst + m * ldd + c);
    if (accumulate) {
      const float4 od = *d;
      acc.x += od.x; acc.y += od.y; acc.z += od.z; acc.w += od.w;
    }
    *d = acc;
  }
}

static void launch_splitk_reduce(const float* slab, int splitk, void* C, int64_t M, int64_t N, int64_t ldc,
                                 int out_f32, int atomic, hipStream_t st) {
  if (out_f32 && (N % 4) == 0 && (ldc % 4) == 0 && ((((uintptr_t)slab) | ((uintptr_t)C)) & 15) == 0 &&
      splitk >= 8 && M * N / 4 <= (1 << 20)) {
    const int64_t nb = (M * N / 4 + 31) / 32;
    hipLaunchKernelGGL(splitk_reduce_grp_k, dim3((unsigned)nb), dim3(256), 0, st, slab, M * N, splitk, (float*)C, M,
                       N, ldc, atomic);
    return;
  }
  if (out_f32 && (N % 4) == 0 && (ldc % 4) == 0 && ((((uintptr_t)slab) | ((uintptr_t)C)) & 15) == 0) {
    int nb = (int)std::min<int64_t>((M * N / 4 + 255) / 256, 4096);
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(splitk_reduce_vec_k, dim3(nb), dim3(256), 0, st, slab, M * N, splitk, (float*)C, M, N,
                       ldc, atomic);
    return;
  }
  int nb = (int)std::min<int64_t>((M * N + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_k, dim3(nb), dim3(256), 0, st, slab, M * N, splitk, C, M, N, ldc, out_f32,
                     atomic);
}

// dst[n][m] (fp32, ld ldd) (+)= sum_z slab[z][m][n]: the reduce of a split-K GEMM that
// computed the transposed product (role-swapped weight gradients)
static __global__ void __launch_bounds__(256) splitk_reduce_t_k(const float* __restrict__ slab, int64_t stride,
                                                               int nz, float* __restrict__ dst, int64_t M,
                                                               int64_t N, int64_t ldd, int accumulate) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
    int z = 0;
    for (; z + 1 < nz; z += 2) { a0 += slab[z * stride + i]; a1 += slab[(z + 1) * stride + i]; }
    if (z < nz) a0 += slab[z * stride + i];
    const int64_t m = i / N, n = i - m * N;
    float* d = dst + n * ldd + m;
    *d = accumulate ? *d + (a0 + a1) : (a0 + a1);
  }
}

// split-K product into fp32 slabs (ws: splitk * M * N floats) and a transposed reduce
// into dst[n][m] -- launch_t with the slab forced for every split count
template <class LA, class LB, int WN>
static int launch_t_transposed(const LA& la, const LB& lb, float* dst, int64_t ldd, int accumulate, float* ws,
                               int64_t M, int64_t N, int64_t K, int splitk, hipStream_t st) {
  constexpr int TBN = 32 * WN;
  int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + TBN - 1) / TBN);
  int nkt = (int)((K + BK - 1) / BK);
  if (splitk < 1) splitk = 1;
  if (splitk > nkt) splitk = nkt > 0 ? nkt : 1;
  int ktps = (nkt + splitk - 1) / splitk;
  splitk = (nkt + ktps - 1) / ktps;
  Epi ep{nullptr, nullptr, nullptr, N, 0, 0, 0, 1.f, 0.f, 0, 1, 0, 0, 0, ws, M * N, nullptr};
  dim3 grid(tiles_m * tiles_n, 1, splitk);
  if (ktps > 1)
    hipLaunchKernelGGL((gemm_kernel<LA, LB, 2, WN>), grid, dim3(NT), 0, st, la, lb, ep, M, N, K, tiles_m, tiles_n,
                       ktps);
  else
    hipLaunchKernelGGL((gemm_kernel<LA, LB, 1, WN>), grid, dim3(NT), 0, st, la, lb, ep, M, N, K, tiles_m, tiles_n,
                       ktps);
  int nb = (int)std::min<int64_t>((M * N + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_t_k, dim3(nb), dim3(256), 0, st, ws, M * N, splitk, dst, M, N, ldd, accumulate);
  return (int)hipGetLastError();
}

template <class LA, class LB>
static int launch_big(const LA& la, const LB& lb, const Epi& ep, int64_t M, int64_t N, int64_t K,
                      int batch, int splitk, hipStream_t st) {
  int tiles_m = (int)((M + BIG - 1) / BIG), tiles_n = (int)((N + BIG - 1) / BIG);
  int nkt = (int)((K + BK - 1) / BK);
  if (splitk < 1) splitk = 1;
  if (splitk > nkt) splitk = nkt > 0 ? nkt : 1;
  int ktps = (nkt + splitk - 1) / splitk;
  splitk = (nkt + ktps - 1) / ktps;
  if (splitk < 1) splitk = 1;
  dim3 grid(tiles_m * tiles_n, batch, splitk);
  Epi e1 = ep;
  if (ep.slab && splitk > 1) {
    e1.slab_stride = M * N;
    hipLaunchKernelGGL((gemm_big_kernel<LA, LB>), grid, dim3(BIG_NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                       tiles_n, ktps);
    launch_splitk_reduce(ep.slab, splitk, ep.C, M, N, ep.ldc, ep.out_f32, ep.atomic, st);
    return (int)hipGetLastError();
  }
  e1.slab = nullptr;
  if (splitk > 1) e1.atomic = 1;
  if (ep.C2 || ep.drop_keep > 0.f || ep.gmask) {
    if constexpr (is_buf<LA>::value && is_buf<LB>::value) {
      if ((ep.C2 ? 1 : 0) + (ep.drop_keep > 0.f ? 1 : 0) + (ep.gmask ? 1 : 0) > 1)
        return (int)hipErrorInvalidValue;   // one feature per build
      if (ep.C2)
        hipLaunchKernelGGL((gemm_big_kernel<LA, LB, 1>), grid, dim3(BIG_NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                           tiles_n, ktps);
      else if (ep.gmask)
        hipLaunchKernelGGL((gemm_big_kernel<LA, LB, 4>), grid, dim3(BIG_NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                           tiles_n, ktps);
      else
        hipLaunchKernelGGL((gemm_big_kernel<LA, LB, 2>), grid, dim3(BIG_NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                           tiles_n, ktps);
      return (int)hipGetLastError();
    } else {
      return (int)hipErrorInvalidValue;
    }
  }
  hipLaunchKernelGGL((gemm_big_kernel<LA, LB>), grid, dim3(BIG_NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                     tiles_n, ktps);
  return (int)hipGetLastError();
}

// loader pairs of the data-gradient launches (hetu_conv_dgrad_bf16): the only ones that
// instantiate the BN-backward epilogue of the 128-row tiles
template <class LA, class LB> struct bnx_pair : std::false_type {};
template <bool KF, int NS> struct bnx_pair<BufK<KF, NS>, BufMN<KF, NS>> : std::true_type {};
template <> struct bnx_pair<ConvDgradA, ConvDgradB> : std::true_type {};

// tile: 0 = 128x128 (4 waves, 2 LDS stages, 2 blocks per CU), 1 = 256x256 (8 waves, 1 block
// per CU), 2 = 128x64 (4 waves of 64x32; 64-channel convolutions), 3 = 128x128 single LDS
// stage at 4 blocks per CU (short-K, memory-bound shapes), 5 = 128x96 (4 waves of 64x48),
// 6 / 7 = 128x128 / 128x96 with the two-ahead K loop (ST 3; plain GEMM loaders).
template <class LA, class LB, int WN>
static int launch_t(const LA& la, const LB& lb, const Epi& ep, int64_t M, int64_t N, int64_t K,
                    int batch, int splitk, hipStream_t st, bool single_stage = false, bool two_ahead = false) {
  constexpr int TBN = 32 * WN;
  int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + TBN - 1) / TBN);
  int nkt = (int)((K + BK - 1) / BK);
  if (splitk < 1) splitk = 1;
  if (splitk > nkt) splitk = nkt > 0 ? nkt : 1;
  int ktps = (nkt + splitk - 1) / splitk;
  splitk = (nkt + ktps - 1) / ktps;
  if (splitk < 1) splitk = 1;
  dim3 grid(tiles_m * tiles_n, batch, splitk);
  Epi e1 = ep;
  const bool slab = ep.slab && splitk > 1;
  if (slab) {
    e1.slab_stride = M * N;
  } else {
    e1.slab = nullptr;
    if (splitk > 1) e1.atomic = 1;
  }
  const bool bnx = ep.bnx || ep.cin_w;
  if (ep.C2 || ep.drop_keep > 0.f || ep.gmask) {
    // pre-activation copy / epilogue dropout / gradient mask: the EX builds of the plain-GEMM
    // loader pairs
    if constexpr (is_buf<LA>::value && is_buf<LB>::value) {
      if (bnx || (ep.C2 ? 1 : 0) + (ep.drop_keep > 0.f ? 1 : 0) + (ep.gmask ? 1 : 0) > 1)
        return (int)hipErrorInvalidValue;   // one feature per build
      auto go = [&](auto ex) {
        constexpr int X = decltype(ex)::value;
        if (ktps > 2 && two_ahead)
          hipLaunchKernelGGL((gemm_kernel<LA, LB, 3, WN, false, X>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K,
                             tiles_m, tiles_n, ktps);
        else if (ktps > 1 && !single_stage)
          hipLaunchKernelGGL((gemm_kernel<LA, LB, 2, WN, false, X>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K,
                             tiles_m, tiles_n, ktps);
        else
          hipLaunchKernelGGL((gemm_kernel<LA, LB, 1, WN, false, X>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K,
                             tiles_m, tiles_n, ktps);
      };
      if (ep.C2) go(std::integral_constant<int, 1>{});
      else if (ep.gmask) go(std::integral_constant<int, 4>{});
      else go(std::integral_constant<int, 2>{});
      return (int)hipGetLastError();
    } else {
      return (int)hipErrorInvalidValue;
    }
  }
  if (bnx) {
    // the BN-backward / subgrid-Cin epilogue: data-gradient loader pairs only
    if constexpr (bnx_pair<LA, LB>::value) {
      if (ktps > 1 && !single_stage)
        hipLaunchKernelGGL((gemm_kernel<LA, LB, 2, WN, true>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                           tiles_n, ktps);
      else
        hipLaunchKernelGGL((gemm_kernel<LA, LB, 1, WN, true>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K, tiles_m,
                           tiles_n, ktps);
    } else {
      return (int)hipErrorInvalidValue;
    }
  } else if (ktps > 2 && two_ahead) {
    if constexpr (is_buf<LA>::value && is_buf<LB>::value)
      hipLaunchKernelGGL((gemm_kernel<LA, LB, 3, WN>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K, tiles_m, tiles_n,
                         ktps);
    else
      return (int)hipErrorInvalidValue;
  } else if (ktps > 1 && !single_stage)
    hipLaunchKernelGGL((gemm_kernel<LA, LB, 2, WN>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K, tiles_m, tiles_n,
                       ktps);
  else
    hipLaunchKernelGGL((gemm_kernel<LA, LB, 1, WN>), grid, dim3(NT), 0, st, la, lb, e1, M, N, K, tiles_m, tiles_n,
                       ktps);
  if (slab) launch_splitk_reduce(ep.slab, splitk, ep.C, M, N, ep.ldc, ep.out_f32, ep.atomic, st);
  return (int)hipGetLastError();
}

template <class LA, class LB>
static int launch(const LA& la, const LB& lb, const Epi& ep, int64_t M, int64_t N, int64_t K,
                  int batch, int splitk, hipStream_t st, int tile = 0) {
  if (tile == 1) return launch_big(la, lb, ep, M, N, K, batch, splitk, st);
  if (tile == 2) return launch_t<LA, LB, 2>(la, lb, ep, M, N, K, batch, splitk, st);
  if (tile == 3) return launch_t<LA, LB, 4>(la, lb, ep, M, N, K, batch, splitk, st, true);
  if (tile == 5) {
    // 128x96: N = 768 products fill 2 tiles per CU in one round (8192x768: 512 tiles) where
    // the 128-wide tile leaves half the CUs one block short (384).  The 12-thread row
    // groups do not fold by lane shuffles: no fused column statistics on this tile.
    if (ep.colstats) return (int)hipErrorInvalidValue;
    return launch_t<LA, LB, 3>(la, lb, ep, M, N, K, batch, splitk, st);
  }
  // 6 / 7: the 128x128 / 128x96 tiles with the two-ahead K loop (plain GEMM loaders only)
  if (tile == 6 || tile == 7) {
    if constexpr (!(is_buf<LA>::value && is_buf<LB>::value)) return (int)hipErrorInvalidValue;
    if (tile == 7) {
      if (ep.colstats) return (int)hipErrorInvalidValue;
      return launch_t<LA, LB, 3>(la, lb, ep, M, N, K, batch, splitk, st, false, true);
    }
    return launch_t<LA, LB, 4>(la, lb, ep, M, N, K, batch, splitk, st, false, true);
  }
  return launch_t<LA, LB, 4>(la, lb, ep, M, N, K, batch, splitk, st);
}

// split count: ~2 blocks per CU in flight, each slice at least 8 K-tiles
static int pick_splitk(int64_t M, int64_t N, int64_t K) {
  int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int64_t ktiles = (K + BK - 1) / BK;
  int64_t want = (512 + tiles - 1) / tiles;
  int64_t cap = std::max<int64_t>(1, ktiles / 8);
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min(want, cap), 512));
}


template <bool KF>
int launch_buf(const bf16* a, const bf16* b, int a_kmaj, int b_kmaj, int64_t lda, int64_t ldb,
                      int64_t sA, int64_t sB, const Epi& ep, int64_t M, int64_t N, int64_t K, int batch,
                      int splitk, hipStream_t st, int tile) {
  if (a_kmaj && b_kmaj)
    return launch(BufK<KF>{a, lda, M, K, sA}, BufK<KF>{b, ldb, N, K, sB}, ep, M, N, K, batch, splitk, st, tile);
  if (a_kmaj)
    return launch(BufK<KF>{a, lda, M, K, sA}, BufMN<KF>{b, ldb, N, K, sB}, ep, M, N, K, batch, splitk, st, tile);
  if (b_kmaj)
    return launch(BufMN<KF>{a, lda, M, K, sA}, BufK<KF>{b, ldb, N, K, sB}, ep, M, N, K, batch, splitk, st, tile);
  return launch(BufMN<KF>{a, lda, M, K, sA}, BufMN<KF>{b, ldb, N, K, sB}, ep, M, N, K, batch, splitk, st, tile);
}
extern template int launch_buf<true>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t,
                                     const Epi&, int64_t, int64_t, int64_t, int, int, hipStream_t, int);
extern template int launch_buf<false>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t,
                                      const Epi&, int64_t, int64_t, int64_t, int, int, hipStream_t, int);

// 16 B-aligned operand slices below 2 GiB take the buffer-descriptor loaders
inline bool buf_ok(int64_t abytes, int64_t bbytes) { return abytes < (1ll << 31) && bbytes < (1ll << 31); }

static ConvGeom geom(int N, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw) {
  ConvGeom g{N, H, W, C, K, KH, KW, sh, sw, ph, pw, 0, 0};
  g.ctap = 0;
  g.OH = (H + 2 * ph - KH) / sh + 1;
  g.OW = (W + 2 * pw - KW) / sw + 1;
  g.fOW = FastDiv((uint32_t)g.OW);
  g.fOH = FastDiv((uint32_t)g.OH);
  g.fC = FastDiv((uint32_t)C);
  g.fK = FastDiv((uint32_t)K);
  g.fKW = FastDiv((uint32_t)KW);
  return g;
}

}  // namespace gemm
}  // namespace hetu
