// Shared device helpers for the hetu_61a7_amd HIP kernels (gfx950 / CDNA4).
//
// Conventions (SURVEY.md §2.5 "Shared MI355X conventions"):
//   * 256-thread workgroups unless a kernel says otherwise, wave = 64 lanes.
//   * 16-byte vector loads/stores on the streaming paths.
//   * bf16 / fp32 templates; accumulation always in fp32.
//   * shape metadata passed by value in kernel arguments (no per-call H2D
//     metadata copies as in the reference's "(md)" kernels).
//   * every entry point is `extern "C" int hetu_xxx(..., hipStream_t)` and
//     returns 0 on success, a hipError_t otherwise.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define HETU_API extern "C" __attribute__((visibility("default")))

namespace hetu {

constexpr int kWave = 64;

typedef __hip_bfloat16 bf16;

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f(__half x) { return __half2float(x); }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return __float2bfloat16(x); }
template <> __device__ __forceinline__ __half from_f<__half>(float x) { return __float2half(x); }

// raw bf16 bit helpers for packed (ushort) vector paths
__device__ __forceinline__ float bf16_bits_to_f(unsigned short b) {
  return __uint_as_float(((unsigned int)b) << 16);
}
__device__ __forceinline__ unsigned short f_to_bf16_bits(float f) {
  // round-to-nearest-even; NaN stays NaN through the compiler's v_cvt path
  bf16 h = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&h);
}

// wave64 reductions via DPP-backed shuffles
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block reduction for blockDim.x == NT (multiple of 64); `sh` >= NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = (threadIdx.x < NT / 64) ? sh[threadIdx.x] : 0.f;
  if (w == 0) r = wave_sum(r);
  if (threadIdx.x == 0) sh[0] = r;
  __syncthreads();
  r = sh[0];
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = (threadIdx.x < NT / 64) ? sh[threadIdx.x] : -INFINITY;
  if (w == 0) r = wave_max(r);
  if (threadIdx.x == 0) sh[0] = r;
  __syncthreads();
  r = sh[0];
  return r;
}

// grid sizing for streaming kernels: cap at 256 CUs x 8 blocks, grid-stride
__host__ inline int stream_grid(int64_t n, int nt, int per_thread = 1) {
  int64_t b = (n + (int64_t)nt * per_thread - 1) / ((int64_t)nt * per_thread);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

// Philox4x32-10 counter-based RNG (replaces cuRAND device API)
struct Philox {
  __device__ static inline void round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                      uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  // returns 4 uint32 for (seed, counter)
  __device__ static inline uint4 gen(uint64_t seed, uint64_t counter) {
    uint32_t c0 = (uint32_t)counter, c1 = (uint32_t)(counter >> 32), c2 = 0, c3 = 0;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      round(c0, c1, c2, c3, k0, k1);
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
  __device__ static inline float u01(uint32_t x) {  // (0,1]
    return (float)(x >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
  }
};

// Graph-safe RNG: every seeded kernel draws from Philox(rng_seed(seed, off))
// where `seed` is the launch's host seed -- fixed per op and per call within a step, so a
// captured hipGraph replays the same launch arguments -- and `off` points at the device's
// step counter, which the framework advances once per training step with
// hetu_rng_advance (a one-thread kernel on the step's stream, captured with the step).
// A replay therefore draws fresh masks, and eager and replayed steps draw the same ones.
// The forward and the backward of a step read the same counter value.  off == nullptr
// (no counter registered on this device): the host seed alone.
constexpr uint64_t kRngMix = 0x9E3779B97F4A7C15ull;
__device__ __forceinline__ uint64_t rng_seed(uint64_t seed, const uint64_t* off) {
  return off ? seed + *off * kRngMix : seed;
}
// host: the registered step counter of the calling thread's current device (random.hip)
uint64_t* hetu_rng_offset_ptr();

// 16-byte vector load/store helpers (8 bf16 or 4 fp32 per lane)
template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int N = 4; typedef float4 type; };
template <> struct Vec<bf16> { static constexpr int N = 8; typedef uint4 type; };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float (&v)[Vec<T>::N]);
template <>
__device__ __forceinline__ void load_vec<float>(const float* p, float (&v)[4]) {
  float4 x = *reinterpret_cast<const float4*>(p);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
template <>
__device__ __forceinline__ void load_vec<bf16>(const bf16* p, float (&v)[8]) {
  uint4 x = *reinterpret_cast<const uint4*>(p);
  const unsigned int w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float (&v)[Vec<T>::N]);
template <>
__device__ __forceinline__ void store_vec<float>(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void store_vec<bf16>(bf16* p, const float (&v)[8]) {
  unsigned int w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (unsigned)f_to_bf16_bits(v[2 * i]) | ((unsigned)f_to_bf16_bits(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace hetu

#define HETU_LAUNCH_CHECK() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
