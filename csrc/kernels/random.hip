// Random-number kernels and the graph-safe RNG step counter (gfx950).
//
// Reference: src/ops/Dropout2d.cu:4,30-35 (channel dropout), src/ops/Initializers.cu
// (uniform / normal / truncated-normal fills), src/ops/ArraySet.cu, curand-based
// Dropout.cu:24-26 (a fresh seed per forward).  MI355X design: every draw is
// Philox4x32-10 at counter = element (or plane) index, with the seed offset by the
// device's step counter (common.h rng_seed) -- so a hipGraph-replayed step draws fresh
// values without re-capture, and the backward regenerates the forward's mask from the
// same (seed, counter) instead of keeping a mask tensor.
#include "common.h"

namespace hetu {

static uint64_t* g_rng_off[64];

uint64_t* hetu_rng_offset_ptr() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
  return g_rng_off[d];
}

namespace {

__global__ void rng_advance_k(uint64_t* c, uint64_t by) { *c += by; }

// uniform [lo, hi) (fp32 or bf16 out): 4 values per Philox call
template <typename T>
__global__ void __launch_bounds__(256) uniform_k(T* __restrict__ y, int64_t n, float lo, float hi, uint64_t seed_,
                                                 const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n; q += (int64_t)gridDim.x * blockDim.x) {
    const uint4 r = Philox::gen(seed, (uint64_t)q);
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t i = q * 4 + t;
      if (i < n) y[i] = from_f<T>(lo + (hi - lo) * (Philox::u01(rr[t]) - 0.5f / 16777216.0f));
    }
  }
}

// normal(mean, std) by Box-Muller on Philox pairs; trunc > 0: values beyond trunc * std
// are redrawn from the next counters (reference truncated_normal: |x - mean| <= 2 std)
template <typename T>
__global__ void __launch_bounds__(256) normal_k(T* __restrict__ y, int64_t n, float mean, float sd, float trunc,
                                                uint64_t seed_, const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q * 2 < n; q += (int64_t)gridDim.x * blockDim.x) {
    float z[2];
    uint64_t ctr = (uint64_t)q;
    for (int attempt = 0; attempt < 16; ++attempt) {
      const uint4 r = Philox::gen(seed, ctr);
      const float u1 = Philox::u01(r.x), u2 = Philox::u01(r.y);
      const float rad = sqrtf(-2.f * __logf(u1));
      float s, c;
      __sincosf(6.283185307179586f * u2, &s, &c);
      z[0] = rad * c;
      z[1] = rad * s;
      if (trunc <= 0.f || (fabsf(z[0]) <= trunc && fabsf(z[1]) <= trunc)) break;
      ctr += (uint64_t)1 << 40;     // a disjoint counter range per redraw
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int64_t i = q * 2 + t;
      if (i < n) y[i] = from_f<T>(mean + sd * z[t]);
    }
  }
}

// channel dropout: plane p = (n, c) kept with probability keep (Philox(seed, p).x), kept
// planes scaled by 1 / keep.  cl: channels-last memory (element i of plane
// (i / (HW * C), i % C)); else NCHW (plane i / HW).  8 elements per thread when aligned.
template <typename T>
__global__ void __launch_bounds__(256) dropout2d_k(const T* __restrict__ x, T* __restrict__ y, int64_t n, int C,
                                                   int64_t HW, int cl, float keep, uint64_t seed_,
                                                   const uint64_t* __restrict__ rngo) {
  const uint64_t seed = rng_seed(seed_, rngo);
  const float inv = 1.f / keep;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t plane = cl ? (i / (HW * C)) * C + i % C : i / HW;
    const float u = Philox::u01(Philox::gen(seed, (uint64_t)plane).x);
    y[i] = from_f<T>(u < keep ? to_f(x[i]) * inv : 0.f);
  }
}

// y[i] = start + i * step
template <typename T>
__global__ void __launch_bounds__(256) arange_k(T* __restrict__ y, int64_t n, double start, double step) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = from_f<T>((float)(start + (double)i * step));
}

}  // namespace
}  // namespace hetu

using namespace hetu;

// the device's step counter (a framework-owned device uint64, zero-initialised); null
// unregisters it
HETU_API int hetu_rng_register(int device, void* counter) {
  if (device < 0 || device >= 64) return (int)hipErrorInvalidValue;
  g_rng_off[device] = (uint64_t*)counter;
  return 0;
}

// *counter += by on `st` (captured with the step when the stream is capturing)
HETU_API int hetu_rng_advance(void* counter, int64_t by, hipStream_t st) {
  if (counter == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rng_advance_k, dim3(1), dim3(1), 0, st, (uint64_t*)counter, (uint64_t)by);
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_uniform(void* y, int64_t n, float lo, float hi, int64_t seed, int is_bf16, hipStream_t st) {
  if (n <= 0) return 0;
  const int g = stream_grid((n + 3) / 4, 256, 1);
  if (is_bf16)
    hipLaunchKernelGGL(uniform_k<bf16>, dim3(g), dim3(256), 0, st, (bf16*)y, n, lo, hi, (uint64_t)seed,
                       hetu_rng_offset_ptr());
  else
    hipLaunchKernelGGL(uniform_k<float>, dim3(g), dim3(256), 0, st, (float*)y, n, lo, hi, (uint64_t)seed,
                       hetu_rng_offset_ptr());
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_normal(void* y, int64_t n, float mean, float sd, float trunc, int64_t seed, int is_bf16,
                         hipStream_t st) {
  if (n <= 0) return 0;
  const int g = stream_grid((n + 1) / 2, 256, 1);
  if (is_bf16)
    hipLaunchKernelGGL(normal_k<bf16>, dim3(g), dim3(256), 0, st, (bf16*)y, n, mean, sd, trunc, (uint64_t)seed,
                       hetu_rng_offset_ptr());
  else
    hipLaunchKernelGGL(normal_k<float>, dim3(g), dim3(256), 0, st, (float*)y, n, mean, sd, trunc, (uint64_t)seed,
                       hetu_rng_offset_ptr());
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_dropout2d(const void* x, void* y, int64_t n, int C, int64_t HW, int cl, float keep, int64_t seed,
                            int is_bf16, hipStream_t st) {
  if (n <= 0) return 0;
  if (C <= 0 || HW <= 0 || !(keep > 0.f)) return (int)hipErrorInvalidValue;
  const int g = stream_grid(n, 256, 4);
  if (is_bf16)
    hipLaunchKernelGGL(dropout2d_k<bf16>, dim3(g), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n, C, HW, cl, keep,
                       (uint64_t)seed, hetu_rng_offset_ptr());
  else
    hipLaunchKernelGGL(dropout2d_k<float>, dim3(g), dim3(256), 0, st, (const float*)x, (float*)y, n, C, HW, cl, keep,
                       (uint64_t)seed, hetu_rng_offset_ptr());
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_arange(void* y, int64_t n, double start, double step, int is_bf16, hipStream_t st) {
  if (n <= 0) return 0;
  const int g = stream_grid(n, 256, 4);
  if (is_bf16) hipLaunchKernelGGL(arange_k<bf16>, dim3(g), dim3(256), 0, st, (bf16*)y, n, start, step);
  else hipLaunchKernelGGL(arange_k<float>, dim3(g), dim3(256), 0, st, (float*)y, n, start, step);
  HETU_LAUNCH_CHECK();
  return 0;
}
