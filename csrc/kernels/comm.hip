// Kernels of the mixed-precision gradient collective (parallel/rccl.py
// all_reduce_bf16): fp32 <-> bf16 casts of a bucket and the fp32-accumulated sum of
// the P bf16 chunks an all-to-all delivered (chunk p = peer p's copy of this rank's
// shard).  16-byte vectors, grid-stride.
#include "common.h"

using namespace hetu;

// y[0, npad) = bf16(x[0, n)), zero beyond n (the padding of the last chunk)
__global__ void __launch_bounds__(256) cast_f32_bf16_k(const float* __restrict__ x, unsigned short* __restrict__ y,
                                                       int64_t n, int64_t npad) {
  const int64_t n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint2* y4 = reinterpret_cast<uint2*>(y);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = tid; i < n4; i += nth) {
    const float4 v = x4[i];
    y4[i] = make_uint2((uint32_t)f_to_bf16_bits(v.x) | ((uint32_t)f_to_bf16_bits(v.y) << 16),
                       (uint32_t)f_to_bf16_bits(v.z) | ((uint32_t)f_to_bf16_bits(v.w) << 16));
  }
  for (int64_t i = n4 * 4 + tid; i < npad; i += nth) y[i] = i < n ? f_to_bf16_bits(x[i]) : (unsigned short)0;
}

__global__ void __launch_bounds__(256) cast_bf16_f32_k(const unsigned short* __restrict__ x, float* __restrict__ y,
                                                       int64_t n) {
  const int64_t n4 = n / 4;
  const uint2* x4 = reinterpret_cast<const uint2*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = tid; i < n4; i += nth) {
    const uint2 v = x4[i];
    y4[i] = make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                        __uint_as_float(v.y & 0xffff0000u));
  }
  for (int64_t i = n4 * 4 + tid; i < n; i += nth) y[i] = bf16_bits_to_f(x[i]);
}

// out[j] = bf16( sum_p in[p * c + j] ), accumulated in fp32; 8 elements per lane
__global__ void __launch_bounds__(256) sum_chunks_bf16_k(const uint4* __restrict__ in, int P, int64_t c8,
                                                         uint4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c8; i += (int64_t)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < P; ++p) {
      const uint4 v = in[p * c8 + i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[2 * q] += __uint_as_float(w[q] << 16);
        a[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      w[q] = (uint32_t)f_to_bf16_bits(a[2 * q]) | ((uint32_t)f_to_bf16_bits(a[2 * q + 1]) << 16);
    out[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// 16-byte aligned x / 8-byte aligned y; y is written up to npad >= n (zero tail)
HETU_API int hetu_cast_f32_bf16(const float* x, void* y, int64_t n, int64_t npad, hipStream_t st) {
  if (npad < n || (((uintptr_t)x) & 15) || (((uintptr_t)y) & 7)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_f32_bf16_k, dim3(stream_grid(npad / 4 + 1, 256)), dim3(256), 0, st, x,
                     (unsigned short*)y, n, npad);
  return (int)hipGetLastError();
}

HETU_API int hetu_cast_bf16_f32(const void* x, float* y, int64_t n, hipStream_t st) {
  if ((((uintptr_t)y) & 15) || (((uintptr_t)x) & 7)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_bf16_f32_k, dim3(stream_grid(n / 4 + 1, 256)), dim3(256), 0, st, (const unsigned short*)x,
                     y, n);
  return (int)hipGetLastError();
}

// c % 8 == 0, 16-byte aligned buffers
HETU_API int hetu_sum_chunks_bf16(const void* in, int P, int64_t c, void* out, hipStream_t st) {
  if (c & 7) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sum_chunks_bf16_k, dim3(stream_grid(c / 8, 256)), dim3(256), 0, st, (const uint4*)in, P, c / 8,
                     (uint4*)out);
  return (int)hipGetLastError();
}
