// Remaining long-tail kernels of the reference op library:
//   SAM MoE gate helpers   sam_group_sum (+grad), sam_max (+grad), group_topk_idx
//                          (reference SamGroupSum.cu, SamMax.cu, GroupTopKIdx.cu: one
//                          serial thread per row with a local cache[2048] that spills to
//                          scratch; here a wave per row, values in registers)
//   instance_norm2d        per-(n, c) statistics over H*W and the fused backward
//                          (reference InstanceNorm2d.cu: cuDNN ReduceTensor + 3 passes)
//   bicubic interpolate    forward and scatter-add backward, A = -0.75 with border clamp
//                          (reference Interpolate.cu; PyTorch upsample_bicubic2d numerics)
#include "common.h"

using namespace hetu;

namespace {

// ---- SAM --------------------------------------------------------------------------------
// out[t, g] = sum_{e in [g*w, (g+1)*w)} x[t, e], w = E / G
__global__ void __launch_bounds__(256) sam_group_sum_k(const float* __restrict__ x, float* __restrict__ out,
                                                       int64_t T, int E, int G) {
  const int w = E / G;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T * G; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / G;
    const int g = (int)(i - t * G);
    float s = 0.f;
    for (int e = g * w; e < (g + 1) * w; ++e) s += x[t * E + e];
    out[i] = s;
  }
}

__global__ void __launch_bounds__(256) sam_group_sum_grad_k(const float* __restrict__ g, float* __restrict__ dx,
                                                            int64_t T, int E, int G) {
  const int w = E / G;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T * E; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / E;
    const int e = (int)(i - t * E);
    dx[i] = g[t * G + e / w];
  }
}

// y[t, e] = max(0, x[t,e] - x[t, tk[t]]) for e outside [grp[t]*n, (grp[t]+1)*n)
__global__ void __launch_bounds__(256) sam_max_k(const float* __restrict__ x, const int64_t* __restrict__ grp,
                                                 const int64_t* __restrict__ tk, float* __restrict__ y, int64_t T,
                                                 int E, int n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T * E; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / E;
    const int e = (int)(i - t * E);
    const int64_t g = grp[t];
    const bool outside = e < g * n || e >= (g + 1) * n;
    const float d = x[i] - x[t * E + tk[t]];
    y[i] = (outside && d > 0.f) ? d : 0.f;
  }
}

// dx[t, e] = m[t,e] * g[t,e];  dx[t, tk[t]] -= sum_e m[t,e] * g[t,e]   (one wave per row)
__global__ void __launch_bounds__(256) sam_max_grad_k(const float* __restrict__ g, const float* __restrict__ x,
                                                      const int64_t* __restrict__ grp, const int64_t* __restrict__ tk,
                                                      float* __restrict__ dx, int64_t T, int E, int n) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t gg = grp[t], k = tk[t];
  const float ref = x[t * E + k];
  auto val = [&](int e) {
    const bool outside = e < gg * n || e >= (gg + 1) * n;
    return (outside && x[t * E + e] - ref > 0.f) ? g[t * E + e] : 0.f;
  };
  float s = 0.f;
  for (int e = lane; e < E; e += 64) s += val(e);
  s = wave_sum(s);
  for (int e = lane; e < E; e += 64) dx[t * E + e] = val(e) - (e == k ? s : 0.f);
}

// top-k expert ids of row t inside group grp[t] (columns [g*n, (g+1)*n)), descending,
// ties to the lower index; one wave per row, k rounds of a wave arg-max
__global__ void __launch_bounds__(256) group_topk_k(const float* __restrict__ x, const int64_t* __restrict__ grp,
                                                    int64_t* __restrict__ out, int64_t T, int E, int n, int k) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t g = grp[t];
  uint64_t taken = 0;   // lanes' own column choices taken so far (per stripe index)
  for (int r = 0; r < k; ++r) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    int stripe = 0;
    for (int e = (int)(g * n) + lane, j = 0; e < (g + 1) * n && e < E; e += 64, ++j) {
      if (taken >> j & 1ull) continue;
      const float v = x[t * E + e];
      if (v > best || (v == best && e < bi)) { best = v; bi = e; stripe = j; }
    }
    float b = best;
    int i = bi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(i, o, 64);
      if (ob > b || (ob == b && oi < i)) { b = ob; i = oi; }
    }
    if (bi == i && bi != 0x7fffffff) taken |= 1ull << stripe;
    if (lane == 0) out[t * k + r] = i == 0x7fffffff ? (int64_t)(g * n) : (int64_t)i;
  }
}

// ---- instance norm 2d ----------------------------------------------------------------------
// x viewed as [N*C lines][HW] with element strides (line = n*C + c): off = n*sN + c*sC + p*sP
template <typename T>
__global__ void __launch_bounds__(256) inorm_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                   float* __restrict__ mean, float* __restrict__ rstd, int C,
                                                   int64_t HW, int64_t sN, int64_t sC, int64_t sP, float eps) {
  __shared__ float sh[4];
  const int64_t line = blockIdx.x;
  const int64_t n = line / C, c = line % C;
  const int64_t base = n * sN + c * sC;
  float s = 0.f;
  for (int64_t p = threadIdx.x; p < HW; p += blockDim.x) s += to_f(x[base + p * sP]);
  const float mu = block_sum<256>(s, sh) / (float)HW;
  float q = 0.f;
  for (int64_t p = threadIdx.x; p < HW; p += blockDim.x) {
    const float d = to_f(x[base + p * sP]) - mu;
    q += d * d;
  }
  const float rs = rsqrtf(block_sum<256>(q, sh) / (float)HW + eps);
  for (int64_t p = threadIdx.x; p < HW; p += blockDim.x)
    y[base + p * sP] = from_f<T>((to_f(x[base + p * sP]) - mu) * rs);
  if (threadIdx.x == 0) {
    mean[line] = mu;
    rstd[line] = rs;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) over each (n, c)
template <typename T>
__global__ void __launch_bounds__(256) inorm_bwd_k(const T* __restrict__ g, const T* __restrict__ x,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   T* __restrict__ dx, int C, int64_t HW, int64_t sN, int64_t sC,
                                                   int64_t sP) {
  __shared__ float sh[4];
  const int64_t line = blockIdx.x;
  const int64_t n = line / C, c = line % C;
  const int64_t base = n * sN + c * sC;
  const float mu = mean[line], rs = rstd[line];
  float a = 0.f, b = 0.f;
  for (int64_t p = threadIdx.x; p < HW; p += blockDim.x) {
    const float gv = to_f(g[base + p * sP]);
    a += gv;
    b += gv * (to_f(x[base + p * sP]) - mu) * rs;
  }
  const float mg = block_sum<256>(a, sh) / (float)HW;
  const float mgx = block_sum<256>(b, sh) / (float)HW;
  for (int64_t p = threadIdx.x; p < HW; p += blockDim.x) {
    const float xh = (to_f(x[base + p * sP]) - mu) * rs;
    dx[base + p * sP] = from_f<T>(rs * (to_f(g[base + p * sP]) - mg - xh * mgx));
  }
}

// ---- bicubic (PyTorch upsample_bicubic2d numerics) -------------------------------------------------
__device__ __forceinline__ float cc1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cc2(float x, float A) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }

__device__ __forceinline__ void cubic_w(float t, float (&w)[4]) {
  const float A = -0.75f;
  w[0] = cc2(t + 1.f, A);
  w[1] = cc1(t, A);
  w[2] = cc1(1.f - t, A);
  w[3] = cc2(2.f - t, A);
}

__device__ __forceinline__ float src_index(float scale, int64_t dst, int align) {
  return align ? scale * (float)dst : scale * ((float)dst + 0.5f) - 0.5f;
}

// x, y contiguous NCHW fp32
__global__ void __launch_bounds__(256) bicubic_fwd_k(const float* __restrict__ x, float* __restrict__ y, int64_t NC,
                                                     int H, int W, int OH, int OW, float sh, float sw, int align) {
  const int64_t total = NC * OH * OW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const int64_t nc = i / ((int64_t)OW * OH);
    const float ry = src_index(sh, oy, align), rx = src_index(sw, ox, align);
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    float wy[4], wx[4];
    cubic_w(ry - iy, wy);
    cubic_w(rx - ix, wx);
    const float* xp = x + nc * H * W;
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int yy = min(max(iy - 1 + a, 0), H - 1);
      float r = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b) r += wx[b] * xp[(int64_t)yy * W + min(max(ix - 1 + b, 0), W - 1)];
      acc += wy[a] * r;
    }
    y[i] = acc;
  }
}

// dx (fp32, zeroed) += the transpose of the forward stencil
__global__ void __launch_bounds__(256) bicubic_bwd_k(const float* __restrict__ g, float* __restrict__ dx, int64_t NC,
                                                     int H, int W, int OH, int OW, float sh, float sw, int align) {
  const int64_t total = NC * OH * OW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const int64_t nc = i / ((int64_t)OW * OH);
    const float ry = src_index(sh, oy, align), rx = src_index(sw, ox, align);
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    float wy[4], wx[4];
    cubic_w(ry - iy, wy);
    cubic_w(rx - ix, wx);
    float* dp = dx + nc * H * W;
    const float gv = g[i];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int yy = min(max(iy - 1 + a, 0), H - 1);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        unsafeAtomicAdd(dp + (int64_t)yy * W + min(max(ix - 1 + b, 0), W - 1), gv * wy[a] * wx[b]);
    }
  }
}

}  // namespace

HETU_API int hetu_sam_group_sum(const float* x, float* out, int64_t T, int E, int G, hipStream_t st) {
  if (T * G == 0 || G <= 0 || E % G) return T * G == 0 ? 0 : (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sam_group_sum_k, dim3(stream_grid(T * G, 256)), dim3(256), 0, st, x, out, T, E, G);
  return (int)hipGetLastError();
}

HETU_API int hetu_sam_group_sum_grad(const float* g, float* dx, int64_t T, int E, int G, hipStream_t st) {
  if (T * E == 0 || G <= 0 || E % G) return T * E == 0 ? 0 : (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sam_group_sum_grad_k, dim3(stream_grid(T * E, 256)), dim3(256), 0, st, g, dx, T, E, G);
  return (int)hipGetLastError();
}

HETU_API int hetu_sam_max(const float* x, const int64_t* grp, const int64_t* tk, float* y, int64_t T, int E, int n,
                          hipStream_t st) {
  if (T * E == 0) return 0;
  hipLaunchKernelGGL(sam_max_k, dim3(stream_grid(T * E, 256)), dim3(256), 0, st, x, grp, tk, y, T, E, n);
  return (int)hipGetLastError();
}

HETU_API int hetu_sam_max_grad(const float* g, const float* x, const int64_t* grp, const int64_t* tk, float* dx,
                               int64_t T, int E, int n, hipStream_t st) {
  if (T == 0) return 0;
  hipLaunchKernelGGL(sam_max_grad_k, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, st, g, x, grp, tk, dx, T, E, n);
  return (int)hipGetLastError();
}

// n (the group width) <= 64 * 64 columns, k <= n
HETU_API int hetu_group_topk_idx(const float* x, const int64_t* grp, int64_t* out, int64_t T, int E, int n, int k,
                                 hipStream_t st) {
  if (T == 0) return 0;
  if (n > 64 * 64 || k > n) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(group_topk_k, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, st, x, grp, out, T, E, n, k);
  return (int)hipGetLastError();
}

HETU_API int hetu_instance_norm2d(const void* x, void* y, float* mean, float* rstd, int N, int C, int64_t HW,
                                  int64_t sN, int64_t sC, int64_t sP, float eps, int bf, hipStream_t st) {
  if ((int64_t)N * C == 0) return 0;
  const dim3 g((unsigned)((int64_t)N * C));
  if (bf) hipLaunchKernelGGL(inorm_fwd_k<bf16>, g, dim3(256), 0, st, (const bf16*)x, (bf16*)y, mean, rstd, C, HW, sN, sC, sP, eps);
  else hipLaunchKernelGGL(inorm_fwd_k<float>, g, dim3(256), 0, st, (const float*)x, (float*)y, mean, rstd, C, HW, sN, sC, sP, eps);
  return (int)hipGetLastError();
}

HETU_API int hetu_instance_norm2d_grad(const void* g, const void* x, const float* mean, const float* rstd, void* dx,
                                       int N, int C, int64_t HW, int64_t sN, int64_t sC, int64_t sP, int bf,
                                       hipStream_t st) {
  if ((int64_t)N * C == 0) return 0;
  const dim3 gr((unsigned)((int64_t)N * C));
  if (bf) hipLaunchKernelGGL(inorm_bwd_k<bf16>, gr, dim3(256), 0, st, (const bf16*)g, (const bf16*)x, mean, rstd, (bf16*)dx, C, HW, sN, sC, sP);
  else hipLaunchKernelGGL(inorm_bwd_k<float>, gr, dim3(256), 0, st, (const float*)g, (const float*)x, mean, rstd, (float*)dx, C, HW, sN, sC, sP);
  return (int)hipGetLastError();
}

HETU_API int hetu_bicubic(const float* x, float* y, int64_t NC, int H, int W, int OH, int OW, float sh, float sw,
                          int align, hipStream_t st) {
  if (NC * OH * OW == 0) return 0;
  hipLaunchKernelGGL(bicubic_fwd_k, dim3(stream_grid(NC * OH * OW, 256)), dim3(256), 0, st, x, y, NC, H, W, OH, OW, sh,
                     sw, align);
  return (int)hipGetLastError();
}

HETU_API int hetu_bicubic_grad(const float* g, float* dx, int64_t NC, int H, int W, int OH, int OW, float sh, float sw,
                               int align, hipStream_t st) {
  if (NC * OH * OW == 0) return 0;
  hipLaunchKernelGGL(bicubic_bwd_k, dim3(stream_grid(NC * OH * OW, 256)), dim3(256), 0, st, g, dx, NC, H, W, OH, OW,
                     sh, sw, align);
  return (int)hipGetLastError();
}
