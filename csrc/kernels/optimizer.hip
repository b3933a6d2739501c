// Multi-tensor fused optimizers over FLAT parameter/gradient/state buffers.
//
// The reference launches one kernel per parameter per step (src/ops/Optimizers.cu,
// optimizer.py:184-225) and computes LAMB norms through cuDNN reductions.  Here all
// trainable dense parameters of an OptimizerOp live in one contiguous fp32 buffer
// (params are views into it), gradients land in a matching flat buffer (which is
// also what the bucketed RCCL all-reduce operates on), so one launch updates every
// parameter.  Optionally the kernel also emits the bf16 compute copy of the
// weights in the same pass (mixed precision: fp32 master, bf16 MFMA operands).
//
// Update rules match the reference kernels exactly (Optimizers.cu:3-284):
//   SGD       p -= lr*g
//   Momentum  v = mu*v - lr*g ; p += v
//   Nesterov  t = lr*g ; v = mu*(v - t) ; p += v - t
//   AdaGrad   a += g^2 ; p -= lr*g/(sqrt(a)+eps)
//   Adam      m,v EMA ; p -= lr*mhat/(sqrt(vhat)+eps)
//   AdamW     p -= lr*(mhat/(sqrt(vhat)+eps) + wd*p)
//   LAMB      u = mhat/(sqrt(vhat)+eps) ; p -= lr*(|p|/|u|)*(u + wd*p)   (per tensor)
// with g = gscale*grad + l2reg*p  (AddL2Regularization folded in).
#include "common.h"
#include <stdlib.h>

namespace hetu {

struct OptArgs {
  float lr, l2, mu, beta1, beta2, beta1t, beta2t, eps, wd, gscale;
  // optional device scalars {lr, beta1t, beta2t, gscale}: when set they override the
  // by-value ones, so a captured hipGraph sees per-step values (LR schedules,
  // Adam bias correction) without re-capture
  const float* dyn;
};

enum { OPT_SGD = 0, OPT_MOMENTUM = 1, OPT_NESTEROV = 2, OPT_ADAGRAD = 3, OPT_ADAM = 4,
       OPT_ADAMW = 5, OPT_LAMB = 6 };

// the update rule on 4 consecutive elements (cnt <= 4 valid)
template <int MODE>
__device__ __forceinline__ void opt_rule4(float (&pv)[4], float (&gv)[4], float (&x1)[4], float (&x2)[4], int cnt,
                                          const OptArgs& a, float lr, float b1t, float b2t, float gsc) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= cnt) break;
    float gr = gv[k] * gsc + a.l2 * pv[k];
    if (MODE == OPT_SGD) {
      pv[k] -= lr * gr;
    } else if (MODE == OPT_MOMENTUM) {
      x1[k] = a.mu * x1[k] - lr * gr;
      pv[k] += x1[k];
    } else if (MODE == OPT_NESTEROV) {
      float t = lr * gr;
      x1[k] = a.mu * (x1[k] - t);
      pv[k] += x1[k] - t;
    } else if (MODE == OPT_ADAGRAD) {
      x1[k] += gr * gr;
      pv[k] -= lr * gr / (sqrtf(x1[k]) + a.eps);
    } else {
      x1[k] = a.beta1 * x1[k] + (1.f - a.beta1) * gr;
      x2[k] = a.beta2 * x2[k] + (1.f - a.beta2) * gr * gr;
      float mh = x1[k] / (1.f - b1t), vh = x2[k] / (1.f - b2t);
      float u = mh / (sqrtf(vh) + a.eps);
      if (MODE == OPT_ADAM) pv[k] -= lr * u;
      else if (MODE == OPT_ADAMW) pv[k] -= lr * (u + a.wd * pv[k]);
      else gv[k] = u;  // LAMB phase 1: update kept in the grad buffer
    }
  }
}

typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef unsigned nt_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void ld4_nt(const float* p, float (&v)[4]) {
  const nt_f4 t = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
__device__ __forceinline__ void st4_nt(float* p, const float (&v)[4]) {
  const nt_f4 t = {v[0], v[1], v[2], v[3]};
  __builtin_nontemporal_store(t, reinterpret_cast<nt_f4*>(p));
}
__device__ __forceinline__ void st_bf16x4_nt(unsigned short* p, const float (&v)[4]) {
  const nt_u2 w = {(unsigned)f_to_bf16_bits(v[0]) | ((unsigned)f_to_bf16_bits(v[1]) << 16),
                   (unsigned)f_to_bf16_bits(v[2]) | ((unsigned)f_to_bf16_bits(v[3]) << 16)};
  __builtin_nontemporal_store(w, reinterpret_cast<nt_u2*>(p));
}

// Aligned form (16-byte aligned buffers; the n % 4 tail by one thread): two float4 groups per thread and
// iteration with all their loads issued before the math, non-temporal loads and stores
// (every byte is touched once per step: no reuse to keep in L2 / MALL).
template <int MODE, bool SHADOW>
__global__ void __launch_bounds__(256) opt_flat2_k(float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ s1, float* __restrict__ s2,
                                                    unsigned short* __restrict__ shadow, int64_t n, OptArgs a) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float lr = a.lr, b1t = a.beta1t, b2t = a.beta2t, gsc = a.gscale;
  if (a.dyn) { lr = a.dyn[0]; b1t = a.dyn[1]; b2t = a.dyn[2]; gsc = a.dyn[3]; }
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    float pv[2][4], gv[2][4], x1[2][4], x2[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t b = (i + u * stride) * 4;
      ld4_nt(p + b, pv[u]);
      ld4_nt(g + b, gv[u]);
      if (MODE != OPT_SGD) ld4_nt(s1 + b, x1[u]);
      if (MODE >= OPT_ADAM) ld4_nt(s2 + b, x2[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t b = (i + u * stride) * 4;
      opt_rule4<MODE>(pv[u], gv[u], x1[u], x2[u], 4, a, lr, b1t, b2t, gsc);
      if (MODE != OPT_LAMB) st4_nt(p + b, pv[u]);
      else st4_nt(g + b, gv[u]);
      if (MODE != OPT_SGD) st4_nt(s1 + b, x1[u]);
      if (MODE >= OPT_ADAM) st4_nt(s2 + b, x2[u]);
      if (SHADOW && MODE != OPT_LAMB) st_bf16x4_nt(shadow + b, pv[u]);
    }
  }
  for (; i < n4; i += stride) {
    const int64_t b = i * 4;
    float pv[4], gv[4], x1[4], x2[4];
    ld4_nt(p + b, pv);
    ld4_nt(g + b, gv);
    if (MODE != OPT_SGD) ld4_nt(s1 + b, x1);
    if (MODE >= OPT_ADAM) ld4_nt(s2 + b, x2);
    opt_rule4<MODE>(pv, gv, x1, x2, 4, a, lr, b1t, b2t, gsc);
    if (MODE != OPT_LAMB) st4_nt(p + b, pv);
    else st4_nt(g + b, gv);
    if (MODE != OPT_SGD) st4_nt(s1 + b, x1);
    if (MODE >= OPT_ADAM) st4_nt(s2 + b, x2);
    if (SHADOW && MODE != OPT_LAMB) st_bf16x4_nt(shadow + b, pv);
  }
  // the n % 4 tail elements (the flat buffer ends with the last parameter's numel)
  const int cnt = (int)(n - n4 * 4);
  if (cnt > 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t b = n4 * 4;
    float pv[4] = {0.f, 0.f, 0.f, 0.f}, gv[4] = {0.f, 0.f, 0.f, 0.f}, x1[4] = {0.f, 0.f, 0.f, 0.f},
          x2[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < cnt; ++k) {
      pv[k] = p[b + k]; gv[k] = g[b + k];
      if (MODE != OPT_SGD) x1[k] = s1[b + k];
      if (MODE >= OPT_ADAM) x2[k] = s2[b + k];
    }
    opt_rule4<MODE>(pv, gv, x1, x2, cnt, a, lr, b1t, b2t, gsc);
    for (int k = 0; k < cnt; ++k) {
      if (MODE != OPT_LAMB) p[b + k] = pv[k]; else g[b + k] = gv[k];
      if (MODE != OPT_SGD) s1[b + k] = x1[k];
      if (MODE >= OPT_ADAM) s2[b + k] = x2[k];
      if (SHADOW && MODE != OPT_LAMB) shadow[b + k] = f_to_bf16_bits(pv[k]);
    }
  }
}

template <int MODE, bool SHADOW>
__global__ void __launch_bounds__(256) opt_flat_k(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ s1, float* __restrict__ s2,
                                                   unsigned short* __restrict__ shadow, int64_t n,
                                                   OptArgs a) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4 + (n & 3 ? 1 : 0);
       i += stride) {
    const int64_t base = i * 4;
    const int cnt = (base + 4 <= n) ? 4 : (int)(n - base);
    float pv[4], gv[4], x1[4], x2[4];
    if (cnt == 4) {
      float4 t = *reinterpret_cast<float4*>(p + base);
      pv[0] = t.x; pv[1] = t.y; pv[2] = t.z; pv[3] = t.w;
      t = *reinterpret_cast<float4*>(g + base);
      gv[0] = t.x; gv[1] = t.y; gv[2] = t.z; gv[3] = t.w;
      if (MODE != OPT_SGD) {
        t = *reinterpret_cast<float4*>(s1 + base);
        x1[0] = t.x; x1[1] = t.y; x1[2] = t.z; x1[3] = t.w;
      }
      if (MODE >= OPT_ADAM) {
        t = *reinterpret_cast<float4*>(s2 + base);
        x2[0] = t.x; x2[1] = t.y; x2[2] = t.z; x2[3] = t.w;
      }
    } else {
      for (int k = 0; k < cnt; ++k) {
        pv[k] = p[base + k]; gv[k] = g[base + k];
        if (MODE != OPT_SGD) x1[k] = s1[base + k];
        if (MODE >= OPT_ADAM) x2[k] = s2[base + k];
      }
    }
    float lr = a.lr, b1t = a.beta1t, b2t = a.beta2t, gsc = a.gscale;
    if (a.dyn) { lr = a.dyn[0]; b1t = a.dyn[1]; b2t = a.dyn[2]; gsc = a.dyn[3]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= cnt) break;
      float gr = gv[k] * gsc + a.l2 * pv[k];
      if (MODE == OPT_SGD) {
        pv[k] -= lr * gr;
      } else if (MODE == OPT_MOMENTUM) {
        x1[k] = a.mu * x1[k] - lr * gr;
        pv[k] += x1[k];
      } else if (MODE == OPT_NESTEROV) {
        float t = lr * gr;
        x1[k] = a.mu * (x1[k] - t);
        pv[k] += x1[k] - t;
      } else if (MODE == OPT_ADAGRAD) {
        x1[k] += gr * gr;
        pv[k] -= lr * gr / (sqrtf(x1[k]) + a.eps);
      } else {
        x1[k] = a.beta1 * x1[k] + (1.f - a.beta1) * gr;
        x2[k] = a.beta2 * x2[k] + (1.f - a.beta2) * gr * gr;
        float mh = x1[k] / (1.f - b1t), vh = x2[k] / (1.f - b2t);
        float u = mh / (sqrtf(vh) + a.eps);
        if (MODE == OPT_ADAM) pv[k] -= lr * u;
        else if (MODE == OPT_ADAMW) pv[k] -= lr * (u + a.wd * pv[k]);
        else gv[k] = u;  // LAMB phase 1: update kept in the grad buffer
      }
    }
    if (cnt == 4) {
      if (MODE != OPT_LAMB) *reinterpret_cast<float4*>(p + base) = make_float4(pv[0], pv[1], pv[2], pv[3]);
      else *reinterpret_cast<float4*>(g + base) = make_float4(gv[0], gv[1], gv[2], gv[3]);
      if (MODE != OPT_SGD) *reinterpret_cast<float4*>(s1 + base) = make_float4(x1[0], x1[1], x1[2], x1[3]);
      if (MODE >= OPT_ADAM) *reinterpret_cast<float4*>(s2 + base) = make_float4(x2[0], x2[1], x2[2], x2[3]);
      if (SHADOW && MODE != OPT_LAMB) {
        uint2 w;
        w.x = (unsigned)f_to_bf16_bits(pv[0]) | ((unsigned)f_to_bf16_bits(pv[1]) << 16);
        w.y = (unsigned)f_to_bf16_bits(pv[2]) | ((unsigned)f_to_bf16_bits(pv[3]) << 16);
        *reinterpret_cast<uint2*>(shadow + base) = w;
      }
    } else {
      for (int k = 0; k < cnt; ++k) {
        if (MODE != OPT_LAMB) p[base + k] = pv[k]; else g[base + k] = gv[k];
        if (MODE != OPT_SGD) s1[base + k] = x1[k];
        if (MODE >= OPT_ADAM) s2[base + k] = x2[k];
        if (SHADOW && MODE != OPT_LAMB) shadow[base + k] = f_to_bf16_bits(pv[k]);
      }
    }
  }
}

__device__ __forceinline__ int find_seg(const int64_t* __restrict__ off, int nseg, int64_t i) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// per-segment squared norms of p and u (u lives in g): norms[2*seg + {0,1}]
__global__ void __launch_bounds__(256) seg_norms_k(const float* __restrict__ p, const float* __restrict__ u,
                                                    const int64_t* __restrict__ off, int nseg,
                                                    int64_t n, float* __restrict__ norms) {
  // each block handles a contiguous range; flush partial sums at segment edges
  __shared__ float sh[8];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per;
  int64_t b1 = b0 + per;
  if (b1 > n) b1 = n;
  if (b0 >= b1) return;
  int seg = find_seg(off, nseg, b0);
  int64_t cur = b0;
  while (cur < b1) {
    int64_t end = off[seg + 1] < b1 ? off[seg + 1] : b1;
    float sp = 0.f, su = 0.f;
    for (int64_t i = cur + threadIdx.x; i < end; i += blockDim.x) {
      float a = p[i], b = u[i];
      sp += a * a;
      su += b * b;
    }
    sp = block_sum<256>(sp, sh);
    su = block_sum<256>(su, sh);
    if (threadIdx.x == 0) {
      atomicAdd(norms + 2 * seg, sp);
      atomicAdd(norms + 2 * seg + 1, su);
    }
    cur = end;
    ++seg;
  }
}

template <bool SHADOW>
__global__ void __launch_bounds__(256) lamb_apply_k(float* __restrict__ p, const float* __restrict__ u,
                                                     const int64_t* __restrict__ off, int nseg,
                                                     const float* __restrict__ norms,
                                                     unsigned short* __restrict__ shadow, int64_t n,
                                                     float lr, float wd, const float* __restrict__ dyn) {
  if (dyn) lr = dyn[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int s = find_seg(off, nseg, i);
    float np_ = sqrtf(norms[2 * s]), nu = sqrtf(norms[2 * s + 1]);
    float ratio = (np_ > 0.f && nu > 0.f) ? np_ / nu : 1.f;
    float pv = p[i];
    pv -= lr * ratio * (u[i] + wd * pv);
    p[i] = pv;
    if (SHADOW) shadow[i] = f_to_bf16_bits(pv);
  }
}

__global__ void f32_to_bf16_k(const float* __restrict__ x, unsigned short* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f_to_bf16_bits(x[i]);
}

}  // namespace hetu

using namespace hetu;

template <int MODE>
static void launch_opt(float* p, float* g, float* s1, float* s2, unsigned short* sh, int64_t n,
                       const OptArgs& a, hipStream_t st) {
  static const bool v2 = [] {
    const char* e = getenv("HETU_OPT_V2");
    return e == nullptr || e[0] != '0';
  }();
  const uintptr_t al = (uintptr_t)p | (uintptr_t)g | (uintptr_t)s1 | (uintptr_t)s2 | (uintptr_t)sh;
  if (v2 && n >= 4 && (al & 15) == 0 && (!sh || ((uintptr_t)sh & 7) == 0)) {
    const int grid = stream_grid(n / 4, 256, 4);
    if (sh) hipLaunchKernelGGL((opt_flat2_k<MODE, true>), dim3(grid), dim3(256), 0, st, p, g, s1, s2, sh, n, a);
    else hipLaunchKernelGGL((opt_flat2_k<MODE, false>), dim3(grid), dim3(256), 0, st, p, g, s1, s2, sh, n, a);
    return;
  }
  int grid = stream_grid((n + 3) / 4, 256, 2);
  if (sh) hipLaunchKernelGGL((opt_flat_k<MODE, true>), dim3(grid), dim3(256), 0, st, p, g, s1, s2, sh, n, a);
  else hipLaunchKernelGGL((opt_flat_k<MODE, false>), dim3(grid), dim3(256), 0, st, p, g, s1, s2, sh, n, a);
}

// p,g,s1,s2: fp32 flat buffers (16-byte aligned); shadow: optional bf16 copy of p.
// For LAMB pass seg_off (device int64[nseg+1]) and norms_ws (device fp32[2*nseg]).
HETU_API int hetu_optimizer_flat(int mode, float* p, float* g, float* s1, float* s2, void* shadow,
                                 int64_t n, float lr, float l2, float mu, float beta1, float beta2,
                                 float beta1t, float beta2t, float eps, float wd, float gscale,
                                 const int64_t* seg_off, int nseg, float* norms_ws,
                                 const float* dyn, hipStream_t st) {
  OptArgs a{lr, l2, mu, beta1, beta2, beta1t, beta2t, eps, wd, gscale};
  a.dyn = dyn;
  unsigned short* sh = (unsigned short*)shadow;
  switch (mode) {
    case OPT_SGD: launch_opt<OPT_SGD>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_MOMENTUM: launch_opt<OPT_MOMENTUM>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_NESTEROV: launch_opt<OPT_NESTEROV>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_ADAGRAD: launch_opt<OPT_ADAGRAD>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_ADAM: launch_opt<OPT_ADAM>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_ADAMW: launch_opt<OPT_ADAMW>(p, g, s1, s2, sh, n, a, st); break;
    case OPT_LAMB: {
      launch_opt<OPT_LAMB>(p, g, s1, s2, nullptr, n, a, st);
      (void)hipMemsetAsync(norms_ws, 0, sizeof(float) * 2 * nseg, st);
      int blocks = (int)((n + 65535) / 65536);
      if (blocks < 1) blocks = 1;
      if (blocks > 2048) blocks = 2048;
      hipLaunchKernelGGL(seg_norms_k, dim3(blocks), dim3(256), 0, st, p, g, seg_off, nseg, n, norms_ws);
      int grid = stream_grid(n, 256, 4);
      if (sh) hipLaunchKernelGGL(lamb_apply_k<true>, dim3(grid), dim3(256), 0, st, p, g, seg_off, nseg, norms_ws, sh, n, lr, wd, dyn);
      else hipLaunchKernelGGL(lamb_apply_k<false>, dim3(grid), dim3(256), 0, st, p, g, seg_off, nseg, norms_ws, sh, n, lr, wd, dyn);
      break;
    }
    default: return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_f32_to_bf16(const float* x, void* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(f32_to_bf16_k, dim3(stream_grid(n, 256, 4)), dim3(256), 0, st, x,
                     (unsigned short*)y, n);
  HETU_LAUNCH_CHECK();
  return 0;
}
