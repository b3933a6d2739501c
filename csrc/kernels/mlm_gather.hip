// Masked-LM head over the masked positions only (BERT pretraining).
//
// The reference scores every token against the 30 522-word vocabulary and ignores the
// unmasked ones in the loss (examples/nlp/bert/hetu_bert.py: softmaxcrossentropy_sparse_op
// with ignored_index=-1 over [B*S, V]); those rows contribute neither loss nor gradient.
// Here the rows with a label are compacted first -- C slots per sequence, the original
// BERT's max_predictions_per_seq -- so the head's three GEMMs and its softmax-CE run over
// B*C rows instead of B*S (~1/6 at 15 % masking).
//
//   hetu_masked_positions: one wave per sequence, a ballot prefix count in position order;
//     slot k of sequence b holds the k-th labelled row (or -1); a sequence with more than C
//     labels sets the overflow word (the host reads it one step late and raises).
//   hetu_take_rows / hetu_put_rows: row gather into the slots (fill for empty slots) and
//     its adjoint (the slots' rows written back, every other row zero).
#include "common.h"

namespace hetu {

// labels: int64, int32 or fp32 (mixed-precision feeds keep class indices as fp32)
template <typename L>
__global__ void __launch_bounds__(64) masked_positions_k(const L* __restrict__ labels, int S, int C,
                                                         int64_t* __restrict__ idx, int* __restrict__ overflow) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const L* lab = labels + (int64_t)b * S;
  int64_t* out = idx + (int64_t)b * C;
  for (int k = lane; k < C; k += 64) out[k] = -1;
  __syncthreads();
  int base = 0;
  for (int s0 = 0; s0 < S; s0 += 64) {
    const int s = s0 + lane;
    const bool m = s < S && lab[s] != (L)-1;
    const uint64_t bal = __ballot(m);
    const int k = base + __popcll(bal & ((1ull << lane) - 1ull));
    if (m && k < C) out[k] = (int64_t)b * S + s;
    base += __popcll(bal);
  }
  if (lane == 0 && base > C) *overflow = base;   // any non-zero value flags an overflow
}

// out[j] = x[idx[j]] (a row of W 16-byte words), or the fill word for idx[j] < 0
__global__ void __launch_bounds__(256) take_rows16_k(const uint4* __restrict__ x, const int64_t* __restrict__ idx,
                                                     int64_t n, int W, uint4 fill, uint4* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * W) return;
  const int64_t j = t / W, w = t - j * W;
  const int64_t r = idx[j];
  out[t] = r >= 0 ? x[r * W + w] : fill;
}

// element-wise form (rows not a multiple of 16 bytes; labels: 8-byte elements)
template <typename T>
__global__ void __launch_bounds__(256) take_rows_k(const T* __restrict__ x, const int64_t* __restrict__ idx,
                                                   int64_t n, int H, T fill, T* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * H) return;
  const int64_t j = t / H, h = t - j * H;
  const int64_t r = idx[j];
  out[t] = r >= 0 ? x[r * H + h] : fill;
}

// out[idx[j]] = g[j] (rows of W 16-byte words); out zero-filled beforehand
__global__ void __launch_bounds__(256) put_rows16_k(const uint4* __restrict__ g, const int64_t* __restrict__ idx,
                                                    int64_t n, int W, uint4* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * W) return;
  const int64_t j = t / W, w = t - j * W;
  const int64_t r = idx[j];
  if (r >= 0) out[r * W + w] = g[t];
}

template <typename T>
__global__ void __launch_bounds__(256) put_rows_k(const T* __restrict__ g, const int64_t* __restrict__ idx,
                                                  int64_t n, int H, T* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * H) return;
  const int64_t j = t / H, h = t - j * H;
  const int64_t r = idx[j];
  if (r >= 0) out[r * H + h] = g[t];
}

}  // namespace hetu

using namespace hetu;

// kind: 0 int64, 1 int32, 2 fp32 labels
HETU_API int hetu_masked_positions(const void* labels, int kind, int B, int S, int C, int64_t* idx, int* overflow,
                                   hipStream_t st) {
  if (B <= 0 || S <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (kind == 0)
    hipLaunchKernelGGL((masked_positions_k<int64_t>), dim3((unsigned)B), dim3(64), 0, st, (const int64_t*)labels, S,
                       C, idx, overflow);
  else if (kind == 1)
    hipLaunchKernelGGL((masked_positions_k<int>), dim3((unsigned)B), dim3(64), 0, st, (const int*)labels, S, C, idx,
                       overflow);
  else if (kind == 2)
    hipLaunchKernelGGL((masked_positions_k<float>), dim3((unsigned)B), dim3(64), 0, st, (const float*)labels, S, C,
                       idx, overflow);
  else
    return (int)hipErrorInvalidValue;
  HETU_LAUNCH_CHECK();
  return 0;
}

// esize: bytes per element (2 bf16 / 4 fp32 or int32 / 8 int64); fill_neg1: 0 -> fill 0,
// 1 -> integer -1 (int32 / int64 labels), 2 -> -1.0f (fp32 labels: mixed-precision feeds
// keep class indices as fp32)
HETU_API int hetu_take_rows(const void* x, const int64_t* idx, int64_t n, int H, int esize, int fill_neg1,
                            void* out, hipStream_t st) {
  if (n <= 0 || H <= 0) return 0;
  const int64_t rowb = (int64_t)H * esize;
  if (rowb % 16 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 && !fill_neg1) {
    const int W = (int)(rowb / 16);
    const int64_t tot = n * W;
    hipLaunchKernelGGL(take_rows16_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const uint4*)x, idx, n,
                       W, make_uint4(0, 0, 0, 0), (uint4*)out);
  } else {
    const int64_t tot = n * H;
    const dim3 g((unsigned)((tot + 255) / 256));
    if (esize == 8)
      hipLaunchKernelGGL((take_rows_k<int64_t>), g, dim3(256), 0, st, (const int64_t*)x, idx, n, H,
                         (int64_t)(fill_neg1 ? -1 : 0), (int64_t*)out);
    else if (esize == 4 && fill_neg1 == 1)
      hipLaunchKernelGGL((take_rows_k<int>), g, dim3(256), 0, st, (const int*)x, idx, n, H, -1, (int*)out);
    else if (esize == 4)
      hipLaunchKernelGGL((take_rows_k<float>), g, dim3(256), 0, st, (const float*)x, idx, n, H,
                         fill_neg1 == 2 ? -1.f : 0.f, (float*)out);
    else if (esize == 2)
      hipLaunchKernelGGL((take_rows_k<unsigned short>), g, dim3(256), 0, st, (const unsigned short*)x, idx, n, H,
                         (unsigned short)0, (unsigned short*)out);
    else
      return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}

HETU_API int hetu_put_rows(const void* g, const int64_t* idx, int64_t n, int H, int esize, void* out,
                           hipStream_t st) {
  if (n <= 0 || H <= 0) return 0;
  const int64_t rowb = (int64_t)H * esize;
  if (rowb % 16 == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    const int W = (int)(rowb / 16);
    const int64_t tot = n * W;
    hipLaunchKernelGGL(put_rows16_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const uint4*)g, idx, n,
                       W, (uint4*)out);
  } else {
    const int64_t tot = n * H;
    const dim3 gr((unsigned)((tot + 255) / 256));
    if (esize == 4)
      hipLaunchKernelGGL((put_rows_k<float>), gr, dim3(256), 0, st, (const float*)g, idx, n, H, (float*)out);
    else if (esize == 2)
      hipLaunchKernelGGL((put_rows_k<unsigned short>), gr, dim3(256), 0, st, (const unsigned short*)g, idx, n, H,
                         (unsigned short*)out);
    else
      return (int)hipErrorInvalidValue;
  }
  HETU_LAUNCH_CHECK();
  return 0;
}
