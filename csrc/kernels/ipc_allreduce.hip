// One-shot small-message all-reduce over IPC-mapped peer buffers (last
// bullet): for loss scalars, gate histograms and bench max-reduces, a single kernel per
// rank replaces an RCCL ring (whose per-call latency is several microseconds of protocol
// for a few hundred bytes).  Every rank owns one fine-grained device slab
//
//     [ data parity 0 : cap floats ][ data parity 1 : cap floats ][ flags : 64 x u32 ]
//
// exported with hipIpcGetMemHandle and opened by every peer.  Call e (host epoch, from 1):
//   1. copy the input into the own slab's data[e & 1];
//   2. release: system-scope fence, then write e into flags[rank] of EVERY peer's slab
//      (plain vector stores through the mapped pointers);
//   3. acquire: one lane spins on the own slab's flags[j] >= e for all j, with an
//      iteration cap (on expiry it records an error word and the call returns garbage
//      instead of hanging the GPU);
//   4. every thread sums data[e & 1][i] over all ranks' slabs (xGMI peer reads).
// Reuse: rank r rewrites parity p only at call e + 2, after every peer has signalled e + 1,
// which each peer does only after finishing call e -- so two parities suffice.
#include "common.h"
#include <string.h>

namespace hetu {
namespace ipcar {

constexpr int kMaxRanks = 16;
constexpr int kFlagWords = 64;

struct Peers {
  float* data[kMaxRanks];           // slab base of each rank (own one included)
};

__device__ __forceinline__ uint32_t load_acquire_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_release_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// op: 0 sum, 1 max.  One workgroup (the payloads are small; the latency is the flag trip).
__global__ void __launch_bounds__(256) oneshot_k(const float* __restrict__ x, float* __restrict__ out, int n,
                                                 int cap, uint32_t epoch, int rank, int nranks, Peers peers,
                                                 int op, uint32_t* err, int spin_cap) {
  const int par = (int)(epoch & 1u);
  float* mine = peers.data[rank] + (size_t)par * cap;
  for (int i = threadIdx.x; i < n; i += blockDim.x) mine[i] = x[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) {
    uint32_t* fl = reinterpret_cast<uint32_t*>(peers.data[threadIdx.x] + 2 * (size_t)cap);
    store_release_sys(fl + rank, epoch);
  }
  if (threadIdx.x == 0) {
    const uint32_t* fl = reinterpret_cast<const uint32_t*>(peers.data[rank] + 2 * (size_t)cap);
    int spins = 0;
    for (int j = 0; j < nranks; ++j) {
      while (load_acquire_sys(fl + j) < epoch) {
        if (++spins > spin_cap) {
          err[0] = epoch;               // timed out: report, do not hang
          j = nranks;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float acc = peers.data[0][(size_t)par * cap + i];
    for (int j = 1; j < nranks; ++j) {
      const float v = peers.data[j][(size_t)par * cap + i];
      acc = op == 1 ? fmaxf(acc, v) : acc + v;
    }
    out[i] = acc;
  }
}

}  // namespace ipcar
}  // namespace hetu

using namespace hetu;
using namespace hetu::ipcar;

// slab bytes for a capacity of `cap` floats per parity
HETU_API int64_t hetu_ipcar_slab_bytes(int cap) { return (int64_t)(2 * (int64_t)cap) * 4 + kFlagWords * 4; }

// fine-grained (coherent across processes / devices) slab, zeroed; handle: 64 bytes out
// (fine-grained first; an allocator that cannot export it gets a coarse-grained slab, which
// the system-scope release / acquire pair above keeps coherent at the flag handshake)
HETU_API int hetu_ipcar_alloc(int cap, void** slab, void* handle) {
  const size_t bytes = (size_t)hetu_ipcar_slab_bytes(cap);
  hipIpcMemHandle_t h;
  hipError_t e = hipExtMallocWithFlags(slab, bytes, hipDeviceMallocFinegrained);
  if (e == hipSuccess) {
    e = hipIpcGetMemHandle(&h, *slab);
    if (e != hipSuccess) {
      (void)hipFree(*slab);
      *slab = nullptr;
    }
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipMalloc(slab, bytes);
    if (e != hipSuccess) return (int)e;
    e = hipIpcGetMemHandle(&h, *slab);
    if (e != hipSuccess) return (int)e;
  }
  e = hipMemset(*slab, 0, bytes);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  memcpy(handle, &h, sizeof(h) < 64 ? sizeof(h) : 64);
  return 0;
}

HETU_API int hetu_ipcar_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

HETU_API int hetu_ipcar_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

HETU_API int hetu_ipcar_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }
HETU_API int hetu_ipcar_free(void* slab) { return (int)hipFree(slab); }

// ptrs: nranks slab pointers (own included); err: a device u32 (0 = ok, else the epoch
// that timed out)
HETU_API int hetu_ipcar_allreduce(const float* x, float* out, int n, int cap, uint32_t epoch, int rank, int nranks,
                                  void* const* ptrs, int op, uint32_t* err, int spin_cap, hipStream_t st) {
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || n < 0 || n > cap || epoch == 0)
    return (int)hipErrorInvalidValue;
  Peers p;
  for (int j = 0; j < kMaxRanks; ++j) p.data[j] = j < nranks ? (float*)ptrs[j] : nullptr;
  hipLaunchKernelGGL(oneshot_k, dim3(1), dim3(256), 0, st, x, out, n, cap, epoch, rank, nranks, p, op, err,
                     spin_cap);
  return (int)hipGetLastError();
}
