// Transposing LDS fragment reads that do not drain the operand prefetch.
//
// __builtin_amdgcn_ds_read_tr16_b64 carries no alias information, so the compiler's
// waitcnt pass puts an `s_waitcnt vmcnt(0)` in front of it whenever a global_load_lds /
// buffer_load ... lds is in flight: every MN-major fragment read then waits for the NEXT
// K-tile's DMA, and a double-buffered K loop degenerates into load-then-compute.  The
// inline-asm form below is invisible to that pass.  Its result is NOT tracked by the
// compiler's lgkmcnt bookkeeping either: every consumer calls frag_wait() (an explicit
// lgkmcnt(0) followed by a sched_barrier, so no MFMA is hoisted above it) between the reads
// and the first use.
#pragma once
#include <stdint.h>

namespace hetu {

typedef short tr_v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ tr_v4s ds_tr16(const char* p) {
  tr_v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

__device__ __forceinline__ void frag_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace hetu
