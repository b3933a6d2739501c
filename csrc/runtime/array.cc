// Framework-owned strided arrays (the reference's DLArray C runtime:
// src/common/dlarray.h:18-66 -- data, ctx, ndim, shape, stride -- and
// c_runtime_api.cc:93-142 DLArrayAlloc / Free / CopyFromTo).
//
// MI355X design: an array is a refcounted header {data, byte offset, device, dtype,
// ndim, shape, strides (elements)} over an allocation from the framework's own pools --
// the BFC HBM pool of the device (stream-ordered reuse), the pinned-host BFC pool
// (hipHostMalloc: async H2D / D2H) or plain host memory.  Views (reshape, transpose,
// slice, broadcast with stride 0) share the allocation.  Arrays export to DLPack, so
// torch (kernel wrappers, tests) sees them as non-owning tensors: the DLPack deleter
// drops a reference and the last reference returns the memory to the pool.  Allocation
// and release go through the same pools torch's pluggable-allocator hook uses, so a
// framework array and a torch tensor never contend for memory.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "bfc_allocator.h"

#define HETU_RT_API extern "C" __attribute__((visibility("default")))

// ---- DLPack ABI (dlpack.h v0.8 layout) -------------------------------------------------
extern "C" {
typedef struct { int32_t device_type; int32_t device_id; } DLDevice;
typedef struct { uint8_t code; uint8_t bits; uint16_t lanes; } DLDataType;
typedef struct {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
} DLTensor;
typedef struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct DLManagedTensor* self);
} DLManagedTensor;
}
enum { kDLCPU = 1, kDLCUDAHost = 3, kDLROCM = 10, kDLROCMHost = 11 };
enum { kDLInt = 0, kDLUInt = 1, kDLFloat = 2, kDLBfloat = 4 };

namespace hetu {

// dtype codes of the framework (ndarray.py DTYPE_CODES)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI32 = 3, kI64 = 4, kU8 = 5, kF64 = 6, kI8 = 7, kBool = 8 };
static int dtype_size(int dt) {
  switch (dt) {
    case kF32: case kI32: return 4;
    case kBF16: case kF16: return 2;
    case kI64: case kF64: return 8;
    default: return 1;
  }
}
static DLDataType to_dl(int dt) {
  switch (dt) {
    case kF32: return {kDLFloat, 32, 1};
    case kBF16: return {kDLBfloat, 16, 1};
    case kF16: return {kDLFloat, 16, 1};
    case kI32: return {kDLInt, 32, 1};
    case kI64: return {kDLInt, 64, 1};
    case kF64: return {kDLFloat, 64, 1};
    case kI8: return {kDLInt, 8, 1};
    case kBool: return {6 /* kDLBool */, 8, 1};
    default: return {kDLUInt, 8, 1};
  }
}

// memory kinds of an array's allocation
enum Mem : int { kDev = 0, kPinned = 1, kHostMem = 2, kBorrowed = 3 };
constexpr int kMaxDim = 8;

struct Array;
struct Alloc {                    // one allocation, shared by its views
  std::atomic<int> refs{1};
  void* ptr = nullptr;
  int64_t bytes = 0;
  int mem = kDev;
  int device = 0;
  BFCAllocator* pool = nullptr;
  hipStream_t stream = nullptr;   // device pool: the stream the memory is ordered on
  DLManagedTensor* borrowed = nullptr;   // kBorrowed: the producer's tensor, deleted last
};

struct Array {
  std::atomic<int> refs{1};
  Alloc* alloc = nullptr;
  int64_t offset = 0;             // bytes from alloc->ptr
  int dtype = kF32;
  int device_type = 1;            // 1 cpu, 2 gpu (DLContext encoding)
  int device_id = 0;
  int ndim = 0;
  int64_t shape[kMaxDim];
  int64_t strides[kMaxDim];       // elements
  DLManagedTensor dl;             // export record (one live export at a time per header)
};

static std::atomic<int64_t> g_live_arrays{0}, g_live_allocs{0}, g_created{0};

// pools: device memory through the pluggable-allocator entry points of bfc_allocator.cc
// (the device BFC pool, or the private graph-capture pool while a capture is active on
// the allocating stream) and one pinned-host pool
extern "C" void* hetu_torch_alloc(ssize_t size, int device, hipStream_t stream);
extern "C" void hetu_torch_free(void* ptr, ssize_t size, int device, hipStream_t stream);
static BFCAllocator* pinned_pool() {
  static BFCAllocator* p = nullptr;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (!p) p = new BFCAllocator(MemKind::kPinnedHost, 0, 0, (size_t)256 << 20);
  return p;
}

static void alloc_release(Alloc* a) {
  if (a->refs.fetch_sub(1) != 1) return;
  if (a->mem == kDev) {
    if (a->ptr) hetu_torch_free(a->ptr, (ssize_t)a->bytes, a->device, a->stream);
  } else if (a->mem == kPinned) {
    if (a->pool && a->ptr) a->pool->deallocate(a->ptr, a->stream);
  } else if (a->mem == kHostMem) {
    free(a->ptr);
  } else if (a->mem == kBorrowed && a->borrowed && a->borrowed->deleter) {
    a->borrowed->deleter(a->borrowed);
  }
  g_live_allocs.fetch_sub(1);
  delete a;
}

static void array_release(Array* x) {
  if (x->refs.fetch_sub(1) != 1) return;
  alloc_release(x->alloc);
  g_live_arrays.fetch_sub(1);
  delete x;
}

static Array* new_header(Alloc* a, int64_t offset, int dtype, int dev_type, int dev_id, int ndim,
                         const int64_t* shape, const int64_t* strides) {
  Array* x = new Array();
  x->alloc = a;
  x->offset = offset;
  x->dtype = dtype;
  x->device_type = dev_type;
  x->device_id = dev_id;
  x->ndim = ndim;
  int64_t st = 1;
  for (int d = ndim - 1; d >= 0; --d) {
    x->shape[d] = shape[d];
    x->strides[d] = strides ? strides[d] : st;
    st *= shape[d];
  }
  g_live_arrays.fetch_add(1);
  g_created.fetch_add(1);
  return x;
}

}  // namespace hetu

using namespace hetu;

// Allocate a contiguous (row-major) array.  device_type 2: HBM of device_id from the
// device BFC pool, ordered on `stream`; 1 + pinned: pinned host; 1: host memory.
HETU_RT_API int hetu_array_empty(int ndim, const int64_t* shape, int dtype, int device_type, int device_id,
                                 int pinned, void* stream, void** out) {
  if (ndim < 0 || ndim > kMaxDim) return 1;
  int64_t n = 1;
  for (int d = 0; d < ndim; ++d) {
    if (shape[d] < 0) return 1;
    n *= shape[d];
  }
  const int64_t bytes = n * dtype_size(dtype);
  Alloc* a = new Alloc();
  a->bytes = bytes;
  a->device = device_id;
  if (device_type == 2) {
    a->mem = kDev;
    a->stream = (hipStream_t)stream;
    a->ptr = hetu_torch_alloc((ssize_t)(bytes ? bytes : 1), device_id, a->stream);
  } else if (pinned) {
    a->mem = kPinned;
    a->pool = pinned_pool();
    a->ptr = a->pool->allocate((size_t)(bytes ? bytes : 1), nullptr);
  } else {
    a->mem = kHostMem;
    a->ptr = aligned_alloc(256, (size_t)((bytes + 255) / 256 * 256 + (bytes ? 0 : 256)));
  }
  if (!a->ptr) {
    delete a;
    return 2;   // out of memory
  }
  g_live_allocs.fetch_add(1);
  *out = new_header(a, 0, dtype, device_type, device_id, ndim, shape, nullptr);
  return 0;
}

// Zero-copy view of `src`: new shape / strides (elements) / extra byte offset over the same
// allocation (reshape, transpose, slice, broadcast_to with stride 0).  Bounds are checked
// against the allocation.
HETU_RT_API int hetu_array_view(void* src, int ndim, const int64_t* shape, const int64_t* strides,
                                int64_t byte_offset, void** out) {
  Array* s = (Array*)src;
  if (ndim < 0 || ndim > kMaxDim) return 1;
  const int es = dtype_size(s->dtype);
  int64_t lo = s->offset + byte_offset, hi = lo;
  for (int d = 0; d < ndim; ++d) {
    if (shape[d] == 0) { lo = hi = s->offset; break; }
    const int64_t span = (shape[d] - 1) * strides[d] * es;
    if (span < 0) lo += span; else hi += span;
  }
  if (lo < 0 || hi + es > s->alloc->bytes + (s->alloc->bytes == 0 ? es : 0)) return 3;   // out of bounds
  s->alloc->refs.fetch_add(1);
  *out = new_header(s->alloc, s->offset + byte_offset, s->dtype, s->device_type, s->device_id, ndim, shape,
                    strides);
  return 0;
}

HETU_RT_API void hetu_array_retain(void* a) { ((Array*)a)->refs.fetch_add(1); }
HETU_RT_API void hetu_array_release(void* a) {
  if (a) array_release((Array*)a);
}

// header fields: data pointer (with offset), ndim, dtype, device type / id; shape and
// strides copied into caller buffers of kMaxDim entries
HETU_RT_API int hetu_array_info(void* a, void** data, int* ndim, int64_t* shape, int64_t* strides, int* dtype,
                                int* device_type, int* device_id) {
  Array* x = (Array*)a;
  *data = (char*)x->alloc->ptr + x->offset;
  *ndim = x->ndim;
  for (int d = 0; d < x->ndim; ++d) {
    shape[d] = x->shape[d];
    strides[d] = x->strides[d];
  }
  *dtype = x->dtype;
  *device_type = x->device_type;
  *device_id = x->device_id;
  return 0;
}

static bool contiguous(const Array* x) {
  int64_t st = 1;
  for (int d = x->ndim - 1; d >= 0; --d) {
    if (x->shape[d] != 1 && x->strides[d] != st) return false;
    st *= x->shape[d];
  }
  return true;
}

// dst = src (same shape and dtype; reference DLArrayCopyFromTo).  Contiguous arrays move
// with one async copy on `stream` (H2D / D2H / D2D / H2H by the two devices); a strided
// side must be 2-D-collapsible (rows of contiguous elements) and goes through
// hipMemcpy2DAsync.  Everything else is left to the device copy kernels (returns 4).
HETU_RT_API int hetu_array_copy(void* dst, void* src, void* stream) {
  Array* d = (Array*)dst;
  Array* s = (Array*)src;
  if (d->ndim != s->ndim || d->dtype != s->dtype) return 1;
  int64_t n = 1;
  for (int i = 0; i < d->ndim; ++i) {
    if (d->shape[i] != s->shape[i]) return 1;
    n *= d->shape[i];
  }
  if (n == 0) return 0;
  const int es = dtype_size(d->dtype);
  char* dp = (char*)d->alloc->ptr + d->offset;
  const char* sp = (const char*)s->alloc->ptr + s->offset;
  hipStream_t st = (hipStream_t)stream;
  const bool host = d->device_type == 1 && s->device_type == 1;   // host <-> host: no HIP (CPU-only runs)
  if (contiguous(d) && contiguous(s)) {
    if (host) {
      memcpy(dp, sp, (size_t)(n * es));
      return 0;
    }
    return (int)hipMemcpyAsync(dp, sp, (size_t)(n * es), hipMemcpyDefault, st);
  }
  // [rows][cols] with unit inner stride on both sides
  auto rows2 = [](const Array* x, int64_t& rows, int64_t& cols, int64_t& ld) -> bool {
    if (x->ndim == 0 || x->strides[x->ndim - 1] != 1) return false;
    cols = x->shape[x->ndim - 1];
    rows = 1;
    ld = x->ndim >= 2 ? x->strides[x->ndim - 2] : cols;
    int64_t expect = ld;
    for (int i = x->ndim - 2; i >= 0; --i) {
      if (x->shape[i] != 1 && x->strides[i] != expect) return false;
      expect *= x->shape[i];
      rows *= x->shape[i];
    }
    return true;
  };
  int64_t rd, cd, ldd, rs, cs, lds;
  if (rows2(d, rd, cd, ldd) && rows2(s, rs, cs, lds) && rd == rs && cd == cs) {
    if (host) {
      for (int64_t r = 0; r < rd; ++r) memcpy(dp + r * ldd * es, sp + r * lds * es, (size_t)(cd * es));
      return 0;
    }
    return (int)hipMemcpy2DAsync(dp, (size_t)(ldd * es), sp, (size_t)(lds * es), (size_t)(cd * es), (size_t)rd,
                                 hipMemcpyDefault, st);
  }
  return 4;
}

// ---- DLPack export / import ------------------------------------------------------------
static void dl_deleter(DLManagedTensor* self) { array_release((Array*)self->manager_ctx); }

// A DLManagedTensor over `a` (a new reference, dropped by the consumer's deleter call).
// Device arrays export as kDLROCM, host arrays (pinned or not) as kDLCPU.
HETU_RT_API void* hetu_array_to_dlpack(void* a) {
  Array* src = (Array*)a;
  // every export gets its own header (the DLManagedTensor lives inside it)
  src->alloc->refs.fetch_add(1);
  Array* x = new_header(src->alloc, src->offset, src->dtype, src->device_type, src->device_id, src->ndim,
                        src->shape, src->strides);
  DLManagedTensor* m = &x->dl;
  m->dl_tensor.data = (char*)x->alloc->ptr + x->offset;
  // Pinned host memory exports as kDLCPU: it is host-addressable, and torch's DLPack importer
  // rejects kDLROCMHost.  The allocation record keeps the placement (freed to the pinned pool).
  m->dl_tensor.device.device_type = x->device_type == 2 ? kDLROCM : kDLCPU;
  m->dl_tensor.device.device_id = x->device_type == 2 ? x->device_id : 0;
  m->dl_tensor.ndim = x->ndim;
  m->dl_tensor.dtype = to_dl(x->dtype);
  m->dl_tensor.shape = x->shape;
  m->dl_tensor.strides = x->strides;
  m->dl_tensor.byte_offset = 0;
  m->manager_ctx = x;
  m->deleter = dl_deleter;
  return m;
}

// Borrow a producer's DLPack tensor (torch.utils.dlpack.to_dlpack): the array keeps it
// alive and calls its deleter when the last view is released.
HETU_RT_API int hetu_array_from_dlpack(void* managed, int dtype, void** out) {
  DLManagedTensor* m = (DLManagedTensor*)managed;
  const DLTensor& t = m->dl_tensor;
  if (t.ndim > kMaxDim) return 1;
  Alloc* a = new Alloc();
  a->mem = kBorrowed;
  a->borrowed = m;
  a->ptr = (char*)t.data + t.byte_offset;
  // DLPack allows strides == NULL for compact row-major tensors: derive those strides
  int64_t rm[kMaxDim];
  int64_t acc = 1;
  for (int d = t.ndim - 1; d >= 0; --d) { rm[d] = acc; acc *= t.shape[d]; }
  const int64_t* st = t.strides ? t.strides : rm;
  int64_t span = 1;
  bool empty = false;
  for (int d = 0; d < t.ndim; ++d) {
    if (t.shape[d] == 0) empty = true;
    else span += (t.shape[d] - 1) * st[d];
  }
  if (empty) span = 0;
  a->bytes = span * dtype_size(dtype);
  g_live_allocs.fetch_add(1);
  const int dev_type = (t.device.device_type == kDLROCM || t.device.device_type == 2) ? 2 : 1;
  *out = new_header(a, 0, dtype, dev_type, t.device.device_id, t.ndim, t.shape, st);
  return 0;
}

// live headers / allocations and headers created so far (leak checks, allocation census)
HETU_RT_API void hetu_array_stats(int64_t* out) {
  out[0] = g_live_arrays.load();
  out[1] = g_live_allocs.load();
  out[2] = g_created.load();
}
