// BFC allocator implementation + C ABI + PyTorch pluggable-allocator entry
// points (see bfc_allocator.h for the design).
#include "bfc_allocator.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>

namespace hetu {

BFCAllocator::BFCAllocator(MemKind kind, int device, size_t limit_bytes, size_t first_region)
    : kind_(kind), device_(device), limit_(limit_bytes), next_region_(first_region) {
  st_.bytes_limit = (int64_t)limit_bytes;
  if (next_region_ < (2u << 20)) next_region_ = 2u << 20;
  cache_on_ = kind == MemKind::kDevice;
}

void BFCAllocator::set_cache(bool on) {
  std::lock_guard<std::mutex> g(mu_);
  if (!on) flush_cache();
  cache_on_ = on;
}

void BFCAllocator::flush_cache() {
  if (cached_n_ == 0) return;
  for (auto& kv : cache_) {
    for (Chunk* c : kv.second) {
      c->cached = false;
      st_.num_free_chunks--;   // counted as free while cached; free_chunk counts it again
      free_chunk(c);
    }
    kv.second.clear();
  }
  cached_n_ = 0;
}

BFCAllocator::~BFCAllocator() {
  for (auto& r : regions_) {
    Chunk* c = r.first;
    while (c) {
      Chunk* n = c->next;
      delete c;
      c = n;
    }
    sub_free(r.base);
  }
}

int BFCAllocator::bin_of(size_t size) {
  size_t q = size / kMinAlloc;
  int b = 0;
  while (q > 1 && b < kNumBins - 1) {
    q >>= 1;
    ++b;
  }
  return b;
}

void* BFCAllocator::sub_alloc(size_t bytes) {
  void* p = nullptr;
  if (plain_host()) {
    if (posix_memalign(&p, 4096, bytes) != 0) return nullptr;
    return p;
  }
  int cur = 0;
  hipGetDevice(&cur);
  if (cur != device_) hipSetDevice(device_);
  hipError_t e = kind_ == MemKind::kDevice ? hipMalloc(&p, bytes)
                                            : hipHostMalloc(&p, bytes, hipHostMallocPortable);
  if (cur != device_) hipSetDevice(cur);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void BFCAllocator::sub_free(void* p) {
  if (plain_host()) {
    free(p);
    return;
  }
  if (kind_ == MemKind::kDevice) {
    hipFree(p);
  } else {
    hipHostFree(p);
  }
}

BFCAllocator::Bins& BFCAllocator::bins_for(hipStream_t s) {
  if (last_bins_ == nullptr || s != last_stream_) {
    last_bins_ = &bins_[s];
    last_stream_ = s;
  }
  return *last_bins_;
}

void BFCAllocator::insert_free(Chunk* c) {
  bins_for(c->stream).b[bin_of(c->size)].insert(c);
  c->listed = true;
  st_.num_free_chunks++;
}

void BFCAllocator::erase_free(Chunk* c) {
  bins_for(c->stream).b[bin_of(c->size)].erase(c);
  c->listed = false;
  st_.num_free_chunks--;
}

BFCAllocator::Chunk* BFCAllocator::take_from(Bins& bins, size_t size) {
  Chunk key{nullptr, size, false, 0, nullptr, nullptr, nullptr, false, nullptr, false};
  for (int b = bin_of(size); b < kNumBins; ++b) {
    auto it = bins.b[b].lower_bound(&key);
    if (it != bins.b[b].end()) return *it;
  }
  return nullptr;
}

BFCAllocator::Chunk* BFCAllocator::find_chunk(size_t size, hipStream_t s) {
  Chunk* c = take_from(bins_for(s), size);
  if (c == nullptr && s != nullptr) c = take_from(bins_for(nullptr), size);
  if (c == nullptr) return nullptr;
  erase_free(c);
  if (c->size - size >= kMinAlloc) {   // split; the remainder stays free on the same stream
    Chunk* r = new Chunk{c->ptr + size, c->size - size, false, c->region, c, c->next, c->stream, false, nullptr, false};
    if (c->next) c->next->prev = r;
    c->next = r;
    c->size = size;
    insert_free(r);
  }
  return c;
}

bool BFCAllocator::grow(size_t min_bytes) {
  size_t want = std::max(next_region_, min_bytes);
  if (limit_ && (size_t)st_.bytes_reserved + want > limit_) want = min_bytes;
  if (limit_ && (size_t)st_.bytes_reserved + want > limit_) return false;
  void* p = sub_alloc(want);
  if (p == nullptr && want > min_bytes) {
    want = min_bytes;
    p = sub_alloc(want);
  }
  if (p == nullptr) return false;
  Chunk* c = new Chunk{(char*)p, want, false, (int)regions_.size(), nullptr, nullptr, nullptr, false, nullptr, false};
  regions_.push_back(Region{(char*)p, want, c});
  st_.bytes_reserved += (int64_t)want;
  st_.num_regions++;
  next_region_ = std::min<size_t>(next_region_ * 2, (size_t)16 << 30);
  insert_free(c);
  return true;
}

void BFCAllocator::poll_pending(bool wait) {
  size_t k = 0;
  for (size_t i = 0; i < pending_.size(); ++i) {
    Pending& pd = pending_[i];
    bool done = true;
    if (kind_ == MemKind::kDevice) {
      for (hipEvent_t e : pd.evs) {
        if (wait) {
          hipEventSynchronize(e);
        } else if (hipEventQuery(e) != hipSuccess) {
          (void)hipGetLastError();   // hipErrorNotReady is sticky-free but clear it anyway
          done = false;
          break;
        }
      }
    } else {
      done = wait;   // host-tagged (tests): side-stream uses end at the next clean
    }
    if (done) {
      for (hipEvent_t e : pd.evs) hipEventDestroy(e);
      free_chunk(pd.c);
    } else {
      pending_[k++] = pd;
    }
  }
  pending_.resize(k);
}

void BFCAllocator::clean_streams() {
  // wait for every stream that owns free chunks to pass "now", then move those
  // chunks to the clean bins (coalescing with clean neighbours)
  poll_pending(true);
  flush_cache();
  std::vector<Chunk*> moved;
  for (auto& kv : bins_) {
    if (kv.first == nullptr) continue;
    bool any = false;
    for (auto& bin : kv.second.b) any |= !bin.empty();
    if (!any) continue;
    if (kind_ == MemKind::kDevice) {
      // a stream being captured into a graph cannot be waited on: its chunks stay
      // tagged (they are reused by that stream itself, in capture order)
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(kv.first, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) continue;
      hipEvent_t ev;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
        hipEventRecord(ev, kv.first);
        hipEventSynchronize(ev);
        hipEventDestroy(ev);
      } else {
        hipStreamSynchronize(kv.first);
      }
    }
    for (auto& bin : kv.second.b) {
      for (Chunk* c : bin) moved.push_back(c);
      st_.num_free_chunks -= (int64_t)bin.size();
      bin.clear();
    }
  }
  relist_clean(moved);
}

void BFCAllocator::relist_clean(std::vector<Chunk*>& moved) {
  if (moved.empty()) return;
  std::unordered_map<Chunk*, int> mv;
  for (Chunk* c : moved) {
    c->stream = nullptr;
    c->listed = false;
    mv[c] = 1;
  }
  // one pass per region: re-insert moved chunks in address order so each one
  // coalesces with its (already re-listed) free predecessor
  for (auto& r : regions_) {
    Chunk* c = r.base ? r.first : nullptr;
    while (c) {
      if (mv.count(c)) {
        Chunk* m = free_chunk(c);
        c = m->next;
      } else {
        c = c->next;
      }
    }
  }
}

BFCAllocator::Chunk* BFCAllocator::free_chunk(Chunk* c) {
  // c is not in any bin here; merge with free neighbours of the same stream tag
  // (a tagged chunk never swallows clean memory: that would force a clean on the
  // next other-stream allocation)
  c->in_use = false;
  Chunk* p = c->prev;
  if (p && !p->in_use && p->stream == c->stream) {
    if (p->listed) {
      erase_free(p);
      p->size += c->size;
      p->next = c->next;
      if (c->next) c->next->prev = p;
      delete c;
      c = p;
    }
  }
  Chunk* n = c->next;
  if (n && !n->in_use && n->stream == c->stream) {
    if (n->listed) {
      erase_free(n);
      c->size += n->size;
      c->next = n->next;
      if (n->next) n->next->prev = c;
      delete n;
    }
  }
  insert_free(c);
  return c;
}

void* BFCAllocator::allocate(size_t bytes, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  if (!tagged()) stream = nullptr;
  if (!dead_.empty() && stream) dead_.erase(stream);   // a new stream at a recycled address
  size_t size = round_up(bytes ? bytes : 1);
  if (!pending_.empty()) poll_pending(false);
  Chunk* c = nullptr;
  if (cached_n_) {
    auto it = cache_.find(std::make_pair(stream, size));
    if (it != cache_.end() && !it->second.empty()) {
      c = it->second.back();
      it->second.pop_back();
      c->cached = false;
      cached_n_--;
      st_.num_free_chunks--;
    }
  }
  if (c == nullptr) c = find_chunk(size, stream);
  if (c == nullptr && cached_n_) {
    flush_cache();
    c = find_chunk(size, stream);
  }
  if (c == nullptr) {
    clean_streams();
    c = find_chunk(size, stream);
  }
  if (c == nullptr && grow(size)) c = find_chunk(size, stream);
  if (c == nullptr) {
    // last resort: hand wholly free regions back to the driver and retry once
    size_t freed = 0;
    for (size_t i = 0; i < regions_.size(); ++i) {
      Region& r = regions_[i];
      Chunk* f = r.first;
      if (f && !f->in_use && f->listed && f->next == nullptr && f->size == r.size && r.base) {
        erase_free(f);
        delete f;
        sub_free(r.base);
        freed += r.size;
        st_.bytes_reserved -= (int64_t)r.size;
        st_.num_regions--;
        r.base = nullptr;
        r.first = nullptr;
        r.size = 0;
      }
    }
    if (freed && grow(size)) c = find_chunk(size, stream);
    if (c == nullptr) return nullptr;
  }
  c->in_use = true;
  c->stream = stream;
  in_use_[c->ptr] = c;
  st_.num_allocs++;
  st_.bytes_in_use += (int64_t)c->size;
  st_.peak_bytes_in_use = std::max(st_.peak_bytes_in_use, st_.bytes_in_use);
  st_.largest_alloc_size = std::max(st_.largest_alloc_size, (int64_t)c->size);
  return c->ptr;
}

void BFCAllocator::deallocate(void* p, hipStream_t stream) {
  if (p == nullptr) return;
  std::lock_guard<std::mutex> g(mu_);
  auto it = in_use_.find((char*)p);
  if (it == in_use_.end()) {
    fprintf(stderr, "hetu BFC: free of unknown pointer %p\n", p);
    return;
  }
  Chunk* c = it->second;
  in_use_.erase(it);
  st_.bytes_in_use -= (int64_t)c->size;
  if (tagged() && stream != nullptr) c->stream = stream;
  if (!tagged()) c->stream = nullptr;
  if (!dead_.empty() && c->stream && dead_.count(c->stream)) c->stream = nullptr;   // destroyed: work complete
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (c->uses && kind_ == MemKind::kDevice && stream != nullptr &&
      hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    delete c->uses;   // inside a capture the graph's own stream order covers the side uses
    c->uses = nullptr;
  }
  if (c->uses) {   // side-stream uses: hold the chunk until they pass this point
    Pending pd{c, {}};
    if (kind_ == MemKind::kDevice) {
      for (hipStream_t s : *c->uses) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
          hipEventRecord(e, s);
          pd.evs.push_back(e);
        } else {
          hipStreamSynchronize(s);
        }
      }
    }
    delete c->uses;
    c->uses = nullptr;
    c->in_use = false;
    pending_.push_back(pd);
    return;
  }
  if (cache_on_) {
    c->in_use = false;
    c->cached = true;
    cache_[std::make_pair(c->stream, c->size)].push_back(c);
    cached_n_++;
    st_.num_free_chunks++;
    return;
  }
  free_chunk(c);
}

// `s` is about to be destroyed (its work is complete: the caller synchronised it).
// Its free and cached chunks move to the clean bins, and later frees that name it are
// filed clean: a destroyed handle must never be waited on, and a new stream created at
// the same address must not inherit another stream's chunks.
void BFCAllocator::forget_stream(hipStream_t s) {
  if (!s) return;
  std::lock_guard<std::mutex> g(mu_);
  poll_pending(true);
  flush_cache();
  std::vector<Chunk*> moved;
  auto it = bins_.find(s);
  if (it != bins_.end()) {
    for (auto& bin : it->second.b) {
      for (Chunk* c : bin) moved.push_back(c);
      st_.num_free_chunks -= (int64_t)bin.size();
      bin.clear();
    }
    bins_.erase(it);
  }
  last_stream_ = nullptr;
  last_bins_ = nullptr;
  for (Chunk* c : moved) {
    c->stream = nullptr;
    c->listed = false;
  }
  relist_clean(moved);
  for (auto& kv : in_use_) {
    Chunk* c = kv.second;
    if (c->stream == s) c->stream = nullptr;
    if (c->uses) c->uses->erase(std::remove(c->uses->begin(), c->uses->end(), s), c->uses->end());
  }
  dead_.insert(s);
}

void BFCAllocator::record_stream(void* p, hipStream_t stream) {
  if (p == nullptr || !tagged()) return;
  std::lock_guard<std::mutex> g(mu_);
  auto it = in_use_.find((char*)p);
  if (it == in_use_.end()) return;
  Chunk* c = it->second;
  if (stream == c->stream) return;
  if (!c->uses) c->uses = new std::vector<hipStream_t>();
  if (std::find(c->uses->begin(), c->uses->end(), stream) == c->uses->end()) c->uses->push_back(stream);
}

size_t BFCAllocator::allocation_size(void* p) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = in_use_.find((char*)p);
  return it == in_use_.end() ? 0 : it->second->size;
}

AllocatorStats BFCAllocator::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

size_t BFCAllocator::release_free_regions() {
  std::lock_guard<std::mutex> g(mu_);
  clean_streams();   // (flushes the exact-size cache first)
  size_t freed = 0;
  for (auto& r : regions_) {
    Chunk* f = r.first;
    if (r.base && f && !f->in_use && f->listed && f->next == nullptr && f->size == r.size) {
      erase_free(f);
      delete f;
      sub_free(r.base);
      freed += r.size;
      st_.bytes_reserved -= (int64_t)r.size;
      st_.num_regions--;
      r.base = nullptr;
      r.first = nullptr;
      r.size = 0;
    }
  }
  return freed;
}

bool BFCAllocator::check_invariants() {
  std::lock_guard<std::mutex> g(mu_);
  int64_t used = 0, nfree = 0;
  for (auto& r : regions_) {
    if (!r.base) continue;
    size_t total = 0;
    char* expect = r.base;
    for (Chunk* c = r.first; c; c = c->next) {
      if (c->ptr != expect) return false;
      if (c->next && c->next->prev != c) return false;
      if (c->size % kMinAlloc) return false;
      if (c->in_use) {
        used += (int64_t)c->size;
        if (!in_use_.count(c->ptr)) return false;
      } else if (c->cached) {
        if (c->listed) return false;   // exact-size cache: in no bin
        ++nfree;
      } else if (std::any_of(pending_.begin(), pending_.end(), [c](const Pending& pd) { return pd.c == c; })) {
        if (c->listed) return false;   // held back for a side stream: in no bin yet
      } else {
        if (!c->listed || !bins_[c->stream].b[bin_of(c->size)].count(c)) return false;
        ++nfree;
        // no two adjacent free chunks with compatible streams may remain
        if (c->next && !c->next->in_use && c->next->listed && c->next->stream == c->stream) return false;
      }
      expect += c->size;
      total += c->size;
    }
    if (total != r.size) return false;
  }
  return used == st_.bytes_in_use && nfree == st_.num_free_chunks;
}

}  // namespace hetu

// ---------------------------------------------------------------------------
// C ABI (ctypes) and torch.cuda.memory.CUDAPluggableAllocator entry points
using hetu::BFCAllocator;
using hetu::MemKind;

#define HETU_RT_API extern "C" __attribute__((visibility("default")))

HETU_RT_API void* hetu_bfc_create(int kind, int device, int64_t limit_bytes, int64_t first_region) {
  return new BFCAllocator((MemKind)kind, device, (size_t)limit_bytes, (size_t)first_region);
}
HETU_RT_API void hetu_bfc_destroy(void* h) { delete (BFCAllocator*)h; }
HETU_RT_API void* hetu_bfc_alloc(void* h, int64_t bytes, void* stream) {
  return ((BFCAllocator*)h)->allocate((size_t)bytes, (hipStream_t)stream);
}
HETU_RT_API void hetu_bfc_free(void* h, void* p, void* stream) {
  ((BFCAllocator*)h)->deallocate(p, (hipStream_t)stream);
}
HETU_RT_API void hetu_bfc_record_stream(void* h, void* p, void* stream) {
  ((BFCAllocator*)h)->record_stream(p, (hipStream_t)stream);
}
HETU_RT_API void hetu_bfc_forget_stream(void* h, void* stream) {
  ((BFCAllocator*)h)->forget_stream((hipStream_t)stream);
}
HETU_RT_API void hetu_bfc_set_cache(void* h, int on) { ((BFCAllocator*)h)->set_cache(on != 0); }
HETU_RT_API int64_t hetu_bfc_size(void* h, void* p) { return (int64_t)((BFCAllocator*)h)->allocation_size(p); }
HETU_RT_API int64_t hetu_bfc_release(void* h) { return (int64_t)((BFCAllocator*)h)->release_free_regions(); }
HETU_RT_API int hetu_bfc_check(void* h) { return ((BFCAllocator*)h)->check_invariants() ? 1 : 0; }
HETU_RT_API void hetu_bfc_stats(void* h, int64_t* out) {
  hetu::AllocatorStats s = ((BFCAllocator*)h)->stats();
  out[0] = s.num_allocs;
  out[1] = s.bytes_in_use;
  out[2] = s.peak_bytes_in_use;
  out[3] = s.largest_alloc_size;
  out[4] = s.bytes_reserved;
  out[5] = s.bytes_limit;
  out[6] = s.num_regions;
  out[7] = s.num_free_chunks;
}

// One device allocator per GPU for torch's pluggable-allocator hook
// (HETU_ALLOCATOR=bfc).  Limit: HETU_BFC_LIMIT_GB, default 95% of the device.
static BFCAllocator* g_dev[64];
static std::mutex g_dev_mu;

static BFCAllocator* dev_alloc(int device) {
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_dev_mu);
  if (!g_dev[device]) {
    size_t limit = 0;
    const char* env = getenv("HETU_BFC_LIMIT_GB");
    if (env) {
      limit = (size_t)(atof(env) * (double)(1ull << 30));
    } else {
      int cur = 0;
      hipGetDevice(&cur);
      hipSetDevice(device);
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess) limit = (size_t)(tot * 0.95);
      hipSetDevice(cur);
    }
    const char* reg = getenv("HETU_BFC_REGION_MB");
    size_t first = reg ? (size_t)atoll(reg) << 20 : (size_t)1 << 30;
    g_dev[device] = new BFCAllocator(MemKind::kDevice, device, limit, first);
  }
  return g_dev[device];
}

// the device pool itself (framework arrays, csrc/runtime/array.cc, allocate from the same
// BFC pool as torch's pluggable-allocator hook)
HETU_RT_API void* hetu_bfc_device_pool(int device) { return dev_alloc(device); }

// Private pools for hipGraph capture (the native counterpart of torch's graph memory
// pools): between hetu_torch_pool_begin and _end every allocation on the device that is
// made on the capture stream, or on any stream that is capturing at that moment (side
// streams forked into the graph), comes from a pool of its own, so the captured step's
// buffers are never handed to code outside the graph; the graph replays them in
// capture order.  Other streams (another thread's work) keep the device allocator.
// The pool lives until hetu_torch_pool_release (graph destroyed); a pool released while
// some of its chunks are still held (outputs of the graph kept by the caller) retires
// and is deleted by the free that returns its last chunk.
static std::map<int64_t, BFCAllocator*> g_pools;
static std::set<BFCAllocator*> g_retiring;
static std::atomic<int> g_npools{0};
static std::atomic<BFCAllocator*> g_active_pool[64];
static std::atomic<hipStream_t> g_active_stream[64];
static int64_t g_pool_seq = 0;

HETU_RT_API int64_t hetu_torch_pool_begin(int device, hipStream_t stream) {
  if (device < 0 || device >= 64) return -1;
  std::lock_guard<std::mutex> g(g_dev_mu);
  const char* reg = getenv("HETU_BFC_POOL_REGION_MB");
  size_t first = reg ? (size_t)atoll(reg) << 20 : (size_t)64 << 20;
  BFCAllocator* p = new BFCAllocator(MemKind::kDevice, device, 0, first);
  const int64_t id = ++g_pool_seq;
  g_pools[id] = p;
  g_npools.fetch_add(1);
  g_active_stream[device].store(stream);
  g_active_pool[device].store(p);
  return id;
}

HETU_RT_API void hetu_torch_pool_end(int device) {
  if (device < 0 || device >= 64) return;
  std::lock_guard<std::mutex> g(g_dev_mu);
  g_active_pool[device].store(nullptr);
  g_active_stream[device].store(nullptr);
}

HETU_RT_API void hetu_torch_pool_stats(int64_t id, int64_t* out) {
  BFCAllocator* p = nullptr;
  {
    std::lock_guard<std::mutex> g(g_dev_mu);
    auto it = g_pools.find(id);
    if (it != g_pools.end()) p = it->second;
  }
  if (p) hetu_bfc_stats(p, out);
}

// drop a pool (the graph using it must be destroyed): its memory goes back to the
// driver now, or -- while chunks are still held -- when the last one is freed
HETU_RT_API void hetu_torch_pool_release(int64_t id) {
  BFCAllocator* p = nullptr;
  {
    std::lock_guard<std::mutex> g(g_dev_mu);
    auto it = g_pools.find(id);
    if (it == g_pools.end()) return;
    p = it->second;
    for (auto& a : g_active_pool) {
      BFCAllocator* cur = p;
      a.compare_exchange_strong(cur, nullptr);
    }
    if (p->stats().bytes_in_use > 0) {
      g_retiring.insert(p);   // still owns chunks: found by hetu_torch_free until its last free
      return;
    }
    g_pools.erase(it);
    g_npools.fetch_sub(1);
  }
  hipDeviceSynchronize();
  delete p;
}

HETU_RT_API void* hetu_torch_alloc(ssize_t size, int device, hipStream_t stream) {
  BFCAllocator* a = nullptr;
  if (device >= 0 && device < 64) {
    BFCAllocator* p = g_active_pool[device].load();
    if (p) {
      bool mine = stream == g_active_stream[device].load();
      if (!mine) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        mine = hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
      }
      if (mine) a = p;
    }
  }
  if (!a) a = dev_alloc(device);
  return a ? a->allocate((size_t)size, stream) : nullptr;
}

HETU_RT_API void hetu_torch_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  BFCAllocator* d = dev_alloc(device);
  if (g_npools.load() == 0 || (d && d->allocation_size(ptr))) {
    if (d) d->deallocate(ptr, stream);
    return;
  }
  // A capture-pool chunk: the owner lookup, the free and the retire check run under one
  // lock, so a concurrent free of another chunk of a retiring pool can never reach a pool
  // that this free is about to delete.
  BFCAllocator* dead = nullptr;
  {
    std::lock_guard<std::mutex> g(g_dev_mu);
    BFCAllocator* a = nullptr;
    auto owner = g_pools.end();
    for (auto it = g_pools.begin(); it != g_pools.end(); ++it)
      if (it->second->allocation_size(ptr)) { a = it->second; owner = it; break; }
    if (!a) return;
    a->deallocate(ptr, stream);
    if (g_retiring.count(a) && a->stats().bytes_in_use == 0) {
      g_retiring.erase(a);
      g_pools.erase(owner);
      g_npools.fetch_sub(1);
      dead = a;
    }
  }
  if (dead) {
    hipDeviceSynchronize();
    delete dead;
  }
}

HETU_RT_API void hetu_torch_record_stream(int device, void* ptr, hipStream_t stream) {
  BFCAllocator* d = dev_alloc(device);
  if (g_npools.load() == 0 || (d && d->allocation_size(ptr))) {
    if (d) d->record_stream(ptr, stream);
    return;
  }
  std::lock_guard<std::mutex> g(g_dev_mu);   // pool chunks: see hetu_torch_free
  for (auto& kv : g_pools)
    if (kv.second->allocation_size(ptr)) { kv.second->record_stream(ptr, stream); return; }
}

// a framework stream is being destroyed: the device allocator and every capture pool
// forget it (DeviceStream.__del__)
HETU_RT_API void hetu_torch_forget_stream(int device, hipStream_t stream) {
  BFCAllocator* a = dev_alloc(device);
  if (a) a->forget_stream(stream);
  std::lock_guard<std::mutex> g(g_dev_mu);
  for (auto& kv : g_pools) kv.second->forget_stream(stream);
}

HETU_RT_API void hetu_torch_stats(int device, int64_t* out) {
  BFCAllocator* a = dev_alloc(device);
  if (a) hetu_bfc_stats(a, out);
}
