// Best-fit-with-coalescing (BFC) allocator for device HBM and pinned host DRAM
// (reference src/memory_pool/allocator.h:15-248, BFC_allocator.h:13-186 -- a
// header-only design that was never built).
//
// MI355X-first sizing: regions are carved from hipMalloc (device) or
// hipHostMalloc (pinned host) in large, doubling extents (default first region
// 1 GiB, growing to 16 GiB) so a 288 GB HBM3E device is covered by a handful of
// regions and steady-state training never calls into the HIP driver.  Chunks
// are 256-byte aligned, bins are power-of-two size classes (21 bins from 256 B),
// free physical neighbours coalesce.
//
// Stream ordering without per-free events: every free chunk carries the stream
// it was last used on and lives in that stream's bins; an allocation on stream
// S reuses S's chunks or "clean" chunks (no pending work) only.  Neighbours
// coalesce only when their tags agree.  When S finds
// nothing, the allocator first *cleans* the other streams (one event per stream,
// waited once) -- moving their free chunks to the clean bins -- before it grows
// a region.  Same-stream reuse is immediate, as with a caching allocator.
// A chunk also used on side streams (record_stream) is held back when freed until an
// event recorded on each of those streams at the free has completed.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

namespace hetu {

struct AllocatorStats {          // mirrors reference allocator.h:36-55
  int64_t num_allocs = 0;
  int64_t bytes_in_use = 0;
  int64_t peak_bytes_in_use = 0;
  int64_t largest_alloc_size = 0;
  int64_t bytes_reserved = 0;    // bytes obtained from the sub-allocator
  int64_t bytes_limit = 0;
  int64_t num_regions = 0;
  int64_t num_free_chunks = 0;
};

// kHostTagged: plain host memory that keeps the per-stream bookkeeping of
// kDevice (stream handles are opaque tags, no events) -- for CPU unit tests.
enum class MemKind : int { kDevice = 0, kPinnedHost = 1, kHost = 2, kHostTagged = 3 };

class BFCAllocator {
 public:
  BFCAllocator(MemKind kind, int device, size_t limit_bytes, size_t first_region);
  ~BFCAllocator();

  void* allocate(size_t bytes, hipStream_t stream);
  void deallocate(void* p, hipStream_t stream);   // reusable by `stream` at once, by others once clean
  // p is also used on `stream` (a side stream: comm, PS staging, prefetch): once freed,
  // the chunk waits for that stream's work queued up to the free before anyone reuses it
  void record_stream(void* p, hipStream_t stream);
  // `stream` is being destroyed (work complete): its chunks become clean, and frees
  // that still name it are filed clean
  void forget_stream(hipStream_t stream);
  size_t allocation_size(void* p);
  AllocatorStats stats();
  size_t release_free_regions();                  // return wholly free regions; bytes released
  bool check_invariants();                        // debug: chunk-list / bin consistency
  // exact-size reuse cache in front of the bins (default on for device memory): a freed
  // chunk waits, uncoalesced, for the next request of its size on its stream -- training
  // steps repeat their allocation sizes, so most requests are one hash lookup; the cache
  // is flushed into the bins before the pool cleans streams or grows
  void set_cache(bool on);

 private:
  static constexpr int kNumBins = 21;
  static constexpr size_t kMinAlloc = 256;
  struct Chunk {
    char* ptr;
    size_t size;
    bool in_use;
    int region;
    Chunk* prev;   // physical neighbours inside the region
    Chunk* next;
    hipStream_t stream;   // last user (free chunks: owning bin set; nullptr = clean)
    bool listed;          // in a free bin
    std::vector<hipStream_t>* uses;   // record_stream: other streams using the chunk
    bool cached;          // in the exact-size cache
  };
  struct CacheKeyHash {
    size_t operator()(const std::pair<hipStream_t, size_t>& k) const {
      return std::hash<size_t>()(k.second) ^ (std::hash<uintptr_t>()((uintptr_t)k.first) * 0x9e3779b97f4a7c15ull);
    }
  };
  struct Pending {        // freed chunk whose side-stream uses are still in flight
    Chunk* c;
    std::vector<hipEvent_t> evs;
  };
  struct BySize {
    bool operator()(const Chunk* a, const Chunk* b) const {
      return a->size != b->size ? a->size < b->size : a->ptr < b->ptr;
    }
  };
  typedef std::set<Chunk*, BySize> Bin;
  struct Bins {
    Bin b[kNumBins];
  };
  struct Region {
    char* base;
    size_t size;
    Chunk* first;
  };

  static int bin_of(size_t size);
  bool tagged() const { return kind_ == MemKind::kDevice || kind_ == MemKind::kHostTagged; }
  bool plain_host() const { return kind_ == MemKind::kHost || kind_ == MemKind::kHostTagged; }
  static size_t round_up(size_t n) { return (n + kMinAlloc - 1) & ~(kMinAlloc - 1); }
  Chunk* take_from(Bins& bins, size_t size);
  Chunk* find_chunk(size_t size, hipStream_t s);
  bool grow(size_t min_bytes);
  void insert_free(Chunk* c);
  void erase_free(Chunk* c);
  Chunk* free_chunk(Chunk* c);   // returns the (possibly merged) free chunk
  void clean_streams();
  void relist_clean(std::vector<Chunk*>& moved);   // clean chunks back into the bins, coalescing
  void poll_pending(bool wait);   // release pending chunks whose side-stream events completed
  void flush_cache();             // cached chunks back into the bins (coalescing)
  Bins& bins_for(hipStream_t s);
  void* sub_alloc(size_t bytes);
  void sub_free(void* p);

  MemKind kind_;
  int device_;
  size_t limit_;
  size_t next_region_;
  std::mutex mu_;
  std::map<hipStream_t, Bins> bins_;
  hipStream_t last_stream_ = nullptr;   // bins_ lookup cache (map nodes are stable)
  Bins* last_bins_ = nullptr;
  std::vector<Pending> pending_;
  std::set<hipStream_t> dead_;   // destroyed streams (forget_stream) not seen alive since
  bool cache_on_ = false;
  std::unordered_map<std::pair<hipStream_t, size_t>, std::vector<Chunk*>, CacheKeyHash> cache_;
  size_t cached_n_ = 0;
  std::unordered_map<char*, Chunk*> in_use_;
  std::vector<Region> regions_;
  AllocatorStats st_;
};

}  // namespace hetu
