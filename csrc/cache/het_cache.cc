// HET embedding cache (reference src/hetu_cache: cache.h:21-108, cache.cc:14-296,
// lfuopt_cache.cc:5-83, hetu_client.cc:6-105) re-implemented for one MI355X node.
//
// A worker-local cache of embedding rows in host DRAM in front of the shared-memory
// PS (shm_ps).  Bounded staleness:
//   * lookup: keys are uniqued; every unique key's cached version is sent to the
//     PS (SyncEmbedding); the PS returns only rows whose server version is more
//     than `pull_bound` ahead (or rows the cache does not hold), which are merged
//     with any local, not-yet-pushed gradient;
//   * update: gradients are applied to the cached line and accumulated; a line is
//     pushed (PushEmbedding: data += grad, version += updates) once its local
//     update count exceeds `push_bound`, or when it is evicted.
// Policies: LRU, LFU (O(1) frequency buckets) and LFUOpt (LFU whose insertion of a
// batch promotes the batch's lines together, avoiding thrash on skewed batches).
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../ps/shm_ps.h"

namespace hc {

// A cached row: header + its data and pending-gradient vectors live in one pooled
// record (no per-line heap allocations); policy lists are intrusive.
struct FreqNode;
struct Line {
  int64_t key;
  int64_t ver;      // server version this line reflects
  int64_t updates;  // local updates not yet pushed
  int64_t freq;
  Line* prev;
  Line* next;
  FreqNode* fnode;  // LFU bucket
  bool cached;
  float* data;
  float* grad;
};

struct DList {  // intrusive doubly-linked list of lines, most recent at head
  Line* head = nullptr;
  Line* tail = nullptr;
  bool empty() const { return head == nullptr; }
  void push_front(Line* l) {
    l->prev = nullptr;
    l->next = head;
    if (head) head->prev = l;
    head = l;
    if (!tail) tail = l;
  }
  void remove(Line* l) {
    if (l->prev) l->prev->next = l->next; else head = l->next;
    if (l->next) l->next->prev = l->prev; else tail = l->prev;
    l->prev = l->next = nullptr;
  }
};

// open-addressing int64 -> Line* map (linear probing, backward-shift deletion)
class KeyMap {
 public:
  KeyMap() { rehash(1024); }
  Line* find(int64_t k) const {
    for (size_t i = slot(k);; i = (i + 1) & mask_) {
      if (keys_[i] == kEmpty) return nullptr;
      if (keys_[i] == k) return vals_[i];
    }
  }
  void insert(int64_t k, Line* v) {
    if ((size_ + 1) * 2 > keys_.size()) rehash(keys_.size() * 2);
    size_t i = slot(k);
    while (keys_[i] != kEmpty && keys_[i] != k) i = (i + 1) & mask_;
    if (keys_[i] == kEmpty) ++size_;
    keys_[i] = k;
    vals_[i] = v;
  }
  void erase(int64_t k) {
    size_t i = slot(k);
    while (keys_[i] != k) {
      if (keys_[i] == kEmpty) return;
      i = (i + 1) & mask_;
    }
    // backward shift: move later entries of the probe run into the hole
    size_t j = i;
    for (;;) {
      j = (j + 1) & mask_;
      if (keys_[j] == kEmpty) break;
      size_t h = slot(keys_[j]);
      const bool between = (i <= j) ? (i < h && h <= j) : (i < h || h <= j);
      if (!between) {
        keys_[i] = keys_[j];
        vals_[i] = vals_[j];
        i = j;
      }
    }
    keys_[i] = kEmpty;
    --size_;
  }
  size_t size() const { return size_; }
  template <class F> void for_each(F f) const {
    for (size_t i = 0; i < keys_.size(); ++i)
      if (keys_[i] != kEmpty) f(vals_[i]);
  }
  void clear() {
    keys_.assign(1024, kEmpty);
    vals_.assign(1024, nullptr);
    mask_ = 1023;
    size_ = 0;
  }

 private:
  static constexpr int64_t kEmpty = INT64_MIN;
  size_t slot(int64_t k) const {
    uint64_t x = (uint64_t)k + 0x9e3779b97f4a7c15ull;   // splitmix64 finaliser
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return (size_t)(x ^ (x >> 31)) & mask_;
  }
  void rehash(size_t cap) {
    std::vector<int64_t> ok;
    std::vector<Line*> ov;
    ok.swap(keys_);
    ov.swap(vals_);
    keys_.assign(cap, kEmpty);
    vals_.assign(cap, nullptr);
    mask_ = cap - 1;
    size_ = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmpty) insert(ok[i], ov[i]);
  }
  std::vector<int64_t> keys_;
  std::vector<Line*> vals_;
  size_t mask_ = 0, size_ = 0;
};

// fixed-size record pool: Line header + 2*width floats per record
class LinePool {
 public:
  explicit LinePool(int64_t width) : width_(width) {}
  Line* get() {
    if (free_.empty()) grow();
    Line* l = free_.back();
    free_.pop_back();
    return l;
  }
  void put(Line* l) { free_.push_back(l); }
  void reset() {
    free_.clear();
    chunks_.clear();
  }

 private:
  void grow() {
    const size_t rec = sizeof(Line) + 2 * (size_t)width_ * sizeof(float);
    const size_t recr = (rec + 63) & ~(size_t)63;
    const size_t n = 4096;
    chunks_.emplace_back(new char[recr * n + 64]);
    char* base = (char*)(((uintptr_t)chunks_.back().get() + 63) & ~(uintptr_t)63);
    for (size_t i = 0; i < n; ++i) {
      Line* l = reinterpret_cast<Line*>(base + i * recr);
      l->data = reinterpret_cast<float*>((char*)l + sizeof(Line));
      l->grad = l->data + width_;
      free_.push_back(l);
    }
  }
  int64_t width_;
  std::vector<Line*> free_;
  std::vector<std::unique_ptr<char[]>> chunks_;
};

class Policy {
 public:
  virtual ~Policy() {}
  virtual void touch(Line* l) = 0;
  virtual void insert(Line* l) = 0;
  virtual Line* evict() = 0;  // unlinks and returns the victim
  virtual void reset() = 0;
};

class LRU : public Policy {
 public:
  void touch(Line* l) override {
    lst_.remove(l);
    lst_.push_front(l);
  }
  void insert(Line* l) override { lst_.push_front(l); }
  Line* evict() override {
    Line* v = lst_.tail;
    if (v) lst_.remove(v);
    return v;
  }
  void reset() override { lst_ = DList(); }

 private:
  DList lst_;
};

// O(1) LFU: an ascending list of frequency buckets, each an intrusive list of lines
// (most recently touched first); eviction takes the oldest line of the lowest bucket.
struct FreqNode {
  int64_t freq;
  DList lines;
  FreqNode* prev;
  FreqNode* next;
};

class LFU : public Policy {
 public:
  explicit LFU(bool opt) : opt_(opt) {}
  ~LFU() override { reset(); }
  void touch(Line* l) override {
    FreqNode* f = l->fnode;
    const int64_t nf = f->freq + 1;
    FreqNode* g = f->next;
    if (!g || g->freq != nf) g = link_after(f, nf);
    f->lines.remove(l);
    g->lines.push_front(l);
    l->fnode = g;
    l->freq = nf;
    if (f->lines.empty()) unlink(f);
  }
  void insert(Line* l) override {
    // LFUOpt: a new line enters at the minimum live frequency instead of 1, so a
    // burst of new keys does not immediately evict each other
    int64_t f0 = l->freq;
    if (opt_ && head_) f0 = std::max<int64_t>(f0, head_->freq);
    FreqNode* g = head_;
    if (!g || g->freq != f0) {
      // f0 <= every live frequency (plain LFU inserts at 1, LFUOpt at the minimum)
      g = link_after(nullptr, f0);
    }
    g->lines.push_front(l);
    l->fnode = g;
    l->freq = f0;
  }
  Line* evict() override {
    FreqNode* h = head_;
    if (!h) return nullptr;
    Line* v = h->lines.tail;
    h->lines.remove(v);
    if (h->lines.empty()) unlink(h);
    return v;
  }
  void reset() override {
    for (FreqNode* f = head_; f;) {
      FreqNode* n = f->next;
      delete f;
      f = n;
    }
    head_ = nullptr;
    for (FreqNode* f : spare_) delete f;
    spare_.clear();
  }

 private:
  FreqNode* link_after(FreqNode* f, int64_t freq) {
    FreqNode* g;
    if (!spare_.empty()) {
      g = spare_.back();
      spare_.pop_back();
    } else {
      g = new FreqNode();
    }
    g->freq = freq;
    g->lines = DList();
    g->prev = f;
    g->next = f ? f->next : head_;
    if (g->next) g->next->prev = g;
    if (f) f->next = g; else head_ = g;
    return g;
  }
  void unlink(FreqNode* f) {
    if (f->prev) f->prev->next = f->next; else head_ = f->next;
    if (f->next) f->next->prev = f->prev;
    spare_.push_back(f);
  }
  bool opt_;
  FreqNode* head_ = nullptr;
  std::vector<FreqNode*> spare_;
};

struct Perf {
  int64_t calls = 0, unique = 0, miss = 0, transfer = 0, evict = 0, pushed = 0;
  double t_unique = 0, t_sync = 0, t_copy = 0, t_push = 0;
};

// Small persistent fork-join pool for the cache's row-copy / gradient loops, which
// are host-memory-bandwidth bound on one thread (HETU_CACHE_THREADS, default 4).
// Every run() publishes its own Job (range, part count, callable, chunk counter,
// completion count).  A worker copies the job pointer under the mutex and only ever
// takes chunks from THAT job's counter, so a worker woken for an earlier run that is
// descheduled between wake-up and fetch_add cannot execute a chunk of a later run
// (it finds its old job exhausted), and run() returns only after every chunk of its
// own job has finished.
class ParallelFor {
 public:
  ParallelFor() {
    int n = 4;
    if (const char* e = getenv("HETU_CACHE_THREADS")) n = atoi(e);
    n = std::max(1, std::min(n, 64));
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { worker(); });
    nthreads_ = n;
  }
  ~ParallelFor() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(begin, end) over [0, n) in chunks; runs inline when small or single-threaded
  void run(int64_t n, int64_t min_chunk, const std::function<void(int64_t, int64_t)>& fn) {
    if (nthreads_ == 1 || n < 2 * min_chunk) {
      fn(0, n);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);   // one parallel region at a time
    auto job = std::make_shared<Job>();
    job->n = n;
    job->parts = std::min<int64_t>(nthreads_, n / min_chunk);
    job->fn = &fn;
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    {
      std::unique_lock<std::mutex> g(mu_);
      done_cv_.wait(g, [&] { return job->done == job->parts; });
      job_.reset();   // workers still holding `job` see it exhausted
    }
  }

 private:
  struct Job {
    int64_t n = 0, parts = 0;
    const std::function<void(int64_t, int64_t)>* fn = nullptr;
    std::atomic<int64_t> next{0};
    int64_t done = 0;   // guarded by mu_
  };
  void work(Job& j) {
    for (;;) {
      const int64_t p = j.next.fetch_add(1);
      if (p >= j.parts) return;
      const int64_t b = j.n * p / j.parts, e = j.n * (p + 1) / j.parts;
      (*j.fn)(b, e);
      std::lock_guard<std::mutex> g(mu_);
      if (++j.done == j.parts) done_cv_.notify_all();
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      if (job) work(*job);
    }
  }
  std::vector<std::thread> th_;
  int nthreads_ = 1;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

static ParallelFor& pool() {
  static ParallelFor p;
  return p;
}

// De-duplication of a batch of keys in O(n): an open-addressing scratch table
// (reused across calls, cleared by generation stamps) maps each key to its first
// occurrence.  uniq = distinct keys in first-seen order, pos[r] = index of keys[r].
class Dedup {
 public:
  void run(const int64_t* keys, int64_t n, std::vector<int64_t>& uniq, std::vector<int32_t>& pos) {
    size_t cap = 64;
    while (cap < (size_t)n * 2) cap <<= 1;
    if (cap > tkey_.size()) {
      tkey_.assign(cap, 0);
      tidx_.assign(cap, 0);
      tgen_.assign(cap, 0);
      gen_ = 0;
    }
    const size_t mask = cap - 1;
    if (++gen_ == 0) {               // stamp wrap-around: clear once
      std::fill(tgen_.begin(), tgen_.end(), 0);
      gen_ = 1;
    }
    uniq.clear();
    pos.resize(n);
    for (int64_t r = 0; r < n; ++r) {
      const int64_t k = keys[r];
      uint64_t x = (uint64_t)k * 0x9e3779b97f4a7c15ull;
      size_t i = (size_t)(x >> 32) & mask;
      for (;; i = (i + 1) & mask) {
        if (tgen_[i] != gen_) {
          tgen_[i] = gen_;
          tkey_[i] = k;
          tidx_[i] = (int32_t)uniq.size();
          uniq.push_back(k);
          break;
        }
        if (tkey_[i] == k) break;
      }
      pos[r] = tidx_[i];
    }
  }

 private:
  std::vector<int64_t> tkey_;
  std::vector<int32_t> tidx_;
  std::vector<uint32_t> tgen_;
  uint32_t gen_ = 0;
};

class Cache {
 public:
  Cache(int policy, int64_t limit, int64_t rows, int64_t width, int key, int64_t pull_bound,
        int64_t push_bound)
      : limit_(limit), rows_(rows), width_(width), key_(key), pull_bound_(pull_bound),
        push_bound_(push_bound), policy_(policy), pool_(width) {
    make_policy();
  }
  ~Cache() { pol_.reset(); }

  void lookup(const int64_t* keys, int64_t n, float* dest) {
    std::lock_guard<std::mutex> g(mu_);
    auto t0 = std::chrono::steady_clock::now();
    dedup_.run(keys, n, uniq_, pos_);
    auto t1 = std::chrono::steady_clock::now();
    const int64_t u = (int64_t)uniq_.size();
    vers_.resize(u);
    lines_.resize(u);
    int64_t miss = 0;
    for (int64_t i = 0; i < u; ++i) {
      Line* l = map_.find(uniq_[i]);
      lines_[i] = l;
      vers_[i] = (l && !bypass_) ? l->ver : -1;
      miss += l == nullptr;
    }
    idx_.resize(u);
    nver_.resize(u);
    if ((int64_t)sync_data_.size() < u * width_) sync_data_.resize((size_t)u * width_);
    int64_t cnt = hps_sync_embedding(key_, uniq_.data(), u, vers_.data(), pull_bound_, idx_.data(),
                                     nver_.data(), sync_data_.data());
    auto t2 = std::chrono::steady_clock::now();
    for (int64_t c = 0; c < std::max<int64_t>(cnt, 0); ++c) {
      const int64_t i = idx_[c];
      const float* src = sync_data_.data() + c * width_;
      Line* l = lines_[i];
      if (!l) {
        l = pool_.get();
        l->key = uniq_[i];
        l->updates = 0;
        l->freq = 1;
        l->prev = l->next = nullptr;
        l->fnode = nullptr;
        memcpy(l->data, src, width_ * sizeof(float));
        memset(l->grad, 0, width_ * sizeof(float));
        l->ver = nver_[c];
        admit(l);
        lines_[i] = l;
      } else {
        // server copy + our pending (unpushed) gradient
        for (int64_t j = 0; j < width_; ++j) l->data[j] = src[j] + l->grad[j];
        l->ver = nver_[c];
      }
    }
    for (int64_t i = 0; i < u; ++i)
      if (lines_[i] && lines_[i]->cached) pol_->touch(lines_[i]);
    pool().run(n, 256, [&](int64_t b, int64_t e) {
      for (int64_t r = b; r < e; ++r) {
        const Line* l = lines_[pos_[r]];
        if (l) memcpy(dest + r * width_, l->data, width_ * sizeof(float));
        else memset(dest + r * width_, 0, width_ * sizeof(float));
      }
    });
    flush_pending();   // gradients of dirty lines evicted by this batch's admissions
    release_evicted();
    auto t3 = std::chrono::steady_clock::now();
    if (perf_) {
      perf_rec_.calls++;
      perf_rec_.unique += u;
      perf_rec_.miss += miss;
      perf_rec_.transfer += std::max<int64_t>(cnt, 0);
      perf_rec_.t_unique += std::chrono::duration<double>(t1 - t0).count();
      perf_rec_.t_sync += std::chrono::duration<double>(t2 - t1).count();
      perf_rec_.t_copy += std::chrono::duration<double>(t3 - t2).count();
    }
  }

  void update(const int64_t* keys, int64_t n, const float* grads) {
    std::lock_guard<std::mutex> g(mu_);
    dedup_.run(keys, n, ukeys_, pos_);
    const int64_t u = (int64_t)ukeys_.size();
    // cached rows take their gradient rows directly (no accumulation pass); rows
    // the cache does not hold are summed per key and pushed straight through
    ulines_.resize(u);
    slot_.assign(u, -1);
    int64_t nacc = 0;
    for (int64_t i = 0; i < u; ++i) {
      Line* l = bypass_ ? nullptr : map_.find(ukeys_[i]);
      ulines_[i] = l;
      if (!l) slot_[i] = nacc++;
    }
    acc_.assign((size_t)nacc * width_, 0.f);
    // rows grouped by key (counting sort), then keys split over threads: every key's
    // rows are applied by one thread, so lines and accumulators need no locks
    start_.assign(u + 1, 0);
    for (int64_t r = 0; r < n; ++r) ++start_[pos_[r] + 1];
    for (int64_t i = 0; i < u; ++i) start_[i + 1] += start_[i];
    order_.resize(n);
    fill_ = start_;
    for (int64_t r = 0; r < n; ++r) order_[fill_[pos_[r]]++] = r;
    pool().run(u, 64, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        Line* l = ulines_[i];
        float* __restrict__ d = l ? l->data : acc_.data() + slot_[i] * width_;
        float* __restrict__ gg = l ? l->grad : nullptr;
        const int64_t w = width_;
        for (int64_t q = start_[i]; q < start_[i + 1]; ++q) {
          const float* __restrict__ gr = grads + order_[q] * w;
          if (gg) {
            for (int64_t j = 0; j < w; ++j) {
              d[j] += gr[j];
              gg[j] += gr[j];
            }
          } else {
            for (int64_t j = 0; j < w; ++j) d[j] += gr[j];
          }
        }
      }
    });
    for (int64_t i = 0; i < u; ++i) {
      Line* l = ulines_[i];
      if (!l) {
        const float* a = acc_.data() + slot_[i] * width_;
        prow_.push_back(ukeys_[i]);
        pupd_.push_back(1);
        pdata_.insert(pdata_.end(), a, a + width_);
        continue;
      }
      l->updates += 1;
      if (l->updates > push_bound_) stage_push(l);
    }
    flush_pending();
  }

  void flush_all() {
    std::lock_guard<std::mutex> g(mu_);
    map_.for_each([&](Line* l) {
      if (l->updates > 0) stage_push(l);
    });
    flush_pending();
  }

  int64_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return (int64_t)map_.size();
  }
  // drop every cached line without pushing (after the server's table was
  // replaced, e.g. a checkpoint load): the next lookup re-pulls all rows
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    make_policy();
    map_.clear();
    pool_.reset();
    evicted_.clear();
  }
  void set_bounds(int64_t pull, int64_t push) { pull_bound_ = pull; push_bound_ = push; }
  void set_bypass(bool b) { bypass_ = b; }
  void set_perf(bool b) { perf_ = b; }
  void get_perf(double* out) {
    std::lock_guard<std::mutex> g(mu_);
    out[0] = (double)perf_rec_.calls; out[1] = (double)perf_rec_.unique; out[2] = (double)perf_rec_.miss;
    out[3] = (double)perf_rec_.transfer; out[4] = (double)perf_rec_.evict; out[5] = (double)perf_rec_.pushed;
    out[6] = perf_rec_.t_unique; out[7] = perf_rec_.t_sync; out[8] = perf_rec_.t_copy; out[9] = perf_rec_.t_push;
  }

 private:
  void make_policy() {
    if (policy_ == 0) pol_.reset(new LRU());
    else pol_.reset(new LFU(policy_ == 2));
  }
  void admit(Line* l) {
    while ((int64_t)map_.size() >= limit_ && map_.size() > 0) {
      Line* v = pol_->evict();
      if (!v) break;
      perf_rec_.evict++;
      if (v->updates > 0) stage_push(v);
      map_.erase(v->key);
      v->cached = false;
      evicted_.push_back(v);   // freed after this call: lines_ may still point to it
    }
    pol_->insert(l);
    map_.insert(l->key, l);
    l->cached = true;
  }
  void release_evicted() {
    for (Line* v : evicted_) pool_.put(v);
    evicted_.clear();
  }
  void stage_push(Line* l) {
    prow_.push_back(l->key);
    pupd_.push_back(l->updates);
    pdata_.insert(pdata_.end(), l->grad, l->grad + width_);
    l->ver += l->updates;
    l->updates = 0;
    memset(l->grad, 0, width_ * sizeof(float));
  }
  void flush_pending() {
    if (prow_.empty()) return;
    auto t0 = std::chrono::steady_clock::now();
    hps_push_embedding(key_, prow_.data(), (int64_t)prow_.size(), pdata_.data(), pupd_.data());
    perf_rec_.pushed += (int64_t)prow_.size();
    perf_rec_.t_push += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    prow_.clear();
    pupd_.clear();
    pdata_.clear();
  }

  int64_t limit_, rows_, width_;
  int key_;
  int64_t pull_bound_, push_bound_;
  int policy_;
  bool bypass_ = false, perf_ = false;
  LinePool pool_;
  std::unique_ptr<Policy> pol_;
  KeyMap map_;
  std::vector<Line*> evicted_;
  // per-call scratch, kept to avoid reallocation
  std::vector<int64_t> uniq_, vers_, idx_, nver_, ukeys_, prow_, pupd_;
  std::vector<int32_t> pos_;
  std::vector<int64_t> slot_, start_, fill_, order_;
  Dedup dedup_;
  std::vector<Line*> lines_, ulines_;
  std::vector<float> sync_data_, acc_, pdata_;
  std::mutex mu_;
  Perf perf_rec_;
};

// async executor (the reference's ThreadPool(5) in front of the cache)
class Exec {
 public:
  Exec() {
    for (int i = 0; i < 2; ++i) th_.emplace_back([this] { run(); });
  }
  ~Exec() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int64_t submit(std::function<void()> f) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t t = ++next_;
    pending_[t] = 1;
    q_.emplace_back(t, std::move(f));
    cv_.notify_one();
    return t;
  }
  void wait(int64_t t) {
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return pending_.find(t) == pending_.end(); });
  }
  void drain() {
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return pending_.empty(); });
  }

 private:
  void run() {
    for (;;) {
      std::pair<int64_t, std::function<void()>> j;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        j = std::move(q_.front());
        q_.pop_front();
      }
      j.second();
      {
        std::lock_guard<std::mutex> g(mu_);
        pending_.erase(j.first);
      }
      done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::deque<std::pair<int64_t, std::function<void()>>> q_;
  std::map<int64_t, int> pending_;
  std::vector<std::thread> th_;
  int64_t next_ = 0;
  bool stop_ = false;
};

static std::mutex g_mu;
static std::vector<std::unique_ptr<Cache>> g_caches;
static Exec* g_exec = nullptr;

static Cache* get(int h) {
  std::lock_guard<std::mutex> g(g_mu);
  return (h >= 0 && h < (int)g_caches.size()) ? g_caches[h].get() : nullptr;
}
static Exec* exec() {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_exec) g_exec = new Exec();
  return g_exec;
}

}  // namespace hc

using namespace hc;

extern "C" {

// Self-test of the fork-join pool: alternating parallel regions of
// different sizes, each element must be visited exactly once per region.  Returns
// the number of mis-visited elements (0 = OK).  Driven by the TSan binary
// (csrc/tests/runtime_sanitize.cc) and tests/test_sanitizers_cpu.py.
int64_t hc_parallel_for_selftest(int iters) {
  int64_t bad = 0;
  std::vector<std::atomic<int>> hits(1 << 16);
  for (int it = 0; it < iters; ++it) {
    const int64_t n = (it & 1) ? 4096 + (it % 7) * 1531 : 1024 + (it % 5) * 377;
    for (int64_t i = 0; i < n; ++i) hits[i].store(0, std::memory_order_relaxed);
    pool().run(n, 256, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) hits[i].fetch_add(1, std::memory_order_relaxed);
    });
    for (int64_t i = 0; i < n; ++i) bad += hits[i].load(std::memory_order_relaxed) != 1;
  }
  return bad;
}

// wait for every queued cache operation (called by hps_finalize before the PS
// segment is unmapped, so no cache thread can touch it afterwards)
void hc_drain_all() {
  Exec* e;
  {
    std::lock_guard<std::mutex> g(g_mu);
    e = g_exec;
  }
  if (e) e->drain();
}

// policy: 0 LRU, 1 LFU, 2 LFUOpt
int hc_create(int policy, int64_t limit, int64_t rows, int64_t width, int key, int64_t pull_bound,
              int64_t push_bound) {
  std::lock_guard<std::mutex> g(g_mu);
  g_caches.emplace_back(new Cache(policy, limit, rows, width, key, pull_bound, push_bound));
  return (int)g_caches.size() - 1;
}
int hc_lookup(int h, const int64_t* keys, int64_t n, float* dest) {
  Cache* c = get(h);
  if (!c) return -1;
  c->lookup(keys, n, dest);
  return 0;
}
int hc_update(int h, const int64_t* keys, int64_t n, const float* grads) {
  Cache* c = get(h);
  if (!c) return -1;
  c->update(keys, n, grads);
  return 0;
}
int64_t hc_async_lookup(int h, const int64_t* keys, int64_t n, float* dest) {
  Cache* c = get(h);
  return exec()->submit([=] { c->lookup(keys, n, dest); });
}
int64_t hc_async_update(int h, const int64_t* keys, int64_t n, const float* grads) {
  Cache* c = get(h);
  return exec()->submit([=] { c->update(keys, n, grads); });
}
// push grads of the current batch, then pull the NEXT batch's rows (prefetch)
int64_t hc_async_push_pull(int h, const int64_t* pull_keys, int64_t npull, float* dest,
                           const int64_t* push_keys, int64_t npush, const float* grads) {
  Cache* c = get(h);
  return exec()->submit([=] {
    if (npush > 0) c->update(push_keys, npush, grads);
    if (npull > 0) c->lookup(pull_keys, npull, dest);
  });
}
int hc_wait(int64_t ticket) {
  exec()->wait(ticket);
  return 0;
}
int hc_flush(int h) {
  Cache* c = get(h);
  if (!c) return -1;
  c->flush_all();
  return 0;
}
int hc_clear(int h) {
  Cache* c = get(h);
  if (!c) return -1;
  c->clear();
  return 0;
}
int64_t hc_size(int h) {
  Cache* c = get(h);
  return c ? c->size() : -1;
}
int hc_set_bounds(int h, int64_t pull, int64_t push) {
  Cache* c = get(h);
  if (!c) return -1;
  c->set_bounds(pull, push);
  return 0;
}
int hc_set_bypass(int h, int b) {
  Cache* c = get(h);
  if (!c) return -1;
  c->set_bypass(b != 0);
  return 0;
}
int hc_set_perf(int h, int b) {
  Cache* c = get(h);
  if (!c) return -1;
  c->set_perf(b != 0);
  return 0;
}
int hc_get_perf(int h, double* out10) {
  Cache* c = get(h);
  if (!c) return -1;
  c->get_perf(out10);
  return 0;
}
}
