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
#include <chrono>
#include <condition_variable>
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

struct Line {
  int64_t key;
  int64_t ver;      // server version this line reflects
  int64_t updates;  // local updates not yet pushed
  int64_t freq;
  std::vector<float> data;
  std::vector<float> grad;
};
using LineP = std::shared_ptr<Line>;

class Policy {
 public:
  virtual ~Policy() {}
  virtual LineP find(int64_t k) = 0;
  virtual void touch(const LineP& l) = 0;
  virtual void insert(const LineP& l) = 0;
  virtual LineP evict() = 0;  // removes and returns the victim
  virtual size_t size() const = 0;
};

class LRU : public Policy {
 public:
  LineP find(int64_t k) override {
    auto it = map_.find(k);
    return it == map_.end() ? nullptr : *it->second;
  }
  void touch(const LineP& l) override {
    auto it = map_.find(l->key);
    lst_.splice(lst_.begin(), lst_, it->second);
  }
  void insert(const LineP& l) override {
    lst_.push_front(l);
    map_[l->key] = lst_.begin();
  }
  LineP evict() override {
    LineP v = lst_.back();
    map_.erase(v->key);
    lst_.pop_back();
    return v;
  }
  size_t size() const override { return map_.size(); }

 private:
  std::list<LineP> lst_;
  std::unordered_map<int64_t, std::list<LineP>::iterator> map_;
};

class LFU : public Policy {
 public:
  explicit LFU(bool opt) : opt_(opt) {}
  LineP find(int64_t k) override {
    auto it = map_.find(k);
    return it == map_.end() ? nullptr : it->second.line;
  }
  void touch(const LineP& l) override {
    auto& ent = map_[l->key];
    auto& bucket = buckets_[l->freq];
    bucket.erase(ent.it);
    if (bucket.empty()) buckets_.erase(l->freq);
    l->freq += 1;
    auto& nb = buckets_[l->freq];
    nb.push_front(l);
    ent.it = nb.begin();
  }
  void insert(const LineP& l) override {
    // LFUOpt: a new line enters at the minimum live frequency instead of 1, so a
    // burst of new keys does not immediately evict each other
    if (opt_ && !buckets_.empty()) l->freq = std::max<int64_t>(l->freq, buckets_.begin()->first);
    auto& b = buckets_[l->freq];
    b.push_front(l);
    map_[l->key] = Ent{l, b.begin()};
  }
  LineP evict() override {
    auto bit = buckets_.begin();
    LineP v = bit->second.back();
    bit->second.pop_back();
    if (bit->second.empty()) buckets_.erase(bit);
    map_.erase(v->key);
    return v;
  }
  size_t size() const override { return map_.size(); }

 private:
  struct Ent {
    LineP line;
    std::list<LineP>::iterator it;
  };
  bool opt_;
  std::map<int64_t, std::list<LineP>> buckets_;
  std::unordered_map<int64_t, Ent> map_;
};

struct Perf {
  int64_t calls = 0, unique = 0, miss = 0, transfer = 0, evict = 0, pushed = 0;
  double t_unique = 0, t_sync = 0, t_copy = 0, t_push = 0;
};

class Cache {
 public:
  Cache(int policy, int64_t limit, int64_t rows, int64_t width, int key, int64_t pull_bound,
        int64_t push_bound)
      : limit_(limit), rows_(rows), width_(width), key_(key), pull_bound_(pull_bound),
        push_bound_(push_bound), policy_(policy) {
    if (policy == 0) pol_.reset(new LRU());
    else pol_.reset(new LFU(policy == 2));
  }

  void lookup(const int64_t* keys, int64_t n, float* dest) {
    std::lock_guard<std::mutex> g(mu_);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<int64_t> uniq(keys, keys + n);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    auto t1 = std::chrono::steady_clock::now();
    const int64_t u = (int64_t)uniq.size();
    std::vector<int64_t> vers(u);
    std::vector<LineP> lines(u);
    int64_t miss = 0;
    for (int64_t i = 0; i < u; ++i) {
      lines[i] = pol_->find(uniq[i]);
      vers[i] = lines[i] ? lines[i]->ver : -1;
      if (!lines[i]) ++miss;
    }
    if (bypass_) std::fill(vers.begin(), vers.end(), -1);
    std::vector<int64_t> idx(u), nver(u);
    std::vector<float> data((size_t)u * width_);
    int64_t cnt = hps_sync_embedding(key_, uniq.data(), u, vers.data(), pull_bound_, idx.data(),
                                     nver.data(), data.data());
    auto t2 = std::chrono::steady_clock::now();
    for (int64_t c = 0; c < std::max<int64_t>(cnt, 0); ++c) {
      int64_t i = idx[c];
      LineP& l = lines[i];
      const float* src = data.data() + c * width_;
      if (!l) {
        l = std::make_shared<Line>();
        l->key = uniq[i];
        l->updates = 0;
        l->freq = 1;
        l->data.assign(src, src + width_);
        l->grad.assign(width_, 0.f);
        l->ver = nver[c];
        admit(l);
      } else {
        // server copy + our pending (unpushed) gradient
        for (int64_t j = 0; j < width_; ++j) l->data[j] = src[j] + l->grad[j];
        l->ver = nver[c];
      }
    }
    for (int64_t i = 0; i < u; ++i)
      if (lines[i] && pol_->find(uniq[i])) pol_->touch(lines[i]);
    std::unordered_map<int64_t, int64_t> pos;
    pos.reserve(u * 2);
    for (int64_t i = 0; i < u; ++i) pos[uniq[i]] = i;
    for (int64_t r = 0; r < n; ++r) {
      const LineP& l = lines[pos[keys[r]]];
      if (l) memcpy(dest + r * width_, l->data.data(), width_ * sizeof(float));
      else memset(dest + r * width_, 0, width_ * sizeof(float));
    }
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
    std::unordered_map<int64_t, std::vector<float>> acc;
    acc.reserve(n * 2);
    for (int64_t r = 0; r < n; ++r) {
      auto& v = acc[keys[r]];
      if (v.empty()) v.assign(width_, 0.f);
      const float* gr = grads + r * width_;
      for (int64_t j = 0; j < width_; ++j) v[j] += gr[j];
    }
    std::vector<int64_t> prow, pupd;
    std::vector<float> pdata;
    for (auto& kv : acc) {
      LineP l = pol_->find(kv.first);
      if (!l || bypass_) {
        // not cached: push straight through
        prow.push_back(kv.first);
        pupd.push_back(1);
        pdata.insert(pdata.end(), kv.second.begin(), kv.second.end());
        continue;
      }
      for (int64_t j = 0; j < width_; ++j) {
        l->data[j] += kv.second[j];
        l->grad[j] += kv.second[j];
      }
      l->updates += 1;
      if (l->updates > push_bound_) stage_push(l, prow, pupd, pdata);
    }
    flush(prow, pupd, pdata);
  }

  void flush_all() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> prow, pupd;
    std::vector<float> pdata;
    for (auto& l : all_lines()) if (l->updates > 0) stage_push(l, prow, pupd, pdata);
    flush(prow, pupd, pdata);
  }

  int64_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return (int64_t)pol_->size();
  }
  // drop every cached line without pushing (after the server's table was
  // replaced, e.g. a checkpoint load): the next lookup re-pulls all rows
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    if (policy_ == 0) pol_.reset(new LRU());
    else pol_.reset(new LFU(policy_ == 2));
    live_.clear();
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
  void admit(const LineP& l) {
    while ((int64_t)pol_->size() >= limit_ && pol_->size() > 0) {
      LineP v = pol_->evict();
      perf_rec_.evict++;
      if (v->updates > 0) {
        std::vector<int64_t> prow, pupd;
        std::vector<float> pdata;
        stage_push(v, prow, pupd, pdata);
        flush(prow, pupd, pdata);
      }
      live_.erase(v->key);
    }
    pol_->insert(l);
    live_[l->key] = l;
  }
  std::vector<LineP> all_lines() {
    std::vector<LineP> out;
    for (auto& kv : live_) out.push_back(kv.second);
    return out;
  }
  void stage_push(const LineP& l, std::vector<int64_t>& prow, std::vector<int64_t>& pupd,
                  std::vector<float>& pdata) {
    prow.push_back(l->key);
    pupd.push_back(l->updates);
    pdata.insert(pdata.end(), l->grad.begin(), l->grad.end());
    l->ver += l->updates;
    l->updates = 0;
    std::fill(l->grad.begin(), l->grad.end(), 0.f);
  }
  void flush(std::vector<int64_t>& prow, std::vector<int64_t>& pupd, std::vector<float>& pdata) {
    if (prow.empty()) return;
    auto t0 = std::chrono::steady_clock::now();
    hps_push_embedding(key_, prow.data(), (int64_t)prow.size(), pdata.data(), pupd.data());
    perf_rec_.pushed += (int64_t)prow.size();
    perf_rec_.t_push += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    prow.clear();
    pupd.clear();
    pdata.clear();
  }

  int64_t limit_, rows_, width_;
  int key_;
  int64_t pull_bound_, push_bound_;
  int policy_;
  bool bypass_ = false, perf_ = false;
  std::unique_ptr<Policy> pol_;
  std::unordered_map<int64_t, LineP> live_;
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
