// Single-node parameter server over POSIX shared memory.  See shm_ps.h.
#include "shm_ps.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <unordered_set>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace hps {

constexpr uint64_t kMagic = 0x4845545550530001ull;  // "HETUPS" v1
constexpr int kMaxNodes = 256;
constexpr int kMaxParams = 4096;
constexpr int kMaxSsp = 64;
constexpr int kMaxPreduce = 64;
constexpr int kStripes = 1 << 16;
constexpr int kPsfKinds = 16;

enum Psf { DENSE_PULL, DENSE_PUSH, DD_PUSHPULL, SPARSE_PULL, SPARSE_PUSH, SD_PUSHPULL, SS_PUSHPULL,
           PUSH_EMB, SYNC_EMB, PARAM_INIT, SAVE, LOAD, SSP_SYNC, PREDUCE, BARRIER, CLEAR };

struct ParamEntry {
  std::atomic<int32_t> state;  // 0 empty, 1 initialising, 2 ready
  int32_t key;
  int32_t ptype;
  int32_t pad;
  int64_t rows, width;
  uint64_t data_off, ver_off;
};

struct SspState {
  std::atomic<int32_t> used;
  int32_t key, group_size;
  int64_t tolerance;
  std::atomic<int64_t> clocks[kMaxNodes];
};

struct PReduceState {
  std::atomic<int32_t> used;
  int32_t key;
  std::atomic<uint32_t> lock;
  int32_t required;
  int64_t gen;            // group generation (bumped when a group closes)
  int64_t open_since_ns;  // first arrival of the open group
  float wait_ms;
  int32_t nmembers;
  int32_t members[kMaxNodes];
  int32_t closed_members[kMaxNodes];
  int32_t closed_n;
};

struct Header {
  uint64_t magic;
  int32_t nworkers, nservers;
  uint64_t heap_off, heap_size;
  std::atomic<uint64_t> heap_top;
  std::atomic<int32_t> next_worker;
  std::atomic<int32_t> finalized;
  std::atomic<int32_t> bar_count;
  std::atomic<int32_t> bar_gen;
  std::atomic<uint32_t> dir_lock;
  std::atomic<int64_t> heartbeat[kMaxNodes];
  std::atomic<int32_t> recovered;   // workers that took over a dead rank
  std::atomic<int32_t> hb_on;       // some worker refreshes its heartbeat (PS_HEARTBEAT_INTERVAL > 0)
  SspState ssp[kMaxSsp];
  PReduceState pre[kMaxPreduce];
  ParamEntry params[kMaxParams];
  std::atomic<uint32_t> stripes[kStripes];
};

// ------------------------------------------------------------------ process state
static Header* H = nullptr;
static char* BASE = nullptr;
static size_t MAP_BYTES = 0;
static int ROLE = -1;
static int RANK = -1;
static std::string NAME;
static double DROP_P = 0.0;
static int RESEND = 0;
static int RESEND_MS = 1000;

static int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

static inline void spin_lock(std::atomic<uint32_t>& l) {
  int spins = 0;
  uint32_t exp = 0;
  while (!l.compare_exchange_weak(exp, 1, std::memory_order_acquire)) {
    exp = 0;
    if (++spins > 64) { std::this_thread::yield(); spins = 0; }
  }
}
static inline void spin_unlock(std::atomic<uint32_t>& l) { l.store(0, std::memory_order_release); }

static inline std::atomic<uint32_t>& stripe(int key, int64_t row) {
  uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull ^ (uint64_t)row * 0xC2B2AE3D27D4EB4Full;
  return H->stripes[(h >> 17) & (kStripes - 1)];
}

static ParamEntry* find_param(int key, bool create) {
  uint32_t h = (uint32_t)key * 2654435761u;
  for (int i = 0; i < kMaxParams; ++i) {
    ParamEntry& e = H->params[(h + i) % kMaxParams];
    int st = e.state.load(std::memory_order_acquire);
    if (st != 0 && e.key == key) return &e;
    if (st == 0) {
      if (!create) return nullptr;
      spin_lock(H->dir_lock);
      // re-check under the directory lock
      for (int j = 0; j < kMaxParams; ++j) {
        ParamEntry& f = H->params[(h + j) % kMaxParams];
        int s2 = f.state.load(std::memory_order_acquire);
        if (s2 != 0 && f.key == key) { spin_unlock(H->dir_lock); return &f; }
        if (s2 == 0) {
          f.key = key;
          f.state.store(1, std::memory_order_release);
          spin_unlock(H->dir_lock);
          return &f;
        }
      }
      spin_unlock(H->dir_lock);
      return nullptr;
    }
  }
  return nullptr;
}

static uint64_t heap_alloc(uint64_t bytes) {
  bytes = (bytes + 63) & ~63ull;
  uint64_t off = H->heap_top.fetch_add(bytes);
  if (off + bytes > H->heap_size) return ~0ull;
  return H->heap_off + off;
}

static inline float* pdata(ParamEntry* e) { return (float*)(BASE + e->data_off); }
static inline int64_t* pver(ParamEntry* e) { return (int64_t*)(BASE + e->ver_off); }

static ParamEntry* ready_param(int key) {
  ParamEntry* e = find_param(key, false);
  if (!e) return nullptr;
  while (e->state.load(std::memory_order_acquire) != 2) std::this_thread::yield();
  return e;
}

// ------------------------------------------------------------------ load recording
static std::atomic<int64_t> g_cnt[kPsfKinds];
static std::atomic<int64_t> g_bytes[kPsfKinds];
static bool g_record = false;
static inline void rec(int psf, int64_t bytes) {
  if (!g_record) return;
  g_cnt[psf].fetch_add(1);
  g_bytes[psf].fetch_add(bytes);
}

// Fault injection and reliable delivery (reference ps-lite van.cc:362-443, resender.h:15-150;
// SURVEY §5.3).  PS_DROP_MSG=<percent> loses a message: either the REQUEST (the PSF never
// runs) or its ACK (the PSF ran but the sender does not know).  Without PS_RESEND the
// caller gets -EIO.  With PS_RESEND=1 the sender re-sends after PS_RESEND_TIMEOUT ms, up
// to 10 times, and every message carries a (sender, sequence) id: the receiving side keeps
// the ids it has applied, so a re-sent message whose first copy was applied (lost ack) is
// acknowledged again but NOT re-applied -- each request takes effect exactly once.
static std::atomic<int64_t> g_fault[4];   // dropped requests, dropped acks, resends, duplicates
static std::atomic<uint64_t> g_msg_seq{1};
static std::mutex g_applied_mu;
static std::unordered_set<uint64_t> g_applied;   // ids applied of messages still in delivery

static thread_local std::mt19937_64 tl_rng(std::random_device{}());
static bool drop_now() {
  if (DROP_P <= 0.0) return false;
  std::uniform_real_distribution<double> u(0.0, 100.0);
  return u(tl_rng) < DROP_P;
}

template <typename F>
static int deliver(F&& body) {
  if (DROP_P <= 0.0) return body();
  const uint64_t id = g_msg_seq.fetch_add(1);
  // the sender learns the final outcome in this process, so the id leaves the applied set
  // when deliver returns: the set holds only messages still between resends
  auto done = [id](int r) {
    std::lock_guard<std::mutex> g(g_applied_mu);
    g_applied.erase(id);
    return r;
  };
  int applied_r = 0;
  for (int attempt = 0;; ++attempt) {
    if (attempt > 0) {
      g_fault[2].fetch_add(1);
      std::this_thread::sleep_for(std::chrono::milliseconds(RESEND_MS));
    }
    if (drop_now()) {                       // the request is lost on the way
      g_fault[0].fetch_add(1);
    } else {
      bool dup;
      {
        std::lock_guard<std::mutex> g(g_applied_mu);
        dup = !g_applied.insert(id).second;
      }
      if (dup) g_fault[3].fetch_add(1);     // receiver suppresses the re-sent copy
      else applied_r = body();
      if (!drop_now()) return done(applied_r);   // ack arrives
      g_fault[1].fetch_add(1);              // the ack is lost
    }
    if (!RESEND) return done(-EIO);
    if (attempt >= 10) return done(-ETIMEDOUT);
  }
}

// ------------------------------------------------------------------ thread pool
class Pool {
 public:
  explicit Pool(int n) : stop_(false) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int64_t submit(int key, std::function<int()> f) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t t = ++next_;
    pending_[t] = key;
    q_.emplace_back(t, std::move(f));
    cv_.notify_one();
    return t;
  }
  int wait(int64_t t) {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return pending_.find(t) == pending_.end(); });
    auto it = results_.find(t);
    int r = 0;
    if (it != results_.end()) { r = it->second; results_.erase(it); }
    return r;
  }
  int wait_key(int key) {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] {
      for (auto& kv : pending_) if (kv.second == key) return false;
      return true;
    });
    return 0;
  }

 private:
  void run() {
    for (;;) {
      std::pair<int64_t, std::function<int()>> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      int r = job.second();
      {
        std::lock_guard<std::mutex> g(mu_);
        pending_.erase(job.first);
        if (r != 0) results_[job.first] = r;
      }
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::pair<int64_t, std::function<int()>>> q_;
  std::map<int64_t, int> pending_;
  std::unordered_map<int64_t, int> results_;
  std::vector<std::thread> th_;
  int64_t next_ = 0;
  bool stop_;
};

static Pool* POOL = nullptr;
static std::thread* HB = nullptr;
static std::atomic<bool> HB_STOP{false};

// ------------------------------------------------------------------ init helpers
static void fill_init(float* d, int64_t n, int init_type, double a, double b, uint64_t seed) {
  int nth = (int)std::min<int64_t>(16, std::max<int64_t>(1, n / (1 << 20)));
  std::vector<std::thread> ts;
  for (int t = 0; t < nth; ++t) {
    ts.emplace_back([=] {
      int64_t lo = n * t / nth, hi = n * (t + 1) / nth;
      std::mt19937_64 rng(seed * 1000003ull + (uint64_t)t * 7919ull + 17);
      if (init_type == 0) {
        for (int64_t i = lo; i < hi; ++i) d[i] = (float)a;
      } else if (init_type == 1) {
        std::uniform_real_distribution<float> u((float)a, (float)b);
        for (int64_t i = lo; i < hi; ++i) d[i] = u(rng);
      } else if (init_type == 2) {
        std::normal_distribution<float> nd((float)a, (float)b);
        for (int64_t i = lo; i < hi; ++i) d[i] = nd(rng);
      } else {
        std::normal_distribution<float> nd(0.f, 1.f);
        for (int64_t i = lo; i < hi; ++i) {
          float v;
          do { v = nd(rng); } while (std::fabs(v) > 2.f);
          d[i] = (float)a + (float)b * v;
        }
      }
    });
  }
  for (auto& t : ts) t.join();
}

}  // namespace hps

using namespace hps;

extern "C" {

void hc_drain_all();

int hps_init(int role, const char* name, int num_workers, int num_servers, uint64_t heap_bytes) {
  if (H) return 0;
  ROLE = role;
  NAME = name ? name : "/hetu_ps";
  if (const char* d = getenv("PS_DROP_MSG")) DROP_P = atof(d);
  if (const char* r = getenv("PS_RESEND")) RESEND = atoi(r);
  if (const char* t = getenv("PS_RESEND_TIMEOUT")) RESEND_MS = atoi(t);
  size_t hdr = (sizeof(Header) + 4095) & ~(size_t)4095;
  int fd = -1;
  if (role == 1) {
    shm_unlink(NAME.c_str());
    fd = shm_open(NAME.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return -errno;
    MAP_BYTES = hdr + heap_bytes;
    if (ftruncate(fd, (off_t)MAP_BYTES) != 0) { close(fd); return -errno; }
  } else {
    // wait for the server to create the segment
    for (int i = 0; i < 6000; ++i) {
      fd = shm_open(NAME.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        fstat(fd, &st);
        if ((size_t)st.st_size >= hdr) {
          MAP_BYTES = (size_t)st.st_size;
          Header* probe = (Header*)mmap(nullptr, hdr, PROT_READ, MAP_SHARED, fd, 0);
          bool ok = probe != MAP_FAILED && probe->magic == kMagic;
          if (probe != MAP_FAILED) munmap(probe, hdr);
          if (ok) break;
        }
        close(fd);
        fd = -1;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    if (fd < 0) return -ENOENT;
  }
  void* p = mmap(nullptr, MAP_BYTES, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -errno;
  BASE = (char*)p;
  H = (Header*)p;
  if (role == 1) {
    memset((void*)H, 0, sizeof(Header));
    H->nworkers = num_workers;
    H->nservers = num_servers;
    H->heap_off = hdr;
    H->heap_size = heap_bytes;
    std::atomic_thread_fence(std::memory_order_release);
    H->magic = kMagic;
  } else if (role == 2) {
    RANK = H->next_worker.fetch_add(1);
    if (RANK >= H->nworkers) {
      // node recovery (reference van.cc:132-160 is_recovery): the cluster is full, so
      // this process replaces a worker whose heartbeat is older than PS_HEARTBEAT_TIMEOUT.
      // Only when heartbeats are live (some worker refreshes them, or the timeout is set
      // explicitly): otherwise every worker's heartbeat is its start time and a live
      // worker would look dead (ps-lite reports no dead nodes at timeout 0, its default).
      const char* ts = getenv("PS_HEARTBEAT_TIMEOUT");
      const double to = ts ? atof(ts) : 60.0;
      RANK = -1;
      if (to > 0 && (ts || H->hb_on.load())) {
        int dead[kMaxNodes];
        const int nd = hps_dead_nodes(to, dead, kMaxNodes);
        // claim a dead rank by moving its stale heartbeat to now: a concurrent joiner
        // that read the same stale value loses the exchange and tries the next one
        for (int i = 0; i < nd && RANK < 0; ++i) {
          int64_t stale = H->heartbeat[dead[i]].load();
          if (now_ns() - stale > (int64_t)(to * 1e9) &&
              H->heartbeat[dead[i]].compare_exchange_strong(stale, now_ns()))
            RANK = dead[i];
        }
      }
      if (RANK < 0) {
        munmap(p, MAP_BYTES);
        H = nullptr;
        return -EBUSY;
      }
      H->recovered.fetch_add(1);
    }
    int nth = 4;
    if (const char* s = getenv("HETU_PS_THREADS")) nth = std::max(1, atoi(s));
    POOL = new Pool(nth);
    double iv = 0.0;
    if (const char* s = getenv("PS_HEARTBEAT_INTERVAL")) iv = atof(s);
    H->heartbeat[RANK].store(now_ns());
    if (iv > 0) {
      H->hb_on.store(1);
      HB = new std::thread([iv] {
        while (!HB_STOP.load()) {
          hps_heartbeat();
          std::this_thread::sleep_for(std::chrono::milliseconds((int)(iv * 1000)));
        }
      });
    }
  }
  if (const char* dir = getenv("HETU_PS_RECORD")) hps_start_record(dir);
  return 0;
}

int hps_finalize() {
  if (!H) return 0;
  const bool dbg = getenv("HETU_PS_DEBUG") != nullptr;
  if (dbg) fprintf(stderr, "[hps] finalize role=%d\n", ROLE);
  hc_drain_all();
  if (HB) {
    HB_STOP = true;
    HB->join();
    delete HB;
    HB = nullptr;
  }
  if (POOL) {
    delete POOL;
    POOL = nullptr;
  }
  if (dbg) fprintf(stderr, "[hps] pool stopped\n");
  if (ROLE == 2) H->finalized.fetch_add(1);
  if (dbg) fprintf(stderr, "[hps] finalized count bumped\n");
  munmap(BASE, MAP_BYTES);
  if (ROLE == 1) shm_unlink(NAME.c_str());
  H = nullptr;
  BASE = nullptr;
  return 0;
}

int hps_rank() { return RANK; }
int hps_nrank() { return H ? H->nworkers : 0; }

int hps_server_wait_shutdown(double timeout_s) {
  if (!H) return -1;
  int64_t end = now_ns() + (int64_t)(timeout_s * 1e9);
  while (H->finalized.load() < H->nworkers) {
    if (timeout_s > 0 && now_ns() > end) return -ETIMEDOUT;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  return 0;
}

int hps_param_init(int key, int ptype, int64_t rows, int64_t width, int init_type, double a,
                   double b, uint64_t seed) {
  ParamEntry* e = find_param(key, true);
  if (!e) return -ENOMEM;
  // the creator (state 1 set by us under dir lock with data_off == 0) initialises
  spin_lock(stripe(key, -1));
  bool mine = e->data_off == 0 && e->state.load() == 1;
  if (mine) {
    e->ptype = ptype;
    e->rows = rows;
    e->width = width;
    uint64_t off = heap_alloc((uint64_t)rows * width * sizeof(float));
    uint64_t voff = ptype == 2 ? heap_alloc((uint64_t)rows * sizeof(int64_t)) : 0;
    if (off == ~0ull || voff == ~0ull) { spin_unlock(stripe(key, -1)); return -ENOMEM; }
    e->ver_off = voff;
    e->data_off = off;
  }
  spin_unlock(stripe(key, -1));
  if (mine) {
    fill_init(pdata(e), rows * width, init_type, a, b, seed);
    if (ptype == 2) memset(pver(e), 0, rows * sizeof(int64_t));
    e->state.store(2, std::memory_order_release);
  } else {
    while (e->state.load(std::memory_order_acquire) != 2) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  rec(PARAM_INIT, 0);
  return 0;
}

int hps_param_clear(int key) {
  ParamEntry* e = ready_param(key);
  if (!e) return -ENOENT;
  memset(pdata(e), 0, e->rows * e->width * sizeof(float));
  if (e->ptype == 2) memset(pver(e), 0, e->rows * sizeof(int64_t));
  rec(CLEAR, 0);
  return 0;
}

int64_t hps_param_rows(int key) {
  ParamEntry* e = ready_param(key);
  return e ? e->rows : -1;
}
int64_t hps_param_width(int key) {
  ParamEntry* e = ready_param(key);
  return e ? e->width : -1;
}

// dense ops operate on 4096-float chunks, each under its stripe lock
static void dense_apply(ParamEntry* e, const float* in, float* out, int64_t len) {
  float* d = pdata(e);
  const int64_t C = 4096;
  for (int64_t c0 = 0; c0 < len; c0 += C) {
    int64_t c1 = std::min(len, c0 + C);
    auto& l = stripe(e->key, c0 / C);
    spin_lock(l);
    if (in) for (int64_t i = c0; i < c1; ++i) d[i] += in[i];
    if (out) memcpy(out + c0, d + c0, (c1 - c0) * sizeof(float));
    spin_unlock(l);
  }
}

int hps_dense_pull(int key, float* out, int64_t len) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e) return -ENOENT;
    dense_apply(e, nullptr, out, std::min<int64_t>(len, e->rows * e->width));
    rec(DENSE_PULL, len * 4);
    return 0;
  });
}

int hps_dense_push(int key, const float* in, int64_t len) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e) return -ENOENT;
    dense_apply(e, in, nullptr, std::min<int64_t>(len, e->rows * e->width));
    rec(DENSE_PUSH, len * 4);
    return 0;
  });
}

int hps_dd_pushpull(int key, const float* in, float* out, int64_t len) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e) return -ENOENT;
    dense_apply(e, in, out, std::min<int64_t>(len, e->rows * e->width));
    rec(DD_PUSHPULL, len * 8);
    return 0;
  });
}

int hps_sparse_pull(int key, const int64_t* ids, int64_t n, float* out) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e) return -ENOENT;
    const int64_t w = e->width;
    float* d = pdata(e);
    for (int64_t i = 0; i < n; ++i) {
      int64_t r = ids[i];
      if (r < 0 || r >= e->rows) { memset(out + i * w, 0, w * sizeof(float)); continue; }
      auto& l = stripe(key, r);
      spin_lock(l);
      memcpy(out + i * w, d + r * w, w * sizeof(float));
      spin_unlock(l);
    }
    rec(SPARSE_PULL, n * (8 + w * 4));
    return 0;
  });
}

int hps_sparse_push(int key, const int64_t* ids, int64_t n, const float* vals) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e) return -ENOENT;
    const int64_t w = e->width;
    float* d = pdata(e);
    for (int64_t i = 0; i < n; ++i) {
      int64_t r = ids[i];
      if (r < 0 || r >= e->rows) continue;
      auto& l = stripe(key, r);
      spin_lock(l);
      float* row = d + r * w;
      const float* v = vals + i * w;
      for (int64_t j = 0; j < w; ++j) row[j] += v[j];
      spin_unlock(l);
    }
    rec(SPARSE_PUSH, n * (8 + w * 4));
    return 0;
  });
}

int hps_sd_pushpull(int key, const int64_t* ids, int64_t n, const float* vals, float* dense_out,
                    int64_t len) {
  int r = hps_sparse_push(key, ids, n, vals);
  if (r) return r;
  return hps_dense_pull(key, dense_out, len);
}

int hps_ss_pushpull(int key, const int64_t* in_ids, int64_t nin, const float* vals,
                    const int64_t* out_ids, int64_t nout, float* out) {
  int r = hps_sparse_push(key, in_ids, nin, vals);
  if (r) return r;
  return hps_sparse_pull(key, out_ids, nout, out);
}

int hps_push_embedding(int key, const int64_t* rows, int64_t n, const float* data,
                       const int64_t* updates) {
  return deliver([&] {
    ParamEntry* e = ready_param(key);
    if (!e || e->ptype != 2) return -EINVAL;
    const int64_t w = e->width;
    float* d = pdata(e);
    int64_t* ver = pver(e);
    for (int64_t i = 0; i < n; ++i) {
      int64_t r = rows[i];
      if (r < 0 || r >= e->rows) continue;
      auto& l = stripe(key, r);
      spin_lock(l);
      ver[r] += updates[i];
      float* row = d + r * w;
      const float* v = data + i * w;
      for (int64_t j = 0; j < w; ++j) row[j] += v[j];
      spin_unlock(l);
    }
    rec(PUSH_EMB, n * (16 + w * 4));
    return 0;
  });
}

int64_t hps_sync_embedding(int key, const int64_t* rows, int64_t n, const int64_t* vers,
                           int64_t bound, int64_t* out_idx, int64_t* out_ver, float* out_data) {
  ParamEntry* e = ready_param(key);
  if (!e || e->ptype != 2) return -EINVAL;
  const int64_t w = e->width;
  float* d = pdata(e);
  int64_t* ver = pver(e);
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t r = rows[i];
    if (r < 0 || r >= e->rows) continue;
    auto& l = stripe(key, r);
    spin_lock(l);
    int64_t sv = ver[r];
    if (vers[i] == -1 || sv - vers[i] > bound) {
      out_idx[cnt] = i;
      out_ver[cnt] = sv;
      memcpy(out_data + cnt * w, d + r * w, w * sizeof(float));
      ++cnt;
    }
    spin_unlock(l);
  }
  rec(SYNC_EMB, n * 16 + cnt * (16 + w * 4));
  return cnt;
}

#define ASYNC(key, body) (POOL ? POOL->submit(key, [=]() -> int { return body; }) : (int64_t)(body))

int64_t hps_async_dense_pull(int key, float* out, int64_t len) { return ASYNC(key, hps_dense_pull(key, out, len)); }
int64_t hps_async_dense_push(int key, const float* in, int64_t len) { return ASYNC(key, hps_dense_push(key, in, len)); }
int64_t hps_async_dd_pushpull(int key, const float* in, float* out, int64_t len) { return ASYNC(key, hps_dd_pushpull(key, in, out, len)); }
int64_t hps_async_sparse_pull(int key, const int64_t* ids, int64_t n, float* out) { return ASYNC(key, hps_sparse_pull(key, ids, n, out)); }
int64_t hps_async_sparse_push(int key, const int64_t* ids, int64_t n, const float* vals) { return ASYNC(key, hps_sparse_push(key, ids, n, vals)); }
int64_t hps_async_sd_pushpull(int key, const int64_t* ids, int64_t n, const float* vals, float* dense_out, int64_t len) { return ASYNC(key, hps_sd_pushpull(key, ids, n, vals, dense_out, len)); }
int64_t hps_async_ss_pushpull(int key, const int64_t* in_ids, int64_t nin, const float* vals, const int64_t* out_ids, int64_t nout, float* out) { return ASYNC(key, hps_ss_pushpull(key, in_ids, nin, vals, out_ids, nout, out)); }

int hps_wait(int64_t ticket) { return POOL ? POOL->wait(ticket) : 0; }
int hps_wait_key(int key) { return POOL ? POOL->wait_key(key) : 0; }

int hps_barrier_worker() {
  if (!H) return -1;
  int gen = H->bar_gen.load(std::memory_order_acquire);
  int arrived = H->bar_count.fetch_add(1) + 1;
  if (arrived == H->nworkers) {
    H->bar_count.store(0);
    H->bar_gen.fetch_add(1, std::memory_order_release);
  } else {
    while (H->bar_gen.load(std::memory_order_acquire) == gen) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  rec(BARRIER, 0);
  return 0;
}

static SspState* ssp_find(int key, bool create, int group = 0, int64_t tol = 0) {
  for (int i = 0; i < kMaxSsp; ++i) {
    SspState& s = H->ssp[i];
    if (s.used.load() && s.key == key) return &s;
  }
  if (!create) return nullptr;
  spin_lock(H->dir_lock);
  for (int i = 0; i < kMaxSsp; ++i) {
    SspState& s = H->ssp[i];
    if (s.used.load() && s.key == key) { spin_unlock(H->dir_lock); return &s; }
    if (!s.used.load()) {
      s.key = key;
      s.group_size = group;
      s.tolerance = tol;
      for (int j = 0; j < kMaxNodes; ++j) s.clocks[j].store(0);
      s.used.store(1);
      spin_unlock(H->dir_lock);
      return &s;
    }
  }
  spin_unlock(H->dir_lock);
  return nullptr;
}

int hps_ssp_init(int key, int group_size, int64_t tolerance) {
  return ssp_find(key, true, group_size, tolerance) ? 0 : -ENOMEM;
}

// advance my clock to `version`; block while the slowest member lags by more than tolerance
int hps_ssp_sync(int key, int64_t version) {
  SspState* s = ssp_find(key, false);
  if (!s) return -ENOENT;
  s->clocks[RANK].store(version);
  for (;;) {
    int64_t mn = INT64_MAX;
    for (int i = 0; i < s->group_size; ++i) mn = std::min(mn, s->clocks[i].load());
    if (version - mn <= s->tolerance) break;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  rec(SSP_SYNC, 0);
  return 0;
}

// PReduce: group the workers that arrive within wait_ms (at most `required`); the
// result array lists the partner ranks (terminated by -1).  reference preduce_handler.cc:6-56
int hps_preduce_get_partner(int key, int rank, int required, float wait_ms, int* result) {
  PReduceState* st = nullptr;
  for (int i = 0; i < kMaxPreduce && !st; ++i)
    if (H->pre[i].used.load() && H->pre[i].key == key) st = &H->pre[i];
  if (!st) {
    spin_lock(H->dir_lock);
    for (int i = 0; i < kMaxPreduce && !st; ++i) {
      if (H->pre[i].used.load() && H->pre[i].key == key) st = &H->pre[i];
      else if (!H->pre[i].used.load()) {
        st = &H->pre[i];
        st->key = key;
        st->lock.store(0);
        st->gen = 0;
        st->nmembers = 0;
        st->closed_n = 0;
        st->used.store(1);
      }
    }
    spin_unlock(H->dir_lock);
  }
  if (!st) return -ENOMEM;
  spin_lock(st->lock);
  int64_t my_gen = st->gen;
  if (st->nmembers == 0) {
    st->open_since_ns = now_ns();
    st->required = required;
    st->wait_ms = wait_ms;
  }
  st->members[st->nmembers++] = rank;
  auto close_group = [&] {
    st->closed_n = st->nmembers;
    memcpy(st->closed_members, st->members, sizeof(int32_t) * st->nmembers);
    st->nmembers = 0;
    st->gen++;
  };
  if (st->nmembers >= st->required) close_group();
  spin_unlock(st->lock);
  for (;;) {
    spin_lock(st->lock);
    if (st->gen != my_gen) {
      int n = st->closed_n;
      for (int i = 0; i < n; ++i) result[i] = st->closed_members[i];
      result[n] = -1;
      spin_unlock(st->lock);
      break;
    }
    if (now_ns() - st->open_since_ns > (int64_t)(st->wait_ms * 1e6)) close_group();
    spin_unlock(st->lock);
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  rec(PREDUCE, 0);
  return 0;
}

// [dropped requests, dropped acks, resends, duplicates suppressed, workers recovered]
int hps_fault_stats(int64_t* out) {
  for (int i = 0; i < 4; ++i) out[i] = g_fault[i].load();
  out[4] = H ? H->recovered.load() : 0;
  return 0;
}

int hps_heartbeat() {
  if (!H || RANK < 0) return -1;
  H->heartbeat[RANK].store(now_ns());
  return 0;
}

int hps_dead_nodes(double timeout_s, int* out, int max_out) {
  if (!H) return 0;
  int64_t t = now_ns();
  int n = 0;
  int nw = std::min(H->next_worker.load(), H->nworkers);
  for (int i = 0; i < nw && n < max_out; ++i) {
    int64_t hb = H->heartbeat[i].load();
    if (t - hb > (int64_t)(timeout_s * 1e9)) out[n++] = i;
  }
  return n;
}

// <dir>/<key>_<part>.dat : raw float32 rows of server partition `part`
int hps_save_param(int key, const char* dir) {
  ParamEntry* e = ready_param(key);
  if (!e) return -ENOENT;
  int ns = std::max(1, H->nservers);
  const int64_t total = e->rows * e->width;
  for (int p = 0; p < ns; ++p) {
    int64_t lo, hi;
    if (e->ptype == 0) { lo = total * p / ns; hi = total * (p + 1) / ns; }
    else { lo = (e->rows * p / ns) * e->width; hi = (e->rows * (p + 1) / ns) * e->width; }
    char path[4096];
    snprintf(path, sizeof(path), "%s/%d_%d.dat", dir, key, p);
    FILE* f = fopen(path, "wb");
    if (!f) return -errno;
    fwrite(pdata(e) + lo, sizeof(float), hi - lo, f);
    fclose(f);
  }
  rec(SAVE, total * 4);
  return 0;
}

int hps_load_param(int key, const char* dir) {
  ParamEntry* e = ready_param(key);
  if (!e) return -ENOENT;
  int ns = std::max(1, H->nservers);
  const int64_t total = e->rows * e->width;
  for (int p = 0; p < ns; ++p) {
    int64_t lo, hi;
    if (e->ptype == 0) { lo = total * p / ns; hi = total * (p + 1) / ns; }
    else { lo = (e->rows * p / ns) * e->width; hi = (e->rows * (p + 1) / ns) * e->width; }
    char path[4096];
    snprintf(path, sizeof(path), "%s/%d_%d.dat", dir, key, p);
    FILE* f = fopen(path, "rb");
    if (!f) return -errno;
    size_t got = fread(pdata(e) + lo, sizeof(float), hi - lo, f);
    fclose(f);
    if ((int64_t)got != hi - lo) return -EIO;
  }
  if (e->ptype == 2) memset(pver(e), 0, e->rows * sizeof(int64_t));
  rec(LOAD, total * 4);
  return 0;
}

int hps_start_record(const char* dir) {
  (void)dir;
  for (int i = 0; i < kPsfKinds; ++i) { g_cnt[i] = 0; g_bytes[i] = 0; }
  g_record = true;
  return 0;
}

int hps_get_loads(int64_t* counts, int64_t* bytes, int max_psf) {
  int n = std::min(max_psf, kPsfKinds);
  for (int i = 0; i < n; ++i) { counts[i] = g_cnt[i].load(); bytes[i] = g_bytes[i].load(); }
  return n;
}

}  // extern "C"
