// Host-runtime stress test built with sanitizers (SURVEY §5.2 plan: ASan/UBSan and
// TSan builds of the host runtime and PS).  `make -C csrc sanitize` builds
//   build/runtime_asan  (-fsanitize=address,undefined)
//   build/runtime_tsan  (-fsanitize=thread)
// from the runtime sources themselves (BFC allocator, shared-memory PS, HET
// cache), and tests/test_sanitizers_cpu.py runs both.  What is exercised:
//   * BFC allocator: 4 threads of random alloc/free with per-thread stream tags
//     on one allocator, invariant check at the end;
//   * PS: a server process and 2 worker processes (fork) doing concurrent dense
//     push/pull, sparse push/pull and barriers through the shm van, each worker
//     with a 4-thread async pool;
//   * HET cache: bounded-staleness lookups/updates from 2 threads per worker.
// Exit status 0 = clean; a sanitizer report makes the process exit non-zero.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <random>
#include <thread>
#include <vector>

#include "../runtime/bfc_allocator.h"

extern "C" {
int hps_init(int role, const char* name, int num_workers, int num_servers, uint64_t heap_bytes);
int hps_finalize();
int hps_rank();
int hps_server_wait_shutdown(double timeout_s);
int hps_param_init(int key, int ptype, int64_t rows, int64_t width, int init_type, double a, double b,
                   uint64_t seed);
int hps_dense_pull(int key, float* out, int64_t len);
int hps_dense_push(int key, const float* in, int64_t len);
int64_t hps_async_dense_push(int key, const float* in, int64_t len);
int hps_sparse_pull(int key, const int64_t* ids, int64_t n, float* out);
int hps_sparse_push(int key, const int64_t* ids, int64_t n, const float* vals);
int hps_wait(int64_t ticket);
int hps_barrier_worker();
int hc_create(int policy, int64_t limit, int64_t rows, int64_t width, int key, int64_t pull_bound,
              int64_t push_bound);
int hc_lookup(int h, const int64_t* keys, int64_t n, float* dest);
int hc_update(int h, const int64_t* keys, int64_t n, const float* grads);
int hc_flush(int h);
int64_t hc_parallel_for_selftest(int iters);
}

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      _exit(3);                                                           \
    }                                                                     \
  } while (0)

static int test_bfc() {
  hetu::BFCAllocator a(hetu::MemKind::kHostTagged, 0, 64 << 20, 1 << 20);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t) {
    th.emplace_back([&a, t] {
      std::mt19937 rng(t);
      hipStream_t tag = (hipStream_t)(uintptr_t)(0x1000 * (t + 1));
      std::vector<std::pair<char*, size_t>> live;
      for (int i = 0; i < 4000; ++i) {
        if (!live.empty() && rng() % 100 < 45) {
          size_t k = rng() % live.size();
          auto p = live[k];
          for (size_t j = 0; j < p.second; j += 97) CHECK(p.first[j] == (char)t);   // nobody scribbled
          a.deallocate(p.first, tag);
          live[k] = live.back();
          live.pop_back();
        } else {
          size_t n = 1 + rng() % 70000;
          char* p = (char*)a.allocate(n, tag);
          CHECK(p != nullptr);
          memset(p, t, n);
          live.push_back({p, n});
        }
      }
      for (auto& p : live) a.deallocate(p.first, tag);
    });
  }
  for (auto& x : th) x.join();
  CHECK(a.check_invariants());
  CHECK(a.stats().bytes_in_use == 0);
  return 0;
}

static void worker_main(const char* name) {
  CHECK(hps_init(2, name, 2, 1, 0) == 0);
  const int r = hps_rank();
  CHECK(hps_param_init(1, 0, 8192, 1, 0, 0.0, 0.0, 0) == 0);
  CHECK(hps_param_init(2, 1, 256, 16, 0, 0.0, 0.0, 0) == 0);
  std::vector<float> ones(8192, 1.f), out(8192);
  std::vector<int64_t> tickets;
  for (int i = 0; i < 8; ++i) tickets.push_back(hps_async_dense_push(1, ones.data(), 8192));
  for (auto tk : tickets) CHECK(hps_wait(tk) == 0);
  hps_barrier_worker();
  CHECK(hps_dense_pull(1, out.data(), 8192) == 0);
  for (int i = 0; i < 8192; ++i) CHECK(out[i] == 16.f);   // 2 workers x 8 pushes
  // sparse rows: each worker pushes 1.0 into rows {r, 100 + r, 100 + r}
  int64_t ids[3] = {r, 100 + r, 100 + r};
  std::vector<float> vals(3 * 16, 1.f), got(3 * 16);
  CHECK(hps_sparse_push(2, ids, 3, vals.data()) == 0);
  hps_barrier_worker();
  int64_t q[3] = {0, 100, 255};
  CHECK(hps_sparse_pull(2, q, 3, got.data()) == 0);
  CHECK(got[0] == 1.f && got[16] == 2.f && got[32] == 0.f);
  // HET cache (LFUOpt, bound 3) over table key 3, two threads hammering it
  CHECK(hps_param_init(3, 2, 1000, 8, 0, 0.0, 0.0, 0) == 0);
  int h = hc_create(2, 100, 1000, 8, 3, 3, 3);
  CHECK(h >= 0);
  std::vector<std::thread> th;
  for (int t = 0; t < 2; ++t) {
    th.emplace_back([h, t, r] {
      std::mt19937 rng(17 * r + t);
      std::vector<int64_t> k(64);
      std::vector<float> d(64 * 8), gr(64 * 8, 0.01f);
      for (int it = 0; it < 200; ++it) {
        for (auto& x : k) x = rng() % 1000;
        CHECK(hc_lookup(h, k.data(), 64, d.data()) == 0);
        CHECK(hc_update(h, k.data(), 64, gr.data()) == 0);
      }
    });
  }
  for (auto& x : th) x.join();
  CHECK(hc_flush(h) == 0);
  // large batches (> the cache's parallel-loop threshold): the row copy and the
  // gradient application run on the cache's worker threads, with evictions
  int h2 = hc_create(1, 300, 1000, 8, 3, 3, 3);
  CHECK(h2 >= 0);
  {
    std::mt19937 rng(91 + r);
    std::vector<int64_t> k(2048);
    std::vector<float> d(2048 * 8), gr(2048 * 8, 0.01f);
    for (int it = 0; it < 20; ++it) {
      for (auto& x : k) x = rng() % 1000;
      CHECK(hc_lookup(h2, k.data(), 2048, d.data()) == 0);
      CHECK(hc_update(h2, k.data(), 2048, gr.data()) == 0);
    }
    CHECK(hc_flush(h2) == 0);
  }
  hps_barrier_worker();
  CHECK(hps_finalize() == 0);
}

static int test_ps() {
  char name[64];
  snprintf(name, sizeof(name), "/hetu_san_%d", (int)getpid());
  pid_t server = fork();
  if (server == 0) {
    CHECK(hps_init(1, name, 2, 1, 64ull << 20) == 0);
    CHECK(hps_server_wait_shutdown(120) == 0);
    hps_finalize();
    _exit(0);
  }
  pid_t w[2];
  for (int i = 0; i < 2; ++i) {
    w[i] = fork();
    if (w[i] == 0) {
      worker_main(name);
      _exit(0);
    }
  }
  int bad = 0;
  for (pid_t p : {w[0], w[1], server}) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
      fprintf(stderr, "child %d failed (status %d)\n", (int)p, st);
      bad = 1;
    }
  }
  return bad;
}

int main() {
  int rc = test_bfc();
  if (rc) return rc;
  rc = test_ps();
  if (rc) return rc;
  // cache fork-join pool (after the forks: it starts threads): regions of
  // alternating sizes, every element exactly once
  CHECK(hc_parallel_for_selftest(400) == 0);
  printf("runtime sanitize test: OK\n");
  return 0;
}
