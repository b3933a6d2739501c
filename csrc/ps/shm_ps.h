// Single-node parameter server over POSIX shared memory ("shm van").
//
// MI355X node design: one server process owns a
// shared-memory segment in host DRAM that holds every PS table; the 8 worker
// processes (one per GPU) map the same segment.  A PSF request (DensePull,
// SparsePush, SDPushPull, PushEmbedding, SyncEmbedding, ...) is executed by a
// worker-side thread pool directly against the shared tables under striped
// row locks -- no serialisation and no server hop, while keeping ps-lite's
// roles (scheduler/server/worker), worker barriers, heartbeats / dead-node
// detection, SSP clocks, PReduce partner matching, save/load in the
// ``<key>_<partition>.dat`` raw-float32 format and the PS_* fault knobs
// (PS_DROP_MSG drops a request which is then re-sent after PS_RESEND_TIMEOUT).
#pragma once
#include <stdint.h>
#include <stddef.h>

extern "C" {

// ---- lifecycle ------------------------------------------------------------------
// role: 0 scheduler, 1 server, 2 worker.  name: shm object name ("/hetu_ps_<port>").
int hps_init(int role, const char* name, int num_workers, int num_servers, uint64_t heap_bytes);
int hps_finalize();
int hps_rank();     // worker rank (0..nworkers-1), -1 for servers
int hps_nrank();    // number of workers
int hps_server_wait_shutdown(double timeout_s);  // server: block until all workers finalized

// ---- parameters -------------------------------------------------------------------
// ptype: 0 dense, 1 sparse, 2 cache table.  init_type: 0 constant, 1 uniform, 2 normal,
// 3 truncated normal (a, b as in the reference InitTensor).
int hps_param_init(int key, int ptype, int64_t rows, int64_t width, int init_type, double a,
                   double b, uint64_t seed);
int hps_param_clear(int key);
int64_t hps_param_rows(int key);
int64_t hps_param_width(int key);

// ---- synchronous PSF bodies (also used by the async queue) --------------------------
int hps_dense_pull(int key, float* out, int64_t len);
int hps_dense_push(int key, const float* in, int64_t len);
int hps_dd_pushpull(int key, const float* in, float* out, int64_t len);
int hps_sparse_pull(int key, const int64_t* ids, int64_t n, float* out);
int hps_sparse_push(int key, const int64_t* ids, int64_t n, const float* vals);
int hps_sd_pushpull(int key, const int64_t* ids, int64_t n, const float* vals, float* dense_out, int64_t len);
int hps_ss_pushpull(int key, const int64_t* in_ids, int64_t nin, const float* vals,
                    const int64_t* out_ids, int64_t nout, float* out);
// cache table (HET): versions are int64 per row
int hps_push_embedding(int key, const int64_t* rows, int64_t n, const float* data, const int64_t* updates);
// returns number of refreshed rows; idx/ver/data sized n (worst case)
int64_t hps_sync_embedding(int key, const int64_t* rows, int64_t n, const int64_t* vers,
                           int64_t bound, int64_t* out_idx, int64_t* out_ver, float* out_data);

// ---- async queue (worker thread pool) ---------------------------------------------------
// returns a ticket; hps_wait(ticket) blocks; hps_wait_key(key) waits all tickets of key.
int64_t hps_async_dense_pull(int key, float* out, int64_t len);
int64_t hps_async_dense_push(int key, const float* in, int64_t len);
int64_t hps_async_dd_pushpull(int key, const float* in, float* out, int64_t len);
int64_t hps_async_sparse_pull(int key, const int64_t* ids, int64_t n, float* out);
int64_t hps_async_sparse_push(int key, const int64_t* ids, int64_t n, const float* vals);
int64_t hps_async_sd_pushpull(int key, const int64_t* ids, int64_t n, const float* vals, float* dense_out, int64_t len);
int64_t hps_async_ss_pushpull(int key, const int64_t* in_ids, int64_t nin, const float* vals,
                              const int64_t* out_ids, int64_t nout, float* out);
int hps_wait(int64_t ticket);
int hps_wait_key(int key);

// ---- coordination --------------------------------------------------------------------
int hps_barrier_worker();
int hps_ssp_init(int key, int group_size, int64_t tolerance);
int hps_ssp_sync(int key, int64_t version);
int hps_preduce_get_partner(int key, int rank, int required, float wait_ms, int* result);
int hps_heartbeat();
// [dropped requests, dropped acks, resends, duplicates suppressed, workers recovered]
int hps_fault_stats(int64_t* out);
int hps_dead_nodes(double timeout_s, int* out, int max_out);

// ---- persistence (reference PSFHandle.h:389-427 format) ----------------------------------
int hps_save_param(int key, const char* dir);
int hps_load_param(int key, const char* dir);

// ---- load recording (reference kvworker.h:39-51) --------------------------------------------
int hps_start_record(const char* dir);
int hps_get_loads(int64_t* counts, int64_t* bytes, int max_psf);

// ---- pinned-host BFC allocator stats passthrough (runtime/bfc_allocator) ----------------------
}
