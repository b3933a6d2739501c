// In-house RCCL communicator over xGMI (reference src/communication/
// mpi_nccl_communication.cu:31-458, header src/header/mpi_nccl_communication.h:10-84;
// SURVEY.md §2.2 N6, §2.6, §5.8).
//
// MI355X design, not a translation of the reference's MPI+NCCL library:
//  * no MPI: the 128-byte ncclUniqueId is exchanged through the job's TCP store by the
//    Python side (parallel/rccl.py), and mpirun / torchrun environments both work;
//  * RCCL is dlopen'ed from the path the caller names -- the same librccl.so.1 the
//    process already has mapped (torch's), so one RCCL instance serves every
//    communicator of the process;
//  * every collective takes the HIP stream to run on: the caller orders it after the
//    producing kernels with stream/event edges (hipStreamWaitEvent), never a host sync;
//  * sub-groups come from ncclCommSplit (static groups) or a fresh unique id (groups
//    formed at run time among their members only, e.g. partial-reduce partners);
//  * all-to-all (MoE dispatch, Ulysses, the mixed-precision reduce-scatter) is one
//    grouped send/recv per peer: on the 8-GPU xGMI full mesh every peer pair has its
//    own link, so the exchange uses all 7 links at once;
//  * channel counts for the 7-link mesh are set through NCCL_MIN_NCHANNELS /
//    NCCL_MAX_NCHANNELS before the first init (hcomm_set_channels).
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>

#include <rccl/rccl.h>

#define HCOMM_API extern "C" __attribute__((visibility("default")))

namespace {

struct Api {
  void* lib = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
};

Api g;
std::mutex g_mu;

template <class F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.lib, name));
  return f != nullptr;
}

size_t dtype_size(int dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

inline int rc(ncclResult_t r) { return (int)r; }

}  // namespace

// Load RCCL from `path` (the library the process already uses); idempotent.
// Returns 0 on success, -1 when the library or a symbol is missing.
HCOMM_API int hcomm_load(const char* path) {
  std::lock_guard<std::mutex> l(g_mu);
  if (g.lib) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
  if (!h) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) return -1;
  g.lib = h;
  bool ok = sym(g.GetUniqueId, "ncclGetUniqueId") && sym(g.CommInitRank, "ncclCommInitRank") &&
            sym(g.CommDestroy, "ncclCommDestroy") && sym(g.CommAbort, "ncclCommAbort") &&
            sym(g.CommGetAsyncError, "ncclCommGetAsyncError") && sym(g.CommCount, "ncclCommCount") &&
            sym(g.CommUserRank, "ncclCommUserRank") && sym(g.AllReduce, "ncclAllReduce") &&
            sym(g.ReduceScatter, "ncclReduceScatter") && sym(g.AllGather, "ncclAllGather") &&
            sym(g.Broadcast, "ncclBroadcast") && sym(g.Reduce, "ncclReduce") && sym(g.Send, "ncclSend") &&
            sym(g.Recv, "ncclRecv") && sym(g.GroupStart, "ncclGroupStart") && sym(g.GroupEnd, "ncclGroupEnd") &&
            sym(g.GetErrorString, "ncclGetErrorString") && sym(g.GetVersion, "ncclGetVersion");
  sym(g.CommSplit, "ncclCommSplit");   // optional (RCCL >= 2.18)
  sym(g.CommInitAll, "ncclCommInitAll");
  if (!ok) {
    g.lib = nullptr;
    return -1;
  }
  return 0;
}

HCOMM_API int hcomm_loaded() { return g.lib != nullptr; }

HCOMM_API int hcomm_version() {
  int v = 0;
  if (!g.lib || g.GetVersion(&v) != ncclSuccess) return -1;
  return v;
}

HCOMM_API const char* hcomm_error_string(int r) {
  return g.lib ? g.GetErrorString((ncclResult_t)r) : "RCCL not loaded";
}

// Channel counts for the next communicator init (RCCL reads the environment at init):
// on the 8-GPU xGMI mesh a ring per link wants >= 7 channels, more for overlap.
HCOMM_API void hcomm_set_channels(int min_ch, int max_ch) {
  char b[32];
  if (min_ch > 0) {
    snprintf(b, sizeof(b), "%d", min_ch);
    setenv("NCCL_MIN_NCHANNELS", b, 1);
  }
  if (max_ch > 0) {
    snprintf(b, sizeof(b), "%d", max_ch);
    setenv("NCCL_MAX_NCHANNELS", b, 1);
  }
}

HCOMM_API int hcomm_unique_id(char* out) {
  if (!g.lib) return -1;
  ncclUniqueId id;
  ncclResult_t r = g.GetUniqueId(&id);
  if (r == ncclSuccess) memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return rc(r);
}

HCOMM_API int hcomm_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

// The calling thread's current HIP device is the communicator's device.
HCOMM_API int hcomm_init(const char* id_bytes, int nranks, int rank, void** out) {
  if (!g.lib) return -1;
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ncclResult_t r = g.CommInitRank(&c, nranks, id, rank);
  *out = c;
  return rc(r);
}

// Every rank of `comm` calls; color < 0 = not a member (*out = null).
HCOMM_API int hcomm_split(void* comm, int color, int key, void** out) {
  if (!g.lib || !g.CommSplit) return -1;
  ncclComm_t c = nullptr;
  ncclResult_t r = g.CommSplit((ncclComm_t)comm, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &c, nullptr);
  *out = c;
  return rc(r);
}

HCOMM_API int hcomm_destroy(void* comm) { return comm && g.lib ? rc(g.CommDestroy((ncclComm_t)comm)) : 0; }
HCOMM_API int hcomm_abort(void* comm) { return comm && g.lib ? rc(g.CommAbort((ncclComm_t)comm)) : 0; }

// Watchdog probe: the communicator's asynchronous error state.
HCOMM_API int hcomm_async_error(void* comm) {
  ncclResult_t e = ncclSuccess;
  if (!comm || !g.lib) return -1;
  ncclResult_t r = g.CommGetAsyncError((ncclComm_t)comm, &e);
  return r != ncclSuccess ? rc(r) : rc(e);
}

HCOMM_API int hcomm_count(void* comm) {
  int n = -1;
  if (comm && g.lib) g.CommCount((ncclComm_t)comm, &n);
  return n;
}

HCOMM_API int hcomm_user_rank(void* comm) {
  int n = -1;
  if (comm && g.lib) g.CommUserRank((ncclComm_t)comm, &n);
  return n;
}

HCOMM_API int hcomm_all_reduce(void* comm, const void* s, void* r, size_t count, int dt, int op, void* st) {
  return rc(g.AllReduce(s, r, count, (ncclDataType_t)dt, (ncclRedOp_t)op, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_reduce_scatter(void* comm, const void* s, void* r, size_t recvcount, int dt, int op, void* st) {
  return rc(g.ReduceScatter(s, r, recvcount, (ncclDataType_t)dt, (ncclRedOp_t)op, (ncclComm_t)comm,
                            (hipStream_t)st));
}

HCOMM_API int hcomm_all_gather(void* comm, const void* s, void* r, size_t sendcount, int dt, void* st) {
  return rc(g.AllGather(s, r, sendcount, (ncclDataType_t)dt, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_broadcast(void* comm, const void* s, void* r, size_t count, int dt, int root, void* st) {
  return rc(g.Broadcast(s, r, count, (ncclDataType_t)dt, root, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_reduce(void* comm, const void* s, void* r, size_t count, int dt, int op, int root, void* st) {
  return rc(g.Reduce(s, r, count, (ncclDataType_t)dt, (ncclRedOp_t)op, root, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_send(void* comm, const void* s, size_t count, int dt, int peer, void* st) {
  return rc(g.Send(s, count, (ncclDataType_t)dt, peer, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_recv(void* comm, void* r, size_t count, int dt, int peer, void* st) {
  return rc(g.Recv(r, count, (ncclDataType_t)dt, peer, (ncclComm_t)comm, (hipStream_t)st));
}

HCOMM_API int hcomm_group_start() { return rc(g.GroupStart()); }
HCOMM_API int hcomm_group_end() { return rc(g.GroupEnd()); }

// Equal-chunk all-to-all (reference AllToAll semantics, mpi_nccl_communication.cu:245-277):
// chunk p of `s` goes to peer p, chunk q of `r` comes from peer q; one RCCL group.
HCOMM_API int hcomm_all_to_all(void* comm, const void* s, void* r, size_t chunk, int dt, void* st) {
  const int n = hcomm_count(comm);
  if (n <= 0) return -1;
  const size_t bytes = chunk * dtype_size(dt);
  ncclResult_t e = g.GroupStart();
  if (e != ncclSuccess) return rc(e);
  for (int p = 0; p < n && e == ncclSuccess; ++p) {
    e = g.Send((const char*)s + p * bytes, chunk, (ncclDataType_t)dt, p, (ncclComm_t)comm, (hipStream_t)st);
    if (e == ncclSuccess)
      e = g.Recv((char*)r + p * bytes, chunk, (ncclDataType_t)dt, p, (ncclComm_t)comm, (hipStream_t)st);
  }
  ncclResult_t e2 = g.GroupEnd();
  return rc(e != ncclSuccess ? e : e2);
}

// Variable-size all-to-all (element counts / offsets per peer; MoE with uneven routing).
HCOMM_API int hcomm_all_to_all_v(void* comm, const void* s, const int64_t* scounts, const int64_t* soffs, void* r,
                                 const int64_t* rcounts, const int64_t* roffs, int dt, void* st) {
  const int n = hcomm_count(comm);
  if (n <= 0) return -1;
  const size_t es = dtype_size(dt);
  ncclResult_t e = g.GroupStart();
  if (e != ncclSuccess) return rc(e);
  for (int p = 0; p < n && e == ncclSuccess; ++p) {
    if (scounts[p] > 0)
      e = g.Send((const char*)s + soffs[p] * es, (size_t)scounts[p], (ncclDataType_t)dt, p, (ncclComm_t)comm,
                 (hipStream_t)st);
    if (e == ncclSuccess && rcounts[p] > 0)
      e = g.Recv((char*)r + roffs[p] * es, (size_t)rcounts[p], (ncclDataType_t)dt, p, (ncclComm_t)comm,
                 (hipStream_t)st);
  }
  ncclResult_t e2 = g.GroupEnd();
  return rc(e != ncclSuccess ? e : e2);
}

// ---- single-process multi-GPU communicator (reference src/communication/
// nccl_communication.cu:29-69): one process drives `ndev` GPUs through
// ncclCommInitAll; every collective is one RCCL group over the per-device communicators,
// each on its device's stream.
HCOMM_API int hcomm_init_all(int ndev, const int* devs, void** out) {
  if (!g.lib || !g.CommInitAll || ndev <= 0) return -1;
  return rc(g.CommInitAll((ncclComm_t*)out, ndev, devs));
}

HCOMM_API int hcomm_multi_all_reduce(void* const* comms, void* const* send, void* const* recv, size_t count, int dt,
                                     int op, void* const* streams, int ndev) {
  ncclResult_t e = g.GroupStart();
  for (int i = 0; i < ndev && e == ncclSuccess; ++i)
    e = g.AllReduce(send[i], recv[i], count, (ncclDataType_t)dt, (ncclRedOp_t)op, (ncclComm_t)comms[i],
                    (hipStream_t)streams[i]);
  ncclResult_t e2 = g.GroupEnd();
  return rc(e != ncclSuccess ? e : e2);
}

// equal chunks: chunk j of device i's send buffer goes to device j (reference NCCL_AllToAll)
HCOMM_API int hcomm_multi_all_to_all(void* const* comms, void* const* send, void* const* recv, size_t chunk, int dt,
                                     void* const* streams, int ndev) {
  const size_t bytes = chunk * dtype_size(dt);
  ncclResult_t e = g.GroupStart();
  for (int i = 0; i < ndev && e == ncclSuccess; ++i)
    for (int j = 0; j < ndev && e == ncclSuccess; ++j) {
      e = g.Send((const char*)send[i] + j * bytes, chunk, (ncclDataType_t)dt, j, (ncclComm_t)comms[i],
                 (hipStream_t)streams[i]);
      if (e == ncclSuccess)
        e = g.Recv((char*)recv[i] + j * bytes, chunk, (ncclDataType_t)dt, j, (ncclComm_t)comms[i],
                   (hipStream_t)streams[i]);
    }
  ncclResult_t e2 = g.GroupEnd();
  return rc(e != ncclSuccess ? e : e2);
}
