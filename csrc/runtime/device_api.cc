// Device runtime C API: HIP streams, events and copies owned by the framework
// (reference src/cuda_common/gpu_runtime.cc:61-118 DLStreamCreate/Destroy/Sync,
// DLEventCreate/Record/Sync/ElapsedTime; cuda_device_api.cc:24-74 the copy paths;
// SURVEY §2.2 N1/N2).  The executor, the RCCL comm stream, the PS staging streams and
// the dataloader prefetch stream are created here; torch sees them only as external
// streams (torch.cuda.ExternalStream over the handle) when a library op must be ordered
// on them.  Every call returns a hipError_t (0 = success).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HETU_RT_API extern "C" __attribute__((visibility("default")))

// priority: 0 normal, < 0 higher (hipDeviceGetStreamPriorityRange clamps); non-blocking
// w.r.t. the legacy null stream, like torch's pool streams
HETU_RT_API int hetu_stream_create(int device, int priority, void** out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (priority < hi) priority = hi;
  if (priority > lo) priority = lo;
  hipStream_t s = nullptr;
  e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
  *out = (void*)s;
  return (int)e;
}

HETU_RT_API int hetu_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }
HETU_RT_API int hetu_stream_sync(void* s) { return (int)hipStreamSynchronize((hipStream_t)s); }
HETU_RT_API int hetu_stream_query(void* s) { return (int)hipStreamQuery((hipStream_t)s); }   // 0 idle, 600 busy

// timing: 1 -> elapsed-time capable; else hipEventDisableTiming (cheaper record / wait)
HETU_RT_API int hetu_event_create(int device, int timing, void** out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  hipEvent_t ev = nullptr;
  e = hipEventCreateWithFlags(&ev, timing ? hipEventDefault : hipEventDisableTiming);
  *out = (void*)ev;
  return (int)e;
}

HETU_RT_API int hetu_event_destroy(void* ev) { return (int)hipEventDestroy((hipEvent_t)ev); }
HETU_RT_API int hetu_event_record(void* ev, void* stream) { return (int)hipEventRecord((hipEvent_t)ev, (hipStream_t)stream); }
HETU_RT_API int hetu_event_sync(void* ev) { return (int)hipEventSynchronize((hipEvent_t)ev); }
HETU_RT_API int hetu_event_query(void* ev) { return (int)hipEventQuery((hipEvent_t)ev); }     // 0 done, 600 pending

HETU_RT_API int hetu_event_elapsed(void* start, void* end, float* ms) {
  return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
}

// stream waits (on the device) for everything recorded before `ev`
HETU_RT_API int hetu_stream_wait_event(void* stream, void* ev) {
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0);
}

// kind: 0 host->host, 1 host->device, 2 device->host, 3 device->device (same or peer)
HETU_RT_API int hetu_memcpy_async(void* dst, const void* src, int64_t bytes, int kind, void* stream) {
  static const hipMemcpyKind k[4] = {hipMemcpyHostToHost, hipMemcpyHostToDevice, hipMemcpyDeviceToHost,
                                     hipMemcpyDeviceToDevice};
  if (kind < 0 || kind > 3) return (int)hipErrorInvalidValue;
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, k[kind], (hipStream_t)stream);
}

// peer copy over xGMI (reference cuda_device_api.cc cudaMemcpyPeerAsync)
HETU_RT_API int hetu_memcpy_peer_async(void* dst, int dst_dev, const void* src, int src_dev, int64_t bytes,
                                       void* stream) {
  return (int)hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, (size_t)bytes, (hipStream_t)stream);
}

HETU_RT_API int hetu_memset_async(void* dst, int value, int64_t bytes, void* stream) {
  return (int)hipMemsetAsync(dst, value, (size_t)bytes, (hipStream_t)stream);
}

HETU_RT_API int hetu_device_count(int* n) { return (int)hipGetDeviceCount(n); }
HETU_RT_API int hetu_device_sync(int device) {
  hipError_t e = hipSetDevice(device);
  return e != hipSuccess ? (int)e : (int)hipDeviceSynchronize();
}
HETU_RT_API const char* hetu_error_string(int e) { return hipGetErrorString((hipError_t)e); }

// ---- stream capture into a HIP graph (the executor's replayed steady-state step) -------
// mode: 0 global, 1 thread-local, 2 relaxed (the BFC pool may grow a region mid-capture)
HETU_RT_API int hetu_stream_begin_capture(void* s, int mode) {
  static const hipStreamCaptureMode m[3] = {hipStreamCaptureModeGlobal, hipStreamCaptureModeThreadLocal,
                                            hipStreamCaptureModeRelaxed};
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  return (int)hipStreamBeginCapture((hipStream_t)s, m[mode]);
}
HETU_RT_API int hetu_stream_end_capture(void* s, void** graph) {
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture((hipStream_t)s, &g);
  *graph = (void*)g;
  return (int)e;
}
HETU_RT_API int hetu_stream_is_capturing(void* s, int* status) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing((hipStream_t)s, &st);
  *status = (int)st;
  return (int)e;
}
HETU_RT_API int hetu_graph_instantiate(void* graph, void** exec) {
  hipGraphExec_t x = nullptr;
  hipError_t e = hipGraphInstantiate(&x, (hipGraph_t)graph, nullptr, nullptr, 0);
  *exec = (void*)x;
  return (int)e;
}
HETU_RT_API int hetu_graph_nodes(void* graph, int64_t* n) {
  size_t c = 0;
  hipError_t e = hipGraphGetNodes((hipGraph_t)graph, nullptr, &c);
  *n = (int64_t)c;
  return (int)e;
}
HETU_RT_API int hetu_graph_launch(void* exec, void* stream) {
  return (int)hipGraphLaunch((hipGraphExec_t)exec, (hipStream_t)stream);
}
HETU_RT_API int hetu_graph_destroy(void* graph) { return (int)hipGraphDestroy((hipGraph_t)graph); }
HETU_RT_API int hetu_graph_exec_destroy(void* exec) { return (int)hipGraphExecDestroy((hipGraphExec_t)exec); }
