// Runtime helpers of the C ABI (include/rspl.h): device memory, streams,
// HIP-event timers -- all on the system ROCm runtime librspl links against.
#include <vector>

#include "common.hpp"

using namespace rspl;

struct rspl_timer {
  hipEvent_t ev[2] = {nullptr, nullptr};
};

namespace rspl {
// CU mask over the device's CUs: every (ncu / reserve)-th CU is "reserved"; the mask enables
// either everything but the reserved CUs, or only them
int cu_mask(int reserve_cus, bool reserved_only, std::vector<uint32_t>& mask) {
  int dev = 0, ncu = 0;
  RSPL_HIP(hipGetDevice(&dev));
  RSPL_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  RSPL_CHECK_ARG(reserve_cus > 0 && reserve_cus < ncu, "cannot reserve %d of %d CUs", reserve_cus, ncu);
  mask.assign((ncu + 31) / 32, 0u);
  const int step = ncu / reserve_cus;
  int left = reserve_cus;
  for (int c = 0; c < ncu; c++) {
    const bool reserved = left > 0 && c % step == step - 1;
    if (reserved) left--;
    if (reserved == reserved_only) mask[c / 32] |= 1u << (c % 32);
  }
  return RSPL_OK;
}
}  // namespace rspl

extern "C" {

int rspl_device_count(int* count) {
  RSPL_CHECK_ARG(count, "NULL count");
  RSPL_HIP(hipGetDeviceCount(count));
  return RSPL_OK;
}
int rspl_set_device(int device) {
  RSPL_HIP(hipSetDevice(device));
  return RSPL_OK;
}
int rspl_malloc(void** ptr, size_t bytes) {
  RSPL_CHECK_ARG(ptr, "NULL ptr");
  RSPL_HIP(hipMalloc(ptr, bytes ? bytes : 1));
  return RSPL_OK;
}
int rspl_free(void* ptr) {
  RSPL_HIP(hipFree(ptr));
  return RSPL_OK;
}
int rspl_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return RSPL_OK;
  RSPL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  RSPL_HIP(hipStreamSynchronize((hipStream_t)stream));
  return RSPL_OK;
}
int rspl_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return RSPL_OK;
  RSPL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  RSPL_HIP(hipStreamSynchronize((hipStream_t)stream));
  return RSPL_OK;
}
int rspl_memset(void* dst, int value, size_t bytes, void* stream) {
  RSPL_HIP(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream));
  return RSPL_OK;
}
int rspl_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return RSPL_OK;
  RSPL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return RSPL_OK;
}
int rspl_stream_create(void** stream) {
  RSPL_CHECK_ARG(stream, "NULL stream");
  RSPL_HIP(hipStreamCreateWithFlags((hipStream_t*)stream, hipStreamNonBlocking));
  return RSPL_OK;
}
int rspl_stream_create_priority(void** stream, int high) {
  RSPL_CHECK_ARG(stream, "NULL stream");
  int lo = 0, hi = 0;
  RSPL_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  RSPL_HIP(hipStreamCreateWithPriority((hipStream_t*)stream, hipStreamNonBlocking, high ? hi : lo));
  return RSPL_OK;
}

int rspl_stream_create_reserving(void** stream, int reserve_cus) {
  RSPL_CHECK_ARG(stream && reserve_cus >= 0, "rspl_stream_create_reserving: bad arguments");
  if (reserve_cus == 0) {
    RSPL_HIP(hipStreamCreateWithFlags((hipStream_t*)stream, hipStreamNonBlocking));
    return RSPL_OK;
  }
  std::vector<uint32_t> mask;
  int rc = rspl::cu_mask(reserve_cus, false, mask);
  if (rc) return rc;
  RSPL_HIP(hipExtStreamCreateWithCUMask((hipStream_t*)stream, (uint32_t)mask.size(), mask.data()));
  return RSPL_OK;
}
int rspl_stream_destroy(void* stream) {
  RSPL_HIP(hipStreamDestroy((hipStream_t)stream));
  return RSPL_OK;
}
int rspl_stream_synchronize(void* stream) {
  RSPL_HIP(hipStreamSynchronize((hipStream_t)stream));
  return RSPL_OK;
}
int rspl_event_create(void** event) {
  RSPL_CHECK_ARG(event, "NULL event");
  RSPL_HIP(hipEventCreateWithFlags((hipEvent_t*)event, hipEventDisableTiming));
  return RSPL_OK;
}
int rspl_event_record(void* event, void* stream) {
  RSPL_HIP(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
  return RSPL_OK;
}
int rspl_stream_wait_event(void* stream, void* event) {
  RSPL_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return RSPL_OK;
}
int rspl_event_destroy(void* event) {
  RSPL_HIP(hipEventDestroy((hipEvent_t)event));
  return RSPL_OK;
}
int rspl_device_synchronize(void) {
  RSPL_HIP(hipDeviceSynchronize());
  return RSPL_OK;
}
int rspl_timer_create(rspl_timer** t) {
  RSPL_CHECK_ARG(t, "NULL timer");
  auto* x = new rspl_timer();
  if (hipEventCreate(&x->ev[0]) != hipSuccess || hipEventCreate(&x->ev[1]) != hipSuccess) {
    set_error("hipEventCreate failed");
    delete x;
    return RSPL_E_DEVICE;
  }
  *t = x;
  return RSPL_OK;
}
int rspl_timer_record(rspl_timer* t, int which, void* stream) {
  RSPL_CHECK_ARG(t && (which == 0 || which == 1), "bad timer / which");
  RSPL_HIP(hipEventRecord(t->ev[which], (hipStream_t)stream));
  return RSPL_OK;
}
int rspl_timer_elapsed_ms(rspl_timer* t, float* ms) {
  RSPL_CHECK_ARG(t && ms, "bad timer");
  RSPL_HIP(hipEventSynchronize(t->ev[1]));
  RSPL_HIP(hipEventElapsedTime(ms, t->ev[0], t->ev[1]));
  return RSPL_OK;
}
void rspl_timer_destroy(rspl_timer* t) {
  if (!t) return;
  for (auto& e : t->ev)
    if (e) (void)hipEventDestroy(e);
  delete t;
}

}  // extern "C"
