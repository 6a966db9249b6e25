// Common runtime pieces of librspl: error reporting across the C ABI, HIP
// checks, and a bump arena so every handle allocates its device memory once at
// create time (the reference allocates per infer call: buffers.h:209-233).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/rspl.h"

namespace rspl {

void set_error(const char* fmt, ...);
// CU mask of the reserved CUs (every ncu/reserve_cus-th CU) or of all the others
int cu_mask(int reserve_cus, bool reserved_only, std::vector<uint32_t>& mask);

#define RSPL_HIP(expr)                                                                   \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::rspl::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return RSPL_E_DEVICE;                                                              \
    }                                                                                    \
  } while (0)

#define RSPL_CHECK_ARG(cond, ...)    \
  do {                               \
    if (!(cond)) {                   \
      ::rspl::set_error(__VA_ARGS__); \
      return RSPL_E_ARG;             \
    }                                \
  } while (0)

// One hipMalloc per handle; sub-allocations are 256-byte aligned.
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  int reserve(size_t bytes) {
    size = bytes;
    used = 0;
    if (hipMalloc(&base, bytes) != hipSuccess) {
      set_error("hipMalloc(%zu) failed", bytes);
      base = nullptr;
      return RSPL_E_DEVICE;
    }
    return RSPL_OK;
  }
  template <typename T>
  T* take(size_t count) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + count * sizeof(T);
    if (used > size) return nullptr;
    return reinterpret_cast<T*>(base + off);
  }
  void release() {
    if (base) (void)hipFree(base);
    base = nullptr;
  }
};

// Size-only pass of the same carving, so arenas are allocated exactly once.
struct Sizer {
  size_t used = 0;
  template <typename T>
  void take(size_t count) {
    used = ((used + 255) & ~size_t(255)) + count * sizeof(T);
  }
};

// Per-stage device timing: HIP events recorded on the launch stream at stage
// boundaries of each profiled call, kept in a ring and harvested lazily so the
// profiling never adds a host synchronisation to the pipeline.
struct StageTimer {
  static constexpr int kRing = 64, kMax = 8;
  int n = 0;
  bool enabled = false;
  hipEvent_t ev[kRing][kMax + 1] = {};
  bool pending[kRing] = {};
  int head = 0;
  double acc[kMax] = {};
  long calls = 0;
  int init(int nstages) {
    n = nstages;
    for (int r = 0; r < kRing; r++)
      for (int i = 0; i <= n; i++)
        if (hipEventCreate(&ev[r][i]) != hipSuccess) return RSPL_E_DEVICE;
    return RSPL_OK;
  }
  void destroy() {
    for (int r = 0; r < kRing; r++)
      for (int i = 0; i <= n; i++)
        if (ev[r][i]) (void)hipEventDestroy(ev[r][i]);
  }
  void mark(int i, hipStream_t s) {
    if (enabled) (void)hipEventRecord(ev[head][i], s);
  }
  // event i of the current call, to be stamped by a kernel launch itself (hipExtLaunchKernelGGL);
  // null when profiling is off
  hipEvent_t slot(int i) const { return enabled ? ev[head][i] : nullptr; }
  void harvest(int r) {
    if (!pending[r]) return;
    (void)hipEventSynchronize(ev[r][n]);
    for (int i = 0; i < n; i++) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, ev[r][i], ev[r][i + 1]);
      acc[i] += ms;
    }
    pending[r] = false;
    calls++;
  }
  void end_call() {
    if (!enabled) return;
    pending[head] = true;
    head = (head + 1) % kRing;
    harvest(head);  // the slot about to be reused: its call is kRing calls old
  }
  void reset(bool on) {
    for (int r = 0; r < kRing; r++) pending[r] = false;
    for (double& a : acc) a = 0;
    calls = 0;
    head = 0;
    enabled = on;
  }
  int query(float* ms, int* ncalls) {
    for (int k = 0; k < kRing; k++) harvest((head + k) % kRing);
    for (int i = 0; i < n; i++) ms[i] = (float)acc[i];
    if (ncalls) *ncalls = (int)calls;
    return RSPL_OK;
  }
};

// RSPLWT01 weight blob (format: rspl-slam_amd/weights.py).
struct Tensor {
  std::string name;
  std::vector<int64_t> dims;
  std::vector<float> data;
};
int load_blob(const char* path, std::vector<Tensor>& out);

// bytes from host-mapped pinned memory (src_mapped: its device pointer) into device memory by a copy
// kernel on stream s (copy_kernels.hip)
hipError_t upload_mapped(void* dst, const void* src_mapped, size_t bytes, hipStream_t s);
const Tensor* find(const std::vector<Tensor>& ts, const std::string& name, int64_t numel);

}  // namespace rspl
