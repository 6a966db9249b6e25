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

// RSPLWT01 weight blob (format: rspl-slam_amd/weights.py).
struct Tensor {
  std::string name;
  std::vector<int64_t> dims;
  std::vector<float> data;
};
int load_blob(const char* path, std::vector<Tensor>& out);
const Tensor* find(const std::vector<Tensor>& ts, const std::string& name, int64_t numel);

}  // namespace rspl
