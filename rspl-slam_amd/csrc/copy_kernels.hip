// Host -> device uploads as a kernel: the call's packed inputs read over PCIe from host-mapped pinned
// staging memory (its device pointer) by 16-byte loads, written to device memory -- no copy engine.
// hipMemcpyAsync's H2D path stalled the first BA calls after the bench warmup by 7-10 ms each
// (profiles/r05_bench_20step_before.json); for the small per-call uploads of the BA, PnP and
// FrameOptimization handles a kernel on the call's own stream is also the shorter path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "common.hpp"

namespace rspl {

__global__ __launch_bounds__(256) void upload_kernel(uint4* dst, const uint4* src, size_t n16, uint8_t* dtail,
                                                     const uint8_t* stail, int ntail) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (size_t i = t; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
  if (t < (size_t)ntail) dtail[t] = stail[t];
}

hipError_t upload_mapped(void* dst, const void* src_mapped, size_t bytes, hipStream_t s) {
  const size_t n16 = bytes / 16;
  const int ntail = (int)(bytes - 16 * n16);
  if (!bytes) return hipSuccess;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((n16 + 255) / 256, 1024));
  hipLaunchKernelGGL(upload_kernel, dim3(blocks), dim3(256), 0, s, static_cast<uint4*>(dst),
                     static_cast<const uint4*>(src_mapped), n16, static_cast<uint8_t*>(dst) + 16 * n16,
                     static_cast<const uint8_t*>(src_mapped) + 16 * n16, ntail);
  return hipGetLastError();
}

}  // namespace rspl
