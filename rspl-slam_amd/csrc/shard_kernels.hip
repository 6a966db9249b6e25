// In-process group all-reduce (rspl_group): the sum of the ranks' buffers, formed in rank order
// (deterministic, identical on every rank), written to the calling rank's staging buffer.
#include <hip/hip_runtime.h>

#include "shard.hpp"

namespace rspl {
namespace shard {

__global__ __launch_bounds__(256) void group_sum_kernel(SumArgs a) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < a.count; i += (size_t)gridDim.x * 256) {
    double s = a.src[0][i];
    for (int r = 1; r < a.n; r++) s += a.src[r][i];
    a.dst[i] = s;
  }
}

hipError_t group_sum(const SumArgs& a, hipStream_t s) {
  if (a.count == 0) return hipSuccess;
  const int blocks = (int)std::min<size_t>((a.count + 255) / 256, 1024);
  hipLaunchKernelGGL(group_sum_kernel, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace shard
}  // namespace rspl
