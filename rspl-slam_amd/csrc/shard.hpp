#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>

namespace rspl {
namespace shard {

constexpr int kMaxGroup = 16;

struct SumArgs {
  const double* src[kMaxGroup];
  double* dst;
  size_t count;
  int n;
};

hipError_t group_sum(const SumArgs& a, hipStream_t s);

}  // namespace shard
}  // namespace rspl
