// Microbenchmark: cost of a dependent kernel boundary vs a device-wide barrier inside a
// persistent kernel (256 workgroups), to size the BA's per-stage synchronisation.
//   hipcc --offload-arch=gfx950 -O3 tools/sync_bench.hip -o /tmp/sync_bench && /tmp/sync_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void empty_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

// generation barrier: arrive with release, spin relaxed, acquire after
__device__ void grid_sync(unsigned* cnt, unsigned* gen, unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nb - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g && ++spins < (1L << 26))
        __builtin_amdgcn_s_sleep(1);
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
  }
  __syncthreads();
}

__global__ void persistent_kernel(unsigned* bar, int iters, int* sink) {
  for (int i = 0; i < iters; i++) grid_sync(bar, bar + 32, gridDim.x);
  if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] = iters;
}

int main() {
  int* d;
  unsigned* bar;
  hipMalloc(&d, 64);
  hipMalloc(&bar, 256);
  hipMemset(d, 0, 64);
  hipMemset(bar, 0, 256);
  hipStream_t s;
  hipStreamCreate(&s);
  const int N = 2000;
  for (int nb : {64, 256}) {
    for (int rep = 0; rep < 2; rep++) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(256), 0, s, d);
      hipStreamSynchronize(s);
      auto t1 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(persistent_kernel, dim3(nb), dim3(256), 0, s, bar, N, d);
      hipStreamSynchronize(s);
      auto t2 = std::chrono::steady_clock::now();
      if (rep)
        printf("grid %3d: kernel boundary %.2f us, grid barrier %.2f us\n", nb,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
               std::chrono::duration<double, std::micro>(t2 - t1).count() / N);
    }
  }
  return 0;
}
