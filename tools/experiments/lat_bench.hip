// Latency microbenchmarks for the single-workgroup fp64 solver design (cycles from s_memtime, one workgroup):
//   fma    dependent v_fma_f64 chain, 1 wave alone / 4 waves on one SIMD / with 2 busy co-resident waves
//   rcp    dependent rcp64 (v_rcp_f64 + 2 Newton) chain
//   lds    dependent ds_write_b64 -> ds_read_b64 round trips in one wave
//   ping   cross-wave hand-off through an LDS counter (wave A signals, wave B polls, B answers): per one-way trip
//   rdl    dependent readlane64 -> fma chain
// Build: hipcc --offload-arch=gfx950 -O3 lat_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kN = 1024;
typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long now() { return __builtin_readcyclecounter(); }

// mode 0: fma chain on wave 0 only; the other waves (if any) run an independent fma stream (busy) or exit
__global__ void fma_kernel(double* out, unsigned long long* cyc, int busy, double seed) {
  const int w = threadIdx.x >> 6;
  double a = seed + threadIdx.x, b = 1.0000001, c = 1e-9;
  if (w == 0) {
    if (busy >> 4) __builtin_amdgcn_s_setprio(3);
    const unsigned long long t0 = now();
#pragma unroll 16
    for (int i = 0; i < kN; i++) a = fma(a, b, c);
    const unsigned long long t1 = now();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
  } else if (busy & 15) {
    double x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
#pragma unroll 16
    for (int i = 0; i < 4 * kN; i++) {
      x0 = fma(x0, b, c);
      x1 = fma(x1, b, c);
      x2 = fma(x2, b, c);
      x3 = fma(x3, b, c);
    }
    a = x0 + x1 + x2 + x3;
  }
  out[threadIdx.x] = a;
}

__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

__global__ void rcp_kernel(double* out, unsigned long long* cyc, double seed) {
  double a = seed + threadIdx.x * 1e-3;
  const unsigned long long t0 = now();
#pragma unroll 8
  for (int i = 0; i < 256; i++) a = rcp64(a) + 1.0;
  const unsigned long long t1 = now();
  double b = seed + threadIdx.x * 1e-3;
  const unsigned long long t2 = now();
#pragma unroll 8
  for (int i = 0; i < 256; i++) b = __builtin_amdgcn_rcp(b) + 1.0;
  const unsigned long long t3 = now();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t3 - t2;
  }
  out[threadIdx.x] = a + b;
}

__global__ void lds_kernel(double* out, unsigned long long* cyc, double seed) {
  __shared__ double buf[64 * 4];
  const int lane = threadIdx.x & 63;
  double a = seed + lane;
  const unsigned long long t0 = now();
  for (int i = 0; i < 256; i++) {
    buf[(lane + i) & 63] = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    a = buf[(lane + i + 1) & 63] + 1.0;
  }
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = a;
}

// wave 0 and wave 1 (or wave 4: other SIMD) ping-pong an LDS counter
__global__ void ping_kernel(double* out, unsigned long long* cyc, int partner, int sleep) {
  __shared__ int ctr;
  const int w = threadIdx.x >> 6;
  if (threadIdx.x == 0) ctr = 0;
  __syncthreads();
  const int rounds = 256;
  if (w == 0 || w == partner) {
    const int me = w == 0 ? 0 : 1;
    const unsigned long long t0 = now();
    for (int r = 0; r < rounds; r++) {
      const int want = 2 * r + me;
      while (__hip_atomic_load(&ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
        if (sleep) __builtin_amdgcn_s_sleep(1);
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(&ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const unsigned long long t1 = now();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
  }
  out[threadIdx.x] = 0;
}

__global__ void bar_kernel(double* out, unsigned long long* cyc) {
  const unsigned long long t0 = now();
  for (int r = 0; r < 256; r++) __syncthreads();
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = 0;
}

__device__ __forceinline__ double readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__global__ void rdl_kernel(double* out, unsigned long long* cyc, double seed) {
  double a = seed + threadIdx.x;
  const unsigned long long t0 = now();
#pragma unroll 8
  for (int i = 0; i < 256; i++) a = fma(readlane64(a, i & 63), 1.0000001, a);
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = a;
}

// independent fp64 FMAs (8 chains) in one wave: issue rate; fp64 MFMA 16x16x4: independent (4 accumulators) and
// dependent chains
__global__ void thr_kernel(double* out, unsigned long long* cyc, double seed) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = seed + i + threadIdx.x;
  const unsigned long long t0 = now();
#pragma unroll 4
  for (int it = 0; it < 256; it++)
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = fma(x[i], 1.0000001, 1e-9);
  const unsigned long long t1 = now();
  double4_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) acc[i] = (double4_t){x[i], x[i + 1], 0.0, 1.0};
  const double a = x[0] * 1e-3, b = x[1] * 1e-3;
  const unsigned long long t2 = now();
#pragma unroll 4
  for (int it = 0; it < 256; it++)
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  const unsigned long long t3 = now();
  double4_t d = acc[0];
  const unsigned long long t4 = now();
#pragma unroll 4
  for (int it = 0; it < 256; it++) d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
  const unsigned long long t5 = now();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t3 - t2;
    cyc[2] = t5 - t4;
  }
  double s = d[0] + d[1] + d[2] + d[3];
#pragma unroll
  for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 8; i++) s += x[i];
  out[threadIdx.x] = s;
}

// wave 0: dependent fp64 FMA chain; waves 4, 8, 12 (same SIMD) or 1, 2, 3 (other SIMDs): back-to-back fp64 MFMAs
__global__ void mix_kernel(double* out, unsigned long long* cyc, int mode, double seed) {
  const int w = threadIdx.x >> 6;
  double a = seed + threadIdx.x;
  if (w == 0) {
    const unsigned long long t0 = now();
#pragma unroll 16
    for (int i = 0; i < kN; i++) a = fma(a, 1.0000001, 1e-9);
    const unsigned long long t1 = now();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
  } else if (mode == 3 && (w & 3) == 0) {  // fp16 MFMA stream (the front end's convolutions / GNN)
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    typedef float floatx16 __attribute__((ext_vector_type(16)));
    half8 x;
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = (_Float16)(a * 1e-3);
    floatx16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 16; j++) acc[i][j] = 0.f;
#pragma unroll 4
    for (int it = 0; it < 1024; it++)
#pragma unroll
      for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, x, acc[i], 0, 0, 0);
    a = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  } else if (mode == 4 && (w & 3) == 0) {  // fp32 VALU stream
    float x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
#pragma unroll 16
    for (int it = 0; it < 8 * kN; it++) {
      x0 = fmaf(x0, 1.0001f, 1e-9f);
      x1 = fmaf(x1, 1.0001f, 1e-9f);
      x2 = fmaf(x2, 1.0001f, 1e-9f);
      x3 = fmaf(x3, 1.0001f, 1e-9f);
    }
    a = x0 + x1 + x2 + x3;
  } else if ((mode == 1 && (w & 3) == 0) || (mode == 2 && w < 4)) {
    double4_t acc[4];
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = (double4_t){a, a, a, a};
#pragma unroll 4
    for (int it = 0; it < 512; it++)
#pragma unroll
      for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc[i], 0, 0, 0);
    a = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  }
  out[threadIdx.x] = a;
}

// one wave: LDS operand loads -> 2 dependent fp64 MFMAs -> the result read by VALU (LDS store) -> next, 256 times
__global__ void mres_kernel(double* out, unsigned long long* cyc, double seed) {
  __shared__ double buf[4 * 64 + 64];
  const int lane = threadIdx.x & 63;
  buf[lane] = seed + lane;
  buf[64 + lane] = 1e-3 * lane;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double4_t acc = {0, 0, 0, 0};
  const unsigned long long t0 = now();
  for (int it = 0; it < 256; it++) {
    const double a = buf[lane], b = buf[64 + lane];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc, 0, 0, 0);
    buf[lane] = acc[0] * 1e-9 + seed;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = acc[1];
}

int main() {
  double* d_out;
  unsigned long long* d_c;
  CK(hipMalloc(&d_out, 4096 * sizeof(double)));
  CK(hipMalloc(&d_c, 16 * sizeof(unsigned long long)));
  unsigned long long c[16];
  auto get = [&]() {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(c, d_c, sizeof(c), hipMemcpyDeviceToHost));
  };
  for (int rep = 0; rep < 2; rep++) {
    struct {
      int threads, busy;
      const char* name;
    } cf[] = {{64, 0, "1 wave"},
              {256, 1, "+3 busy waves (other SIMDs)"},
              {320, 1, "+4 busy waves (one on its SIMD)"},
              {576, 1, "+8 busy waves (two on its SIMD)"},
              {576, 1 | (3 << 4), "+8 busy waves, s_setprio 3"}};
    for (auto& f : cf) {
      hipLaunchKernelGGL(fma_kernel, dim3(1), dim3(f.threads), 0, 0, d_out, d_c, f.busy, 1.0);
      get();
      printf("fma chain, %-36s %.1f cycles per dependent v_fma_f64\n", f.name, (double)c[0] / kN);
    }
    hipLaunchKernelGGL(rcp_kernel, dim3(1), dim3(64), 0, 0, d_out, d_c, 1.5);
    get();
    printf("rcp64 (rcp + 2 Newton) + add: %.1f cycles; v_rcp_f64 + add: %.1f cycles\n", (double)c[0] / 256,
           (double)c[1] / 256);
    hipLaunchKernelGGL(lds_kernel, dim3(1), dim3(64), 0, 0, d_out, d_c, 1.0);
    get();
    printf("LDS write -> wave fence -> read -> add: %.1f cycles per round trip\n", (double)c[0] / 256);
    for (int partner : {1, 4})
      for (int sl : {0, 1}) {
        hipLaunchKernelGGL(ping_kernel, dim3(1), dim3(512), 0, 0, d_out, d_c, partner, sl);
        get();
        printf("LDS counter hand-off wave 0 <-> wave %d (%s SIMD), sleep %d: %.1f cycles one way\n", partner,
               partner % 4 == 0 ? "same" : "other", sl, (double)c[0] / 512);
      }
    for (int th : {256, 512, 768}) {
      hipLaunchKernelGGL(bar_kernel, dim3(1), dim3(th), 0, 0, d_out, d_c);
      get();
      printf("__syncthreads, %d threads: %.1f cycles\n", th, (double)c[0] / 256);
    }
    hipLaunchKernelGGL(rdl_kernel, dim3(1), dim3(64), 0, 0, d_out, d_c, 1.0);
    get();
    printf("readlane64 -> fma chain: %.1f cycles per step\n", (double)c[0] / 256);
    hipLaunchKernelGGL(mres_kernel, dim3(1), dim3(64), 0, 0, d_out, d_c, 1.0);
    get();
    printf("LDS load -> 2 dependent fp64 MFMAs -> VALU read -> LDS store: %.1f ticks per round\n", (double)c[0] / 256);
    for (int mode : {0, 1, 2, 3, 4}) {
      hipLaunchKernelGGL(mix_kernel, dim3(1), dim3(1024), 0, 0, d_out, d_c, mode, 1.0);
      get();
      printf("fp64 FMA chain with %s: %.1f ticks per FMA\n",
             mode == 0 ? "idle waves" : mode == 1 ? "3 fp64-MFMA-streaming waves on its SIMD" : mode == 2 ? "fp64 MFMA waves on the other SIMDs"
             : mode == 3 ? "3 fp16-MFMA (32x32x16) streaming waves on its SIMD" : "3 fp32-VALU streaming waves on its SIMD",
             (double)c[0] / kN);
    }
    for (int th : {64, 256, 512}) {
      hipLaunchKernelGGL(thr_kernel, dim3(1), dim3(th), 0, 0, d_out, d_c, 1.0);
      get();
      printf("%d threads: independent v_fma_f64 %.2f cycles each (wave 0); mfma_f64_16x16x4 independent %.2f, "
             "dependent %.2f cycles each\n", th, (double)c[0] / 2048, (double)c[1] / 1024, (double)c[2] / 256);
    }
  }
  return 0;
}
