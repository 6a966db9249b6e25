// Standalone microbenchmark of the C5 reduced-camera-system solve (10 < K <= 30): the pose-pair sums in the
// BA's pairfin layout (pair (a <= b) row-major over the upper triangle, 48 doubles: 36 block entries, bp, sum Y bl)
// -> x = (S + lambda I)^-1 (bp - sum Y bl) and the LM scale x.(lambda x + bp).  Variants:
//   v0  the round-6 schur_reg_kernel (copied, with per-step clock stamps)
//   v1  rspl::ba::solve_reg (ba_solve_reg.hpp), the kernel the BA launches
// Checks each against a CPU LDL^T in long double and prints device time per solve (hipEvents over many launches)
// and the v0 phase profile.  Build: hipcc --offload-arch=gfx950 -O3 -I../../rspl-slam_amd/csrc solve_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <cstring>

#include "ba_solve_reg.hpp"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

using namespace rspl::ba;

namespace v0 {
__device__ __forceinline__ int pk(int r, int c) { return r * (r + 1) / 2 + c; }
__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}
__device__ __forceinline__ bool ldl6(const double* Al, int c0, double (&L6)[15], double (&d6)[6], double (&r6)[6]) {
  double a[6][6];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int k = 0; k <= i; k++) a[i][k] = Al[pk(c0 + i, c0 + k)];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const double d = a[j][j];
    ok = ok && d > 0;
    const double r = rcp64(d);
    d6[j] = d;
    r6[j] = r;
    double u[6];
#pragma unroll
    for (int i = j + 1; i < 6; i++) u[i] = a[i][j];
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      const double l = u[i] * r;
      a[i][j] = l;
#pragma unroll
      for (int k = j + 1; k <= i; k++) a[i][k] -= l * u[k];
    }
  }
#pragma unroll
  for (int i = 0, q = 0; i < 6; i++)
#pragma unroll
    for (int k = 0; k < i; k++, q++) L6[q] = a[i][k];
  return ok;
}
__device__ __forceinline__ void pair_of(int pr, int K, int& a, int& b) {
  int base = 0;
  a = 0;
  while (pr >= base + (K - a)) {
    base += K - a;
    a++;
  }
  b = a + (pr - base);
}
__device__ __forceinline__ double readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kRegThreads = 512;
constexpr int kAsmBatch = 22;
__device__ __forceinline__ void stamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0) st[i] = __builtin_readcyclecounter();
}

__device__ __forceinline__ void wstamp(unsigned long long* st, int s, int k) {
  if (st && (threadIdx.x & 63) == 0 && s < 30) st[256 + (s * 8 + (threadIdx.x >> 6)) * 5 + k] = __builtin_readcyclecounter();
}
__global__ __launch_bounds__(kRegThreads) void kernel(const double* pairfin, int K, double lambda, double* xo,
                                                     double* out, int* fail, unsigned long long* st) {
  extern __shared__ double Al[];
  __shared__ int bad;
  const int n = 6 * K, npairs = K * (K + 1) / 2;
  double* z = Al + pk(n, 0);
  double* rdg = Al + pk(n + 1, 0);
  double* ddg = rdg + n;
  double* Ldg = ddg + n;
  double* bpl = Ldg + 15 * K;
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  stamp(st, 0);
  const int nent = npairs * 48;
  int* ptab = reinterpret_cast<int*>(ddg);
  double* ybl = rdg;
  {
    double va[kAsmBatch];
#pragma unroll
    for (int u = 0; u < kAsmBatch; u++) va[u] = pairfin[min(tid + kRegThreads * u, nent - 1)];
    for (int pr = tid; pr < npairs; pr += kRegThreads) {
      int a, b;
      pair_of(pr, K, a, b);
      ptab[2 * pr] = a;
      ptab[2 * pr + 1] = b;
    }
    __syncthreads();
    auto scatter = [&](int idx, double val) {
      if (idx >= nent) return;
      const int pr = idx / 48, v = idx - 48 * pr;
      const int pa = ptab[2 * pr], pb = ptab[2 * pr + 1];
      if (v < 36) {
        const int r = v / 6, cc = v - 6 * r;
        if (pa == pb) {
          if (cc <= r) Al[pk(6 * pa + r, 6 * pa + cc)] = val + (r == cc ? lambda : 0.0);
        } else {
          Al[pk(6 * pb + cc, 6 * pa + r)] = val;
        }
      } else if (pa == pb) {
        if (v < 42) bpl[6 * pa + v - 36] = val;
        else ybl[6 * pa + v - 42] = val;
      }
    };
#pragma unroll
    for (int u = 0; u < kAsmBatch; u++) scatter(tid + kRegThreads * u, va[u]);
#pragma unroll
    for (int u = 0; u < kAsmBatch; u++) va[u] = pairfin[min(tid + kRegThreads * (u + kAsmBatch), nent - 1)];
#pragma unroll
    for (int u = 0; u < kAsmBatch; u++) scatter(tid + kRegThreads * (u + kAsmBatch), va[u]);
  }
  if (*fail) return;
  __syncthreads();
  for (int i = tid; i < n; i += kRegThreads) z[i] = bpl[i] - ybl[i];
  __syncthreads();
  int br = -1, bc = -1;
  {
    int c = 0, base = 0;
    while (c < K && tid >= base + (K - c + 1)) {
      base += K - c + 1;
      c++;
    }
    if (c < K) {
      bc = c;
      br = c + (tid - base);
    }
  }
  const bool own = bc >= 0;
  auto row_of = [&](int a) { return br < K ? 6 * br + a : n; };
  auto valid = [&](int a, int b) { return own && (br < K ? (br > bc || b <= a) : a == 0); };
  double T[6][6];
#pragma unroll
  for (int a = 0; a < 6; a++)
#pragma unroll
    for (int b = 0; b < 6; b++) {
      const bool ok = valid(a, b);
      T[a][b] = Al[ok ? pk(row_of(a), 6 * bc + b) : 0];
      T[a][b] = ok ? T[a][b] : 0.0;
    }
  stamp(st, 1);
  const int wv = tid >> 6, lane = tid & 63;
  for (int s = 0; s < K; s++) {
    const int c0 = 6 * s, r0 = c0 + 6;
    if (bc == s)
#pragma unroll
      for (int a = 0; a < 6; a++)
#pragma unroll
        for (int b = 0; b < 6; b++)
          if (valid(a, b)) Al[pk(row_of(a), c0 + b)] = T[a][b];
    __syncthreads();
    stamp(st, 8 + 3 * s);
    wstamp(st, s, 0);
    {
      double L6[15], d6[6], r6[6];
      const bool ok = ldl6(Al, c0, L6, d6, r6);
      wstamp(st, s, 1);
      if (tid == 0) {
#pragma unroll
        for (int q = 0; q < 15; q++) Ldg[15 * s + q] = L6[q];
#pragma unroll
        for (int k = 0; k < 6; k++) {
          rdg[c0 + k] = r6[k];
          ddg[c0 + k] = d6[k];
        }
        if (!ok) bad = 1;
      }
      for (int i = r0 + tid; i <= n; i += kRegThreads) {
        double* row = Al + pk(i, c0);
        double w[6];
#pragma unroll
        for (int k = 0; k < 6; k++) w[k] = row[k];
#pragma unroll
        for (int k = 0, q = 0; k < 6; k++) {
#pragma unroll
          for (int l = 0; l < k; l++, q++) w[k] -= w[l] * L6[q];
        }
#pragma unroll
        for (int k = 0; k < 6; k++) row[k] = w[k] * r6[k];
      }
    }
    wstamp(st, s, 2);
    __syncthreads();
    stamp(st, 9 + 3 * s);
    wstamp(st, s, 3);
    if (bad) {
      if (tid == 0) atomicOr(fail, 1);
      return;
    }
    if (own && bc > s) {
#pragma unroll
      for (int l = 0; l < 6; l++) {
        const double dl = ddg[c0 + l];
        double wi[6], xk[6];
#pragma unroll
        for (int a = 0; a < 6; a++) {
          wi[a] = Al[pk(row_of(a), c0 + l)] * dl;
          xk[a] = Al[pk(6 * bc + a, c0 + l)];
        }
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
          for (int b = 0; b < 6; b++) T[a][b] -= wi[a] * xk[b];
      }
    }
    stamp(st, 10 + 3 * s);
    wstamp(st, s, 4);
  }
  __syncthreads();
  if (wv != 0) return;
  stamp(st, 2);
  double zr[3];
#pragma unroll
  for (int j = 0; j < 3; j++) zr[j] = z[min(lane + 64 * j, n - 1)];
  double Ac[3][6], Lc[15];
  auto fetch = [&](int stp, double (&Ad)[3][6], double (&Ld)[15]) {
    const int c0 = 6 * stp;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
      for (int l = 0; l < 6; l++) Ad[j][l] = Al[pk(c0 + l, min(lane + 64 * j, c0))];
#pragma unroll
    for (int q = 0; q < 15; q++) Ld[q] = Ldg[15 * stp + q];
  };
  fetch(K - 1, Ac, Lc);
  for (int stp = K - 1; stp >= 0; stp--) {
    const int c0 = 6 * stp;
    double xb[6];
#pragma unroll
    for (int k = 5; k >= 0; k--) {
      const int i = c0 + k, sl = i >> 6;
      double v = readlane64(sl == 0 ? zr[0] : sl == 1 ? zr[1] : zr[2], i & 63);
#pragma unroll
      for (int l = k + 1; l < 6; l++) v -= Lc[l * (l - 1) / 2 + k] * xb[l];
      xb[k] = v;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int i = lane + 64 * j, d = i - c0;
      double v = zr[j];
#pragma unroll
      for (int l = 0; l < 6; l++) v -= Ac[j][l] * xb[l];
      double xs = xb[0];
#pragma unroll
      for (int l = 1; l < 6; l++) xs = d == l ? xb[l] : xs;
      zr[j] = d < 0 ? v : (d < 6 ? xs : zr[j]);
    }
    if (stp > 0) fetch(stp - 1, Ac, Lc);
  }
#pragma unroll
  for (int j = 0; j < 3; j++)
    if (lane + 64 * j < n) z[lane + 64 * j] = zr[j];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < n; i += 64) xo[i] = z[i];
  stamp(st, 3);
  double sc = 0;
  for (int i = lane; i < n; i += 64) sc += z[i] * (lambda * z[i] + bpl[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sc += __shfl_xor(sc, o);
  if (lane == 0) out[0] = sc;
  stamp(st, 4);
}
size_t lds_bytes(int n) {
  const int K = n / 6;
  return sizeof(double) * ((size_t)(n + 1) * (n + 2) / 2 + 3 * n + 15 * K);
}
}  // namespace v0

struct CycleStamp {
  unsigned long long* st;
  __device__ void at(int i) const {
    if (st && threadIdx.x == 0) st[i] = __builtin_readcyclecounter();
  }
  __device__ void step(int s, int ph) const {
    if (st && threadIdx.x == 0) st[8 + 3 * s + ph] = __builtin_readcyclecounter();
  }
  __device__ void wave(int s, int k) const {
    if (st && (threadIdx.x & 63) == 0 && s < 30) st[1024 + (s * 16 + (threadIdx.x >> 6)) * 4 + k] = __builtin_readcyclecounter();
  }
};
__device__ int g_pidx[64];
template <int kAb>
__global__ __launch_bounds__(kSolveRegThreads) void vab_kernel(const double* pairfin, int K, double lambda, double* x,
                                                              double* out, int* fail, unsigned long long* st) {
  extern __shared__ double lds[];
  if (kAb == 3 && st) {  // clock probe: a 1024-long dependent fp64 FMA chain on wave 0 inside this kernel's context
    double a = lambda + threadIdx.x;
    const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 16
    for (int i = 0; i < 1024; i++) a = fma(a, 1.0000001, 1e-9);
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) st[2000] = t1 - t0;
    if (a == 12345.0) x[0] = a;
  }
  solve_reg<NoStamp, kAb>(pairfin, K, lambda, x, out, fail, g_pidx, K, lds, NoStamp{});
}
__global__ __launch_bounds__(kSolveRegThreads) void v1_kernel(const double* pairfin, int K, double lambda, double* x,
                                                             double* out, int* fail, unsigned long long* st) {
  extern __shared__ double lds[];
  solve_reg(pairfin, K, lambda, x, out, fail, g_pidx, K, lds, CycleStamp{st});
}

// the pivot phase alone (one wave, no other work): ldl6 of a fixed SPD block from LDS + three panel rows per lane,
// repeated; cycles per repetition
__global__ void piv_kernel(double* out, unsigned long long* cyc, int nrows) {
  __shared__ double Col[6 * 192];
  __shared__ double Pn[6 * 192];
  __shared__ double Lg[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 6 * 192; i += 64) Col[i] = (i % 7 == 0) ? 4.0 + (i % 5) : 0.1 * ((i * 37) % 11) / 11.0;
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < 64; rep++) {
    double a[6][6], L6[15], d6[6], r6[6];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
      for (int k = 0; k <= i; k++) a[i][k] = Col[6 * i + k] + (i == k ? acc * 1e-30 : 0.0);
    double w[3][6];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int row = 6 + lane + 64 * j;
      if (row < nrows) sr_ld6(Col + 6 * row, w[j]);
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const double d = a[j][j];
      const double r = sr_rcp64(d);
      d6[j] = d;
      r6[j] = r;
      double u[6];
#pragma unroll
      for (int i = j + 1; i < 6; i++) u[i] = a[i][j];
#pragma unroll
      for (int i = j + 1; i < 6; i++) {
        const double l = u[i] * r;
        a[i][j] = l;
#pragma unroll
        for (int k = j + 1; k <= i; k++) a[i][k] -= l * u[k];
      }
    }
#pragma unroll
    for (int i = 0, q = 0; i < 6; i++)
#pragma unroll
      for (int k = 0; k < i; k++, q++) L6[q] = a[i][k];
    if (lane == 0)
#pragma unroll
      for (int q = 0; q < 15; q++) Lg[q] = L6[q];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int row = 6 + lane + 64 * j;
      if (row < nrows) {
#pragma unroll
        for (int k = 0, q = 0; k < 6; k++)
#pragma unroll
          for (int l = 0; l < k; l++, q++) w[j][k] -= w[j][l] * L6[q];
#pragma unroll
        for (int k = 0; k < 6; k++) {
          const double xv = w[j][k] * r6[k];
          Pn[k * 192 + row] = xv;
          acc += xv * d6[k];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (lane == 0) cyc[0] = t1 - t0;
  out[lane] = acc;
}

// the backward substitution alone (1024 threads, synthetic panels): cycles per pose step; kV: sr_backsub variant
template <bool kV>
__global__ __launch_bounds__(kSolveRegThreads) void bs_kernel(double* out, unsigned long long* cyc, int K) {
  extern __shared__ double lds[];
  const SolveRegLayout Ly(K);
  for (int i = threadIdx.x; i < Ly.total; i += blockDim.x) lds[i] = 1e-3 * ((i * 37) % 101);
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  if (threadIdx.x < 64) sr_backsub<kV>(lds, lds + Ly.ld, lds + Ly.xs, K);
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  for (int i = threadIdx.x; i < 6 * K; i += blockDim.x) out[i] = lds[Ly.xs + i];
}

static int pair_index_h(int c, int a, int K) { return c * K - c * (c - 1) / 2 + (a - c); }

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 29;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  const int n = 6 * K, npairs = K * (K + 1) / 2;
  const double lambda = 1e-3;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> N01;
  // S = B B^T / m + diag: SPD, moderately conditioned (like a reduced camera system)
  const int m = n + 40;
  std::vector<double> B((size_t)n * m), S((size_t)n * n, 0.0);
  for (auto& v : B) v = N01(rng);
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      long double s = 0;
      for (int k = 0; k < m; k++) s += (long double)B[(size_t)i * m + k] * B[(size_t)j * m + k];
      S[(size_t)i * n + j] = S[(size_t)j * n + i] = (double)(s / m) * (1.0 + 0.3 * ((i / 6) % 3)) * (1.0 + 0.3 * ((j / 6) % 3));
    }
  std::vector<double> bp(n), ybl(n);
  for (int i = 0; i < n; i++) {
    bp[i] = N01(rng);
    ybl[i] = 0.1 * N01(rng);
  }
  std::vector<double> pf((size_t)npairs * 48, 0.0);
  for (int a = 0; a < K; a++)
    for (int b = a; b < K; b++) {
      double* p = pf.data() + 48 * pair_index_h(a, b, K);
      for (int r = 0; r < 6; r++)
        for (int cc = 0; cc < 6; cc++) p[r * 6 + cc] = S[(size_t)(6 * a + r) * n + 6 * b + cc];
      if (a == b)
        for (int r = 0; r < 6; r++) {
          p[36 + r] = bp[6 * a + r];
          p[42 + r] = ybl[6 * a + r];
        }
    }
  // reference: LDL^T of S + lambda I in long double
  std::vector<long double> A((size_t)n * n), zz(n);
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) A[(size_t)i * n + j] = S[(size_t)i * n + j] + (i == j ? lambda : 0.0);
    zz[i] = (long double)bp[i] - ybl[i];
  }
  std::vector<long double> lc(n);
  for (int j = 0; j < n; j++) {
    for (int i = j + 1; i < n; i++) lc[i] = A[(size_t)i * n + j] / A[(size_t)j * n + j];
    for (int i = j + 1; i < n; i++) {
      for (int k = j + 1; k <= i; k++) A[(size_t)i * n + k] -= lc[i] * A[(size_t)k * n + j];
      zz[i] -= lc[i] * zz[j];
    }
    for (int i = j + 1; i < n; i++) A[(size_t)i * n + j] = lc[i];
  }
  std::vector<long double> xr(n);
  for (int i = n - 1; i >= 0; i--) {
    long double v = zz[i] / A[(size_t)i * n + i];
    for (int k = i + 1; k < n; k++) v -= A[(size_t)k * n + i] * xr[k];
    xr[i] = v;
  }
  long double scr = 0;
  for (int i = 0; i < n; i++) scr += xr[i] * (lambda * xr[i] + bp[i]);

  double *d_pf, *d_x, *d_out;
  int* d_fail;
  unsigned long long* d_st;
  CK(hipMalloc(&d_pf, pf.size() * sizeof(double)));
  CK(hipMalloc(&d_x, 256 * sizeof(double)));
  CK(hipMalloc(&d_out, 8 * sizeof(double)));
  CK(hipMalloc(&d_fail, sizeof(int)));
  CK(hipMalloc(&d_st, 4096 * sizeof(unsigned long long)));
  CK(hipMemcpy(d_pf, pf.data(), pf.size() * sizeof(double), hipMemcpyHostToDevice));
  CK(hipMemset(d_fail, 0, sizeof(int)));
  {
    int pid[64];
    for (int i = 0; i < 64; i++) pid[i] = i;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_pidx), pid, sizeof(pid)));
  }
  const size_t l0 = v0::lds_bytes(n), l1 = solve_reg_lds_bytes(K);
  CK(hipFuncSetAttribute((const void*)v0::kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l0));
  CK(hipFuncSetAttribute((const void*)v1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1));
  {
    std::vector<double> xb0(n), xb(n);
    auto run_bs = [&](auto kern, int v) {
      CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
      unsigned long long best = ~0ull;
      for (int r = 0; r < 5; r++) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(kSolveRegThreads), solve_reg_lds_bytes(K), 0, d_x, d_st, K);
        CK(hipDeviceSynchronize());
        unsigned long long c;
        CK(hipMemcpy(&c, d_st, sizeof(c), hipMemcpyDeviceToHost));
        best = c < best ? c : best;
      }
      CK(hipMemcpy(v == 0 ? xb0.data() : xb.data(), d_x, n * sizeof(double), hipMemcpyDeviceToHost));
      const bool same = v == 0 || memcmp(xb0.data(), xb.data(), n * sizeof(double)) == 0;
      printf("backward substitution alone, variant %d: %.0f cycles (%.0f per pose step)%s\n", v, (double)best,
             (double)best / K, same ? "" : "  RESULT DIFFERS");
    };
    run_bs(bs_kernel<false>, 0);  // (variant 0: the previous form; 1: the ping-pong form of the library)
    run_bs(bs_kernel<true>, 1);
  }
  for (int nr : {6, 70, 175}) {
    hipLaunchKernelGGL(piv_kernel, dim3(1), dim3(64), 0, 0, d_x, d_st, nr);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, d_st, sizeof(c), hipMemcpyDeviceToHost));
    printf("pivot phase alone (one wave, %d rows): %.0f cycles per step\n", nr - 6, (double)c / 64);
  }
  hipEvent_t e0, e1;
  {
    CK(hipFuncSetAttribute((const void*)vab_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<12>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    CK(hipFuncSetAttribute((const void*)vab_kernel<15>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_reg_lds_bytes(K)));
    hipEvent_t a0, a1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    for (int ab : {0, 1, 2, 3, 4, 8, 12, 15}) {
      auto L = [&]() {
        const size_t lb = solve_reg_lds_bytes(K);
        if (ab == 0) hipLaunchKernelGGL(vab_kernel<0>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 1) hipLaunchKernelGGL(vab_kernel<1>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 2) hipLaunchKernelGGL(vab_kernel<2>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 3) hipLaunchKernelGGL(vab_kernel<3>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 4) hipLaunchKernelGGL(vab_kernel<4>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 8) hipLaunchKernelGGL(vab_kernel<8>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 12) hipLaunchKernelGGL(vab_kernel<12>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
        if (ab == 15) hipLaunchKernelGGL(vab_kernel<15>, dim3(1), dim3(kSolveRegThreads), lb, 0, d_pf, K, lambda, d_x, d_out, d_fail, nullptr);
      };
      for (int i = 0; i < 3; i++) L();
      CK(hipEventRecord(a0));
      for (int i = 0; i < reps; i++) L();
      CK(hipEventRecord(a1));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      CK(hipMemset(d_fail, 0, sizeof(int)));
      if (ab == 3) {
        hipLaunchKernelGGL(vab_kernel<3>, dim3(1), dim3(kSolveRegThreads), solve_reg_lds_bytes(K), 0, d_pf, K, lambda, d_x, d_out, d_fail, d_st);
        CK(hipDeviceSynchronize());
        unsigned long long c;
        CK(hipMemcpy(&c, d_st + 2000, sizeof(c), hipMemcpyDeviceToHost));
        printf("clock probe in the solver's context: %.2f ticks per dependent fp64 FMA (lat_bench: 6.5-7.5)\n", c / 1024.0);
      }
      printf("ablation %d (%s): %.2f us per solve\n", ab,
             ab == 0 ? "full" : ab == 1 ? "no trailing MFMA" : ab == 2 ? "no pivot arithmetic" : ab == 3 ? "neither" : ab == 4 ? "no tile assembly" : ab == 8 ? "no pairfin loads" : ab == 12 ? "neither assembly part" : "skeleton only", 1e3 * ms / reps);
    }
  }
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> x0;
  for (int v = 0; v < 2; v++) {
    auto launch = [&](unsigned long long* st) {
      if (v == 0)
        hipLaunchKernelGGL(v0::kernel, dim3(1), dim3(v0::kRegThreads), l0, 0, d_pf, K, lambda, d_x, d_out, d_fail, st);
      else
        hipLaunchKernelGGL(v1_kernel, dim3(1), dim3(kSolveRegThreads), l1, 0, d_pf, K, lambda, d_x, d_out, d_fail, st);
    };
    CK(hipMemset(d_x, 0, 256 * sizeof(double)));
    CK(hipMemset(d_fail, 0, sizeof(int)));
    CK(hipMemset(d_st, 0, 4096 * sizeof(unsigned long long)));
    launch(d_st);
    CK(hipDeviceSynchronize());
    std::vector<double> x(n);
    double sc;
    int fl;
    std::vector<unsigned long long> st(4096);
    CK(hipMemcpy(x.data(), d_x, n * sizeof(double), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&sc, d_out, sizeof(double), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&fl, d_fail, sizeof(int), hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), d_st, 4096 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double err = 0, xm = 0;
    for (int i = 0; i < n; i++) {
      err = fmax(err, fabs((double)(x[i] - xr[i])));
      xm = fmax(xm, fabs((double)xr[i]));
    }
    for (int i = 0; i < 3; i++) launch(nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; i++) launch(nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (v == 0) x0 = x;
    double dv = 0;
    for (int i = 0; i < n; i++) dv = fmax(dv, fabs(x[i] - x0[i]));
    printf("  max|x - x_v0| %.3e\n", dv);
    printf("v%d K=%d n=%d: %.2f us per solve, max|dx| %.3e (|x| %.3e), sc rel %.3e, fail %d\n", v, K, n,
           1e3 * ms / reps, err, xm, fabs((double)((sc - scr) / scr)), fl);
    if (st[0] && st[1]) {  // cycle stamps (s_memtime: shader clock)
      auto c = [&](int a, int b) { return (double)(st[b] - st[a]); };
      printf("  cycles: asm %.0f  factor %.0f  back %.0f  tail %.0f\n", c(0, 1), st[2] ? c(1, 2) : -1.0,
             st[3] ? c(2, 3) : -1.0, st[4] ? c(3, 4) : -1.0);
      printf(v == 0 ? "  per step (barrier wait | pivot+panel | trailing):" : "  per step (gap | inputs+pivot | panel):");
      unsigned long long prev = st[1];
      for (int s = 0; s < K; s++) {
        const unsigned long long a = st[8 + 3 * s], b = st[9 + 3 * s], d = st[10 + 3 * s];
        if (!a) break;
        printf(" [%d %.0f|%.0f|%.0f]", s, (double)(a - prev), (double)(b - a), (double)(d - b));
        prev = d;
      }
      printf("\n");
    }
    if (v == 1)
      for (int s : {0, 1, 5, 10, 20}) {
        if (s >= K) continue;
        printf("  v3 step %d: pivot waves [bar A -> ldl6 | -> panel | -> bar B], tile waves [extract+bars | MFMA issue]:", s);
        for (int w = 0; w < 16; w++) {
          const unsigned long long* q = st.data() + 1024 + (s * 16 + w) * 4;
          if (!q[0]) continue;
          if (w < 3) printf(" w%d[%lld|%lld|%lld]", w, (long long)(q[1] - q[0]), (long long)(q[2] - q[1]), (long long)(q[3] - q[2]));
          else printf(" w%d[%lld|%lld]", w, (long long)(q[1] - q[0]), (long long)(q[2] - q[1]));
        }
        printf("\n");
      }
    if (v == 0)
      for (int s : {0, 1, 5, 10, 20}) {
        if (s >= K) continue;
        printf("  v0 step %d per wave [bar1->ldl6 | ->panel done | ->bar2 | ->trail done]:", s);
        for (int w = 0; w < 8; w++) {
          const unsigned long long* q = st.data() + 256 + (s * 8 + w) * 5;
          if (!q[0]) continue;
          printf(" w%d[%lld|%lld|%lld|%lld]", w, (long long)(q[1] - q[0]), (long long)(q[2] - q[1]),
                 (long long)(q[3] - q[2]), q[4] ? (long long)(q[4] - q[3]) : -1LL);
        }
        printf("\n");
      }
  }
  return 0;
}
