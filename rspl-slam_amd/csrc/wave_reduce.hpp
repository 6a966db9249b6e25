// Wavefront (wave64) reductions shared by the single-wave fp64 solvers (frame_kernels.hip,
// pnp_kernels.hip): DPP all-reduce sums that leave the bitwise-same value in every lane, a
// reduce-scatter all-reduce of the 28-value 6x6 normal equations, and a full-precision
// reciprocal without the divide sequence.
#pragma once
#include <hip/hip_runtime.h>

namespace rspl {
namespace wave {

constexpr int kNV = 28;  // 21 upper-triangular H entries, 6 b entries, chi2

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rdlaned(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// wave64 all-reduce (sum), identical bits in every lane
__device__ __forceinline__ double wsum(double v) {
  v += dppd<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppd<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppd<0x141>(v);  // row_half_mirror
  v += dppd<0x140>(v);  // row_mirror
  return (rdlaned(v, 0) + rdlaned(v, 16)) + (rdlaned(v, 32) + rdlaned(v, 48));
}
__device__ __forceinline__ int wsum_int(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// All-reduce of the 28 system values across the wave as a reduce-scatter: 5 exchange steps
// (xor 32, 16, 8, 4, 2) each halve the values a lane keeps (32 -> 1, padded), one xor-1 step
// completes the sum, then every value is read back from its owner lane with readlane (wave-
// uniform).  32 double exchanges instead of 28 x 6 for per-value butterflies; each value is
// summed by one fixed tree (a + b == b + a in the pair), so the result is deterministic.
// The xor-32 and xor-16 steps (24 of the 32 exchanges) are gfx950's v_permlane32_swap /
// v_permlane16_swap (VALU lane swaps, no LDS-unit round trip); xor 2 and 1 are DPP quad
// permutes; only xor 8 and 4 go through ds_bpermute.  Same pairs, same operands: the sums are
// bitwise those of a plain shuffle tree.
__device__ __forceinline__ double shx(double v, int o) { return __shfl_xor(v, o); }
// lanes (l, l ^ 32) [K32] or (l, l ^ 16) [!K32]: a + partner's a in the lower lane, b + partner's b in the upper
template <bool K32>
__device__ __forceinline__ double swap_sum(double a, double b) {
  const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  unsigned p0, p1, q0, q1;
  if constexpr (K32) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    p0 = lo[0]; q0 = lo[1]; p1 = hi[0]; q1 = hi[1];
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)y, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    p0 = lo[0]; q0 = lo[1]; p1 = hi[0]; q1 = hi[1];
  }
  // lower lane: p = own a, q = partner's a; upper lane: p = partner's b, q = own b
  return __longlong_as_double((long long)((unsigned long long)p1 << 32 | p0)) +
         __longlong_as_double((long long)((unsigned long long)q1 << 32 | q0));
}
// wave64 all-reduce (sum) with the partners of the xor butterfly (32, 16, 8, 4, 2, 1) -- bitwise the result of
// `for (o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o)` (each step adds the same pair; a + b == b + a) -- on VALU lane
// moves: v_permlane32_swap / v_permlane16_swap, DPP row_ror:8 (= xor 8 in a 16-lane row), row_shl:4 / row_shr:4
// selected by lane bit 2, quad permutes; no ds_bpermute round trips on the chain
__device__ __forceinline__ double xsum64(double v) {
  v = swap_sum<true>(v, v);
  v = swap_sum<false>(v, v);
  v += dppd<0x128>(v);  // row_ror:8
  {
    const double up = dppd<0x104>(v), dn = dppd<0x114>(v);  // row_shl:4 (lane + 4) / row_shr:4 (lane - 4)
    v += (threadIdx.x & 4) ? dn : up;
  }
  v += dppd<0x4E>(v);
  return v + dppd<0xB1>(v);
}
// the reduce-scatter: lane L returns the wave's sum of value L >> 1 (values 28..31: 0)
__device__ __forceinline__ double wave_scatter28(const double (&acc)[kNV], int lane) {
  double v[32];
#pragma unroll
  for (int k = 0; k < 32; k++) v[k] = k < kNV ? acc[k] : 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) v[k] = swap_sum<true>(v[k], v[16 + k]);
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = swap_sum<false>(v[k], v[8 + k]);
#pragma unroll
  for (int o = 8, h = 4; o >= 4; o >>= 1, h >>= 1) {
    const bool up = lane & o;  // keep the upper half of the current h*2 values
#pragma unroll
    for (int k = 0; k < h; k++) {
      const double keep = up ? v[h + k] : v[k];
      const double send = up ? v[k] : v[h + k];
      v[k] = keep + shx(send, o);
    }
  }
  {
    const bool up = lane & 2;
    const double keep = up ? v[1] : v[0], send = up ? v[0] : v[1];
    v[0] = keep + dppd<0x4E>(send);  // quad_perm [2,3,0,1]: lane ^ 2
  }
  return v[0] + dppd<0xB1>(v[0]);  // quad_perm [1,0,3,2]: lane ^ 1
}
__device__ __forceinline__ void wave_allreduce28(double (&acc)[kNV], int lane) {
  const double s = wave_scatter28(acc, lane);
#pragma unroll
  for (int j = 0; j < kNV; j++) acc[j] = rdlaned(s, 2 * j);
}

__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

// A workgroup of NW waves (FrameOptimization's frame, PnP's refinement): a wave-reduced value (equal on every
// lane) combined across the NW waves in wave order through LDS; every thread gets the same sum.
template <int NW, int N>
__device__ __forceinline__ void block_combine(double (&v)[N]) {
  if constexpr (NW > 1) {
    __shared__ double cb[NW][N];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < N; k++) cb[wv][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; k++) {
      double t = cb[0][k];
#pragma unroll
      for (int w = 1; w < NW; w++) t += cb[w][k];
      v[k] = t;
    }
    __syncthreads();  // cb is reused by the next combine
  }
}
// wave_allreduce28 + block_combine in one: the waves' scattered sums (lane 2j: value j) go to LDS, lane j < 28 of
// every wave adds value j over the waves in wave order, and readlane hands each sum to the whole wave -- NW reads
// per lane instead of NW x 28, the same additions in the same order (bitwise the two-step result)
template <int NW>
__device__ __forceinline__ void block_allreduce28(double (&acc)[kNV], int lane) {
  const double s = wave_scatter28(acc, lane);
  if constexpr (NW == 1) {
#pragma unroll
    for (int j = 0; j < kNV; j++) acc[j] = rdlaned(s, 2 * j);
  } else {
    __shared__ double cs[NW][32];
    const int wv = threadIdx.x >> 6;
    if (!(lane & 1)) cs[wv][lane >> 1] = s;
    __syncthreads();
    double t = cs[0][lane & 31];
#pragma unroll
    for (int w = 1; w < NW; w++) t += cs[w][lane & 31];
#pragma unroll
    for (int j = 0; j < kNV; j++) acc[j] = rdlaned(t, j);
    __syncthreads();  // cs is reused by the next combine
  }
}
template <int NW>
__device__ __forceinline__ int block_sum_int(int v) {
  v = wsum_int(v);
  if constexpr (NW > 1) {
    __shared__ int ci[NW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) ci[wv] = v;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) t += ci[w];
    __syncthreads();
    v = t;
  }
  return v;
}

}  // namespace wave
}  // namespace rspl
