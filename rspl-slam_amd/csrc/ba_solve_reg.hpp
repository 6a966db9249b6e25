// Reduced camera system of the local BA for 10 < K <= 30 optimised poses (C5's 30-keyframe window, n = 6K = 174):
// (S + lambda I) x = bp - sum Y bl from the pose-pair sums, in ONE 768-thread workgroup.  g2o solves the reduced
// system with a dense factorisation (g2o_optimization.cc:26-36, BlockSolver + LinearSolverEigen); here a
// right-looking LDL^T blocked by the 6x6 pose blocks, every pivot a reciprocal (v_rcp_f64 + two Newton steps).
//
// Measured on gfx950 (tools/experiments/lat_bench.hip, s_memtime ticks): a dependent v_fma_f64 7.5, an independent
// one 5.6 per wave instruction, v_mfma_f64_16x16x4f64 64 (1,024 FMAs), a workgroup barrier 15-20, an LDS round trip
// 84, a cross-wave hand-off through an LDS counter ~240.  So: barriers, not flags; the trailing update on fp64 MFMA
// (one 16 x 16 tile = 2 MFMAs per pose step: 2.9x the VALU rate per instruction, and its operands are 2 LDS loads per
// lane instead of 72); and the pivot chain on one wave per SIMD.
//
// The matrix (lower triangle of S + lambda I, plus the rhs z = bp - sum Y bl as row n) lives in registers as 16 x 16
// MFMA accumulator tiles (I >= J; element (16 I + 4 q + l / 16, 16 J + l % 16) in item q of lane l), dealt to the 13
// waves round-robin in order of decreasing tile column, so the shrinking trailing triangle stays spread over every
// wave and SIMD at every step.  Pose step s (c0 = 6s), two barriers:
//   (1) the owners of the tiles holding columns c0 .. c0 + 5 write them (rows c0 .. n) to the column buffer;
//   (2) waves 0..3 (one per SIMD) factor the 6x6 pivot block (uniform, redundant) and form one panel row each
//       (X = a L^-T D^-1) into panel s (transposed: entry (k, row)) and -X diag(D) into the MFMA A-operand buffer;
//   (3) every wave applies the panel to its tiles that reach the trailing rows / columns: acc += (-X D) X^T, K = 6
//       as two 16x16x4 steps (k = 6, 7 zero), operands outside rows / columns c0 + 6 .. n zero.
// The panels stay for the backward substitution L^T x = y (y = D^-1 L^-1 z: each panel's row n), run on wave 0 by
// pose step with the next step's L entries requested ahead.  A non-positive pivot or a failed landmark inversion
// upstream (*fail) leaves x untouched and sets *fail.
#pragma once
#include <hip/hip_runtime.h>

#include "wave_reduce.hpp"

namespace rspl {
namespace ba {

constexpr int kSolveRegThreads = 768;
constexpr int kSolveRegWaves = kSolveRegThreads / 64;
constexpr int kSolveRegMaxK = 30;
// Waves are dealt to the SIMDs round-robin (wave w on SIMD w % 4).  fp64 MFMA and fp64 VALU share a SIMD's
// datapath: a dependent v_fma_f64 chain beside three waves streaming v_mfma_f64 on its SIMD took 390 ticks per FMA
// instead of 6.5 (lat_bench.hip).  So SIMD 0 carries the pivot chain alone (wave 0; waves 4 and 8 only join the
// barriers) and the tiles live on SIMDs 1..3.  768 threads: 3 waves per SIMD, 168 VGPRs each.
constexpr int kSrTileWaves = 9;   // waves w % 4 != 0
constexpr int kSrMaxTiles = 9;    // tiles per tile wave: NT (NT + 1) / 2 <= 9 * 9 for NT = ceil((6K + 1) / 16) <= 12
static_assert(((6 * kSolveRegMaxK + 16) / 16) * ((6 * kSolveRegMaxK + 16) / 16 + 1) / 2 <= kSrTileWaves * kSrMaxTiles,
              "tiles per wave");
static_assert(6 * kSolveRegMaxK + 1 - 6 <= 3 * 64, "three panel rows per pivot lane");
static_assert(sizeof(double) * 20480 >= 163840, "");

typedef double sr_d4 __attribute__((ext_vector_type(4)));

// panel s: R_s = n - 6s - 4 doubles per k (rows 6s + 6 .. n, padded to even); its offset in the panel store
__host__ __device__ constexpr int sr_panel_ld(int s, int n) { return n - 6 * s - 4; }
__host__ __device__ constexpr int sr_panel_off(int s, int n) { return 6 * (s * (n - 4) - 3 * s * (s - 1)); }

struct SolveRegLayout {
  int n, K, npairs;
  int xd, col, ld, y, xs, bp, ybl, total;  // offsets in doubles (panels at 0)
  __host__ __device__ explicit SolveRegLayout(int K_) : n(6 * K_), K(K_), npairs(K_ * (K_ + 1) / 2) {
    const int ln = (n + 2) & ~1;
    xd = sr_panel_off(K, n);  // [2][6][ln] -X diag(D) of the current step, by row (double-buffered by parity)
    col = xd + 12 * ln;       // [n + 1][6] the pivot column of the current step (rows c0 .. n)
    int end = col + 6 * (n + 1);
    const int stage = 38 * npairs;  // assembly staging (aliases the above)
    end = end > stage ? end : stage;
    ld = end;          // [K][16] each pivot block's strictly-lower unit L (15 used)
    y = ld + 16 * K;   // [n + 2] y of the next block (backward substitution); sum Y bl during the assembly
    xs = y + ln;       // [n + 2] x
    bp = xs + ln;      // [n] pose gradient bp (LM scale)
    ybl = y;
    total = bp + n;
  }
};
inline size_t solve_reg_lds_bytes(int K) { return sizeof(double) * (size_t)SolveRegLayout(K).total; }

__device__ __forceinline__ double sr_rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

__device__ __forceinline__ void sr_ld6(const double* p, double (&v)[6]) {  // 16-byte aligned
  const double2* q = reinterpret_cast<const double2*>(p);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const double2 t = q[i];
    v[2 * i] = t.x;
    v[2 * i + 1] = t.y;
  }
}

// tile t of the wave-ordered tile list (decreasing tile column J, then increasing row I >= J) -> (I, J)
__device__ __forceinline__ void sr_tile_of(int t, int NT, int& I, int& J) {
  J = NT - 1;
  int base = 0;
  while (t >= base + (NT - J)) {
    base += NT - J;
    J--;
  }
  I = J + (t - base);
}

__device__ __forceinline__ double sr_readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Backward substitution L^T x = y after the factor, on wave 0 alone (rows i = lane + 64 j, j < 3; no barriers).
// y_i = X_{s(i)}(n, i % 6).  Pose step st: the block's six y by readlane from the lanes that hold them (no LDS on the
// chain: a wave fence there would also wait for the prefetches), x_k = y_k - sum_{l > k} L(l, k) x_l with the
// block's unit L, then every row i < 6 st: y_i -= sum_l L(6 st + l, i) x_l with L(6 st + l, i) =
// X_{s(i)}(6 st + l, i % 6).  The next step's L entries (three 16-byte loads per row) and unit L (eight) are
// requested a step ahead into the other of two operand sets (two steps per loop iteration: no register copies), by
// every lane (no exec mask, so the compiler waits for exactly the loads a step needs; rows >= 6 st take in-bounds
// entries of no meaning -- their y was read before the step's update and is never read again).  Micro-benchmark
// (solve_bench.hip, K = 29): 1,038 -> 739 cycles per pose step, x bitwise the same.  x -> xv[0 .. n) (lane 0).
// (sr_backsub's unrolled form) step st's operands: the panel entries of every lane's rows (in-bounds for all lanes,
// no exec mask) and the block's unit L
__device__ __forceinline__ void sr_bs_fetch(const double* P, const double* Ldg, const int (&pb)[3], int st,
                                            double (&A)[3][6], double (&L)[16]) {
#pragma unroll
  for (int j = 0; j < 3; j++) sr_ld6(P + max(pb[j] + 6 * st, 0), A[j]);
  const double2* q = reinterpret_cast<const double2*>(Ldg + 16 * st);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const double2 t = q[i];
    L[2 * i] = t.x;
    L[2 * i + 1] = t.y;
  }
}
__device__ __forceinline__ void sr_bs_step(const double* P, const double* Ldg, double* xv, const int (&pb)[3], int st,
                                           int lane, double& z0, double& z1, double& z2, const double (&Ac)[3][6],
                                           const double (&Lc)[16], double (&An)[3][6], double (&Ln)[16]) {
  const int c0 = 6 * st;
  sr_bs_fetch(P, Ldg, pb, max(st - 1, 0), An, Ln);  // the next step's operands, ahead of this step's chain
  double yb[6], xb[6];
  const int s0 = c0 >> 6, s5 = (c0 + 5) >> 6;
  if (s0 == s5) {
    const double src = s0 == 0 ? z0 : (s0 == 1 ? z1 : z2);
#pragma unroll
    for (int k = 0; k < 6; k++) yb[k] = sr_readlane64(src, (c0 + k) & 63);
  } else {  // (rows 60..65 or 126..131: the block straddles two slots)
    const double lo = s0 == 0 ? z0 : z1, hi = s0 == 0 ? z1 : z2;
#pragma unroll
    for (int k = 0; k < 6; k++) yb[k] = sr_readlane64(((c0 + k) >> 6) == s0 ? lo : hi, (c0 + k) & 63);
  }
#pragma unroll
  for (int k = 5; k >= 0; k--) {
    double v = yb[k];
#pragma unroll
    for (int l = 5; l > k; l--) v -= Lc[l * (l - 1) / 2 + k] * xb[l];
    xb[k] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; k++) xv[c0 + k] = xb[k];
  }
#pragma unroll
  for (int l = 5; l >= 0; l--) {
    z0 -= Ac[0][l] * xb[l];
    z1 -= Ac[1][l] * xb[l];
    z2 -= Ac[2][l] * xb[l];
  }
}

template <bool kPingPong = true>  // false: the previous form (micro-benchmark reference, tools/experiments/solve_bench.hip)
__device__ __forceinline__ void sr_backsub(const double* P, const double* Ldg, double* xv, int K) {
  const int n = 6 * K, lane = threadIdx.x & 63;
  int pb[3];
  double zr[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int i = min(lane + 64 * j, n - 1), si = i / 6;
    pb[j] = sr_panel_off(si, n) + (i - 6 * si) * sr_panel_ld(si, n) - (6 * si + 6);
    zr[j] = P[pb[j] + n];
  }
  if constexpr (kPingPong) {
    double A0[3][6], A1[3][6], L0[16], L1[16];
    double z0 = zr[0], z1 = zr[1], z2 = zr[2];
    sr_bs_fetch(P, Ldg, pb, K - 1, A0, L0);
    int st = K - 1;
    for (; st >= 1; st -= 2) {
      sr_bs_step(P, Ldg, xv, pb, st, lane, z0, z1, z2, A0, L0, A1, L1);
      sr_bs_step(P, Ldg, xv, pb, st - 1, lane, z0, z1, z2, A1, L1, A0, L0);
    }
    if (st == 0) sr_bs_step(P, Ldg, xv, pb, 0, lane, z0, z1, z2, A0, L0, A1, L1);
  } else {
    double Ac[3][6];
    auto fetch = [&](int st, double (&Ad)[3][6]) {
#pragma unroll
      for (int j = 0; j < 3; j++) {
        if (lane + 64 * j < 6 * st) sr_ld6(P + pb[j] + 6 * st, Ad[j]);
        else
#pragma unroll
          for (int l = 0; l < 6; l++) Ad[j][l] = 0.0;  // rows >= 6 st: final, never updated
      }
    };
    fetch(K - 1, Ac);
    for (int st = K - 1; st >= 0; st--) {
      const int c0 = 6 * st;
      double Lc[16];
      {
        const double2* q = reinterpret_cast<const double2*>(Ldg + 16 * st);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const double2 t = q[i];
          Lc[2 * i] = t.x;
          Lc[2 * i + 1] = t.y;
        }
      }
      double An[3][6];
      if (st > 0) fetch(st - 1, An);
      double yb[6], xb[6];
      const int s0 = c0 >> 6, s5 = (c0 + 5) >> 6;
      if (s0 == s5) {
        const double src = s0 == 0 ? zr[0] : (s0 == 1 ? zr[1] : zr[2]);
#pragma unroll
        for (int k = 0; k < 6; k++) yb[k] = sr_readlane64(src, (c0 + k) & 63);
      } else {
#pragma unroll
        for (int k = 0; k < 6; k++) {
          const int sl = (c0 + k) >> 6;
          yb[k] = sr_readlane64(sl == 0 ? zr[0] : (sl == 1 ? zr[1] : zr[2]), (c0 + k) & 63);
        }
      }
#pragma unroll
      for (int k = 5; k >= 0; k--) {
        double v = yb[k];
#pragma unroll
        for (int l = 5; l > k; l--) v -= Lc[l * (l - 1) / 2 + k] * xb[l];
        xb[k] = v;
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) xv[c0 + k] = xb[k];
      }
#pragma unroll
      for (int j = 0; j < 3; j++)
#pragma unroll
        for (int l = 5; l >= 0; l--) zr[j] -= Ac[j][l] * xb[l];
      if (st > 0) {
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
          for (int l = 0; l < 6; l++) Ac[j][l] = An[j][l];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The stamp hook: at(slot) -- 0 start, 1 assembly done, 2 factor done, 3 back substitution done, 4 end -- and
// step(s, phase) on thread 0 (0: column out + barrier, 1: pivot + panel + barrier, 2: trailing update issued)
struct NoStamp {
  __device__ void at(int) const {}
  __device__ void step(int, int) const {}
  __device__ void wave(int, int) const {}  // (per-wave phase trace, benchmarks only)
};

// pairfin: [npairs][48] (pair (a <= b) row-major over the upper triangle; entries 0..35 the block S_ab (row r of
// pose a, column cc of pose b; on a diagonal pair only cc <= r is read), 36..41 bp, 42..47 sum Y bl of the pose).
// pidx / np: the pose part of the LM scale runs over the problem's poses p < np (lane p) with pidx[p] >= 0, as the
// other solvers.  Writes x[0 .. 6K) and *sc_out, or sets *fail.  Launch: 1 workgroup of kSolveRegThreads,
// solve_reg_lds_bytes(K) of dynamic LDS, 10 < K <= kSolveRegMaxK.
template <class Stamp, int kAblate = 0>  // kAblate (benchmarks only): 1 no trailing MFMAs, 2 no pivot arithmetic,
                                         // 4 no tile assembly, 8 no pairfin loads
__device__ void solve_reg(const double* __restrict__ pairfin, int K, double lambda, double* __restrict__ x,
                          double* __restrict__ sc_out, int* fail, const int* pidx, int np, double* lds,
                          const Stamp& stamp) {
  const SolveRegLayout Ly(K);
  const int n = Ly.n, npairs = Ly.npairs, NT = (n + 16) / 16, ntiles = NT * (NT + 1) / 2;
  double* P = lds;
  double* XD = lds + Ly.xd;
  double* Col = lds + Ly.col;
  double* Ldg = lds + Ly.ld;
  double* yv = lds + Ly.y;
  double* xv = lds + Ly.xs;
  double* bpl = lds + Ly.bp;
  double* ybl = lds + Ly.ybl;
  double* stg = lds;
  const int xld = (n + 2) & ~1;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lr = lane & 15, lq = lane >> 4;
  __shared__ int bad;
  if (tid == 0) bad = 0;
  stamp.at(0);
  // ---- assembly: pairfin coalesced (768 consecutive doubles per load instruction, all in flight) into the
  // staging rows (pair-major, stride 38); bp and sum Y bl of the diagonal pairs ----
  {
    constexpr int kB = 30;  // 30 x 768 >= 465 pairs x 48
    static_assert(kB * kSolveRegThreads >= kSolveRegMaxK * (kSolveRegMaxK + 1) / 2 * 48, "assembly batch");
    const int nent = npairs * 48;
    double va[kB];
#pragma unroll
    for (int u = 0; u < kB; u++)
      va[u] = (kAblate & 8) ? 1.0 + u : pairfin[min(tid + kSolveRegThreads * u, nent - 1)];
    double vb = 0.0;
    if (tid < 12 * K) {
      const int a = tid / 12;
      vb = pairfin[48 * (a * K - a * (a - 1) / 2) + 36 + (tid - 12 * a)];
    }
#pragma unroll
    for (int u = 0; u < kB; u++) {
      const int idx = tid + kSolveRegThreads * u, pr = idx / 48, e = idx - 48 * pr;
      if (idx < nent && e < 36) stg[38 * pr + e] = va[u];
    }
    if (tid < 12 * K) {
      const int a = tid / 12, e = tid - 12 * a;
      if (e < 6) bpl[6 * a + e] = vb;
      else ybl[6 * a + e - 6] = vb;
    }
  }
  if (*fail) return;  // uniform: a landmark block failed to invert (its flag is out with the sums)
  __syncthreads();
  // ---- a tile wave's tiles (list index tw, tw + 9, ...; tw = its rank among the tile waves), assembled from the
  // staging rows ----
  const bool tilew = (wv & 3) != 0;
  const int tw = wv - 1 - (wv >> 2);
  sr_d4 acc[kSrMaxTiles];
  int tI[kSrMaxTiles], tJ[kSrMaxTiles];
#pragma unroll
  for (int q = 0; q < kSrMaxTiles; q++) {
    const int t = tilew ? tw + kSrTileWaves * q : ntiles;
    tI[q] = -1;
    tJ[q] = -1;
    if (t < ntiles) sr_tile_of(t, NT, tI[q], tJ[q]);
    // element (r, c): pose blocks pr = r / 6 >= pc = c / 6; pair (pc, pr) = pbase + pr; off the diagonal pair its
    // entry (c % 6, r % 6), on it (r % 6, c % 6); row n is the rhs
    const int c = 16 * tJ[q] + lr, pc = c / 6, cc = c - 6 * pc, pbase = pc * K - pc * (pc - 1) / 2 - pc;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int r = 16 * tI[q] + 4 * i + lq, pr = r / 6, rr = r - 6 * pr;
      double v = 0.0;
      if (!(kAblate & 4) && t < ntiles && c < n && r <= n && r >= c) {
        if (r == n) {
          v = bpl[c] - ybl[c];
        } else {
          v = stg[38 * (pbase + pr) + (pr > pc ? 6 * cc + rr : 6 * rr + cc)];
          if (r == c) v += lambda;
        }
      }
      acc[q][i] = v;
    }
  }
  __syncthreads();  // the staging area becomes the panel store
  stamp.at(1);
  // Look-ahead: iteration s (after panel s is out) -- the tile waves update the tiles holding the next pivot
  // column (c1 = 6s + 6) with panel s and write that column out; barrier; the pivot waves factor it (pivot s + 1,
  // panel s + 1) while the tile waves apply panel s to the rest of their tiles; barrier.  XD is double-buffered by
  // step parity (panel s is read while panel s + 1 is written).
  // acc[q] += (-X_s D_s)[rows] X_s[cols]^T over rows / columns 6s+6 .. n: K = 6 as two 16x16x4 steps (k = lq and
  // 4 + lq; zero for k >= 6 and outside the trailing rows / columns)
  auto tile_update = [&](int q, int s) {
    const int r0 = 6 * s + 6;
    const double* Ps = P + sr_panel_off(s, n) - r0;
    const double* XDs = XD + (s & 1) * 6 * xld;
    const int pld = sr_panel_ld(s, n);
    const int ra = 16 * tI[q] + lr, cb = 16 * tJ[q] + lr;
    const bool va = ra >= r0 && ra <= n, vb = cb >= r0 && cb < n;
    const double a0 = va ? XDs[lq * xld + ra] : 0.0;
    const double b0 = vb ? Ps[lq * pld + cb] : 0.0;
    const double a1 = va && lq < 2 ? XDs[(4 + lq) * xld + ra] : 0.0;
    const double b1 = vb && lq < 2 ? Ps[(4 + lq) * pld + cb] : 0.0;
    if (kAblate & 1) return;
    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[q], 0, 0, 0);
    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[q], 0, 0, 0);
  };
  auto holds = [&](int q, int c0) { return tJ[q] >= 0 && 16 * tJ[q] + 15 >= c0 && 16 * tJ[q] <= c0 + 5; };
  auto extract = [&](int q, int c0) {  // columns c0 .. c0 + 5, rows c0 .. n of tile q
    const int c = 16 * tJ[q] + lr - c0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int r = 16 * tI[q] + 4 * i + lq;
      if (c >= 0 && c < 6 && r >= c0 && r <= n) Col[6 * r + c] = acc[q][i];
    }
  };
  if (tilew) {
    // ======== tile waves (SIMDs 1..3) ========
#pragma unroll
    for (int q = 0; q < kSrMaxTiles; q++)
      if (holds(q, 0)) extract(q, 0);
    __syncthreads();
    __syncthreads();  // panel 0
    for (int s = 0; s < K; s++) {
      const int c1 = 6 * s + 6;
      stamp.wave(s, 0);
#pragma unroll
      for (int q = 0; q < kSrMaxTiles; q++)
        if (c1 < n && holds(q, c1)) {  // (uniform) the tiles holding columns c1 .. c1 + 5, then that column out
          tile_update(q, s);
          extract(q, c1);
        }
      __syncthreads();
      stamp.wave(s, 1);
#pragma unroll
      for (int q = 0; q < kSrMaxTiles; q++)
        if (tJ[q] >= 0 && 16 * tJ[q] + 15 >= c1 && !(c1 < n && holds(q, c1))) tile_update(q, s);
      stamp.wave(s, 2);
      __syncthreads();
    }
  } else {
    // ======== SIMD 0: wave 0 factors pivot block s and forms the panel rows 6s + 6 .. n (three per lane) ========
    __syncthreads();  // column 0
    for (int s = 0; s <= K; s++) {
      const int c0 = 6 * s, r0 = c0 + 6;
      stamp.step(s, 0);
      stamp.wave(s, 0);
      if (s < K && wv == 0 && !(kAblate & 2)) {
        double a[6][6], L6[15], d6[6], r6[6];
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
          for (int k = 0; k <= i; k++) a[i][k] = Col[6 * (c0 + i) + k];
        double w[3][6];  // this lane's panel rows, requested with the pivot block
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const int row = r0 + lane + 64 * j;
          if (row <= n) sr_ld6(Col + 6 * row, w[j]);
        }
        // the pivot chain is per pivot: v_rcp_f64, one Newton step (rcp's error squared), and the next pivot
        // d' = a - u^2 r with u^2 formed off the chain (4 dependent ops instead of 7; the other entries as before)
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 6; j++) {
          const double d = a[j][j];
          ok = ok && d > 0;
          const double r0 = __builtin_amdgcn_rcp(d);
          const double r = fma(r0, fma(-d, r0, 1.0), r0);
          d6[j] = d;
          r6[j] = r;
          double u[6];
#pragma unroll
          for (int i = j + 1; i < 6; i++) u[i] = a[i][j];
          if (j < 5) a[j + 1][j + 1] = fma(-(u[j + 1] * u[j + 1]), r, a[j + 1][j + 1]);
#pragma unroll
          for (int i = j + 1; i < 6; i++) {
            const double l = u[i] * r;
            a[i][j] = l;
#pragma unroll
            for (int k = j + 1; k <= i; k++)
              if (!(i == j + 1 && k == j + 1)) a[i][k] -= l * u[k];
          }
        }
#pragma unroll
        for (int i = 0, q = 0; i < 6; i++)
#pragma unroll
          for (int k = 0; k < i; k++, q++) L6[q] = a[i][k];
        stamp.wave(s, 1);
        if (!ok) {
          if (lane == 0) {
            bad = 1;
            atomicOr(fail, 1);
          }
        } else {
          if (lane == 0) {  // (uniform values from one lane: no lane-indexed register selects)
#pragma unroll
            for (int q = 0; q < 15; q++) Ldg[16 * s + q] = L6[q];
          }
          double* Ps = P + sr_panel_off(s, n) - r0;
          double* XDs = XD + (s & 1) * 6 * xld;
          const int pld = sr_panel_ld(s, n);
#pragma unroll
          for (int j = 0; j < 3; j++) {
            const int row = r0 + lane + 64 * j;
            if (row <= n) {  // X = w L^-T D^-1 (unit L: no divides); -X D for the MFMA A operand
#pragma unroll
              for (int k = 0, q = 0; k < 6; k++) {
#pragma unroll
                for (int l = 0; l < k; l++, q++) w[j][k] -= w[j][l] * L6[q];
              }
#pragma unroll
              for (int k = 0; k < 6; k++) {
                const double xv_ = w[j][k] * r6[k];
                Ps[k * pld + row] = xv_;
                XDs[k * xld + row] = -(xv_ * d6[k]);
              }
            }
          }
        }
      }
      stamp.wave(s, 2);
      __syncthreads();  // panel s out
      if (s < K) __syncthreads();  // column s + 1 out (iteration s of the tile waves)
    }
  }
  if (bad) return;  // (a failed pivot: *fail is set; the later steps ran on garbage, same barrier count)
  if (wv != 0) return;
  stamp.at(2);
  sr_backsub(P, Ldg, xv, K);
#pragma unroll
  for (int j = 0; j < 3; j++)
    if (lane + 64 * j < n) x[lane + 64 * j] = xv[lane + 64 * j];
  stamp.at(3);
  // the pose part of the LM scale x.(lambda x + bp) (lane = problem pose)
  const int pose_a = lane < np ? pidx[lane] : -1;
  double sc = 0;
  if (pose_a >= 0)
#pragma unroll
    for (int k = 0; k < 6; k++) sc += xv[6 * pose_a + k] * (lambda * xv[6 * pose_a + k] + bpl[6 * pose_a + k]);
  sc = wave::xsum64(sc);
  if (lane == 0) *sc_out = sc;
  stamp.at(4);
}

}  // namespace ba
}  // namespace rspl
