// Reduced camera system of the local BA for 10 < K <= 30 optimised poses (C5's 30-keyframe window, n = 6K = 174):
// (S + lambda I) x = bp - sum Y bl from the pose-pair sums in ONE workgroup of 12 waves.  g2o solves the reduced
// system with a dense Cholesky-type factorisation (g2o_optimization.cc:26-36, BlockSolver + LinearSolverEigen); here
// a right-looking LDL^T blocked by the 6x6 pose blocks, every pivot a reciprocal (v_rcp_f64 + two Newton steps).
//
// The factor is a chain of K pose steps (pivot block -> panel -> trailing update); per step the chain is what
// matters, not the arithmetic (n^3 / 6 fp64 FMAs is ~5 us of one CU).  So the work is split by role, with look-ahead,
// and the roles synchronise through LDS counters instead of workgroup barriers:
//   * 8 bulk waves own the trailing matrix: thread t holds one 6x6 block of the lower triangle (or the rhs row's six
//     entries of a block column) in registers, column-major.  At step s a bulk wave applies panel s to its blocks of
//     columns >= s + 2 (T -= X_rows(br) D_s X_rows(bc)^T, l ascending per entry) and the owners of column s + 2 then
//     publish it -- "through panel s" -- into the raw-column buffer R[(s + 2) & 1].
//   * 4 pivot waves (at raised issue priority) carry the chain: at step c each lane takes one row of block column c
//     from R, applies panel c - 1 to it (the only update the bulk left out), lanes 0..5 of every pivot wave hold the
//     six pivot rows (redundantly, so no cross-wave hand-off precedes the pivot), the wave factors the 6x6 pivot block
//     (uniform), and each lane forms its panel row X = a L^-T D^-1 into the panel store.
// Per element the same operations in the same order as the barrier-synchronised kernel it replaces (panel by panel,
// l ascending; X D formed as (w r) d): bitwise the same factor.  Counters: panel[s] counts the pivot waves that wrote
// panel s, col[c] the bulk waves that published column c; every wait is a bounded poll with s_sleep, and an abort word
// (non-positive pivot, or a poll over its bound) releases every waiting wave.
//
// Panels are stored transposed (panel s: 6 x R_s doubles, entry (l, row) at l * R_s + row - 6s - 6, R_s = n - 6s - 4
// even), kept for the backward substitution: a bulk wave reads its rows' entries of one l as 16-byte loads, the
// substitution reads L(6 st + l, i) for l = 0..5 as three.  During the assembly the same LDS stages the pose-pair sums
// (pair-major, stride 38), read coalesced from global memory.  Backward substitution L^T x = y on the first pivot wave
// by pose step (y = D^-1 L^-1 z is panel s's rhs row), the next step's entries requested ahead.  A non-positive pivot
// or a failed landmark inversion upstream (*fail) leaves x untouched and sets *fail.
#pragma once
#include <hip/hip_runtime.h>

namespace rspl {
namespace ba {

constexpr int kSrBulkWaves = 8;
constexpr int kSrPivWaves = 4;
constexpr int kSolveRegThreads = 64 * (kSrBulkWaves + kSrPivWaves);  // 768
constexpr int kSolveRegMaxK = 30;  // K (K + 3) / 2 blocks (lower triangle + rhs row) <= 64 * kSrBulkWaves
static_assert(kSolveRegMaxK * (kSolveRegMaxK + 3) / 2 <= 64 * kSrBulkWaves, "one block per bulk thread");
static_assert(kSolveRegMaxK * 6 + 1 - 6 <= 58 * kSrPivWaves, "one row per pivot lane");

// panel s: R_s = n - 6s - 4 doubles per l (rows 6s + 6 .. n, padded to even); offset of panel s in the store
__host__ __device__ constexpr int sr_panel_ld(int s, int n) { return n - 6 * s - 4; }
__host__ __device__ constexpr int sr_panel_off(int s, int n) { return 6 * (s * (n - 4) - 3 * s * (s - 1)); }

struct SolveRegLayout {
  int n, K, npairs;
  int R, bp, ybl, rd, dd, ld, gd, flags, total;  // offsets in doubles (panels at 0)
  __host__ __device__ explicit SolveRegLayout(int K_) : n(6 * K_), K(K_), npairs(K_ * (K_ + 1) / 2) {
    R = sr_panel_off(K, n);            // [2][n + 1][6] raw block columns (behind the panels)
    int end = R + 2 * 6 * (n + 1);
    const int stage = 38 * npairs;     // assembly staging (aliases panels and R)
    end = end > stage ? end : stage;
    bp = end;                          // [n] pose gradient bp (LM scale); x at the end
    ybl = bp + n;                      // [n] sum Y bl (assembly)
    rd = ybl + n;                      // [n] 1/D
    dd = rd + n;                       // [n] D
    ld = dd + n;                       // [K][16] each pivot block's strictly-lower unit L (15 used)
    gd = ld + 16 * K;                  // [kSrPivWaves][36] the pivot rows of each pivot wave
    flags = gd + 36 * kSrPivWaves;     // int [2K + 2]: panel[K], col[K], abort
    total = flags + (2 * K + 2 + 1) / 2;
  }
};
inline size_t solve_reg_lds_bytes(int K) { return sizeof(double) * (size_t)SolveRegLayout(K).total; }

__device__ __forceinline__ double sr_rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

__device__ __forceinline__ double sr_readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
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
__device__ __forceinline__ void sr_st6(double* p, const double (&v)[6]) {
  double2* q = reinterpret_cast<double2*>(p);
#pragma unroll
  for (int i = 0; i < 3; i++) q[i] = make_double2(v[2 * i], v[2 * i + 1]);
}

// bounded wait for *ctr >= target (LDS, workgroup scope, acquire); false on abort (set by a failed pivot or by a
// wait over its bound, which also flags *fail = 1 so the caller sees a failed solve, never a hang)
__device__ __forceinline__ bool sr_wait(int* ctr, int target, int* abort_w, int* fail) {
  for (int it = 0; it < (1 << 22); it++) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  if ((threadIdx.x & 63) == 0) {
    __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    atomicOr(fail, 1);
  }
  return false;
}
// this wave's LDS stores before it, then one increment of *ctr (release)
__device__ __forceinline__ void sr_signal(int* ctr) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDL^T of the 6x6 pivot block (lower triangle of rows a[i][k <= i]): unit L (strictly lower, packed row-major into
// L6), D, 1/D; false unless every pivot is > 0
__device__ __forceinline__ bool sr_ldl6(double (&a)[6][6], double (&L6)[15], double (&d6)[6], double (&r6)[6]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const double d = a[j][j];
    ok = ok && d > 0;
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
  return ok;
}

// The stamp hook: at(slot) -- 0 start, 1 assembly done, 2 factor done, 3 back substitution done, 4 end -- and
// step(c, phase) of the first pivot wave (0: inputs of step c in, 1: pivot block factored, 2: panel c out)
struct NoStamp {
  __device__ void at(int) const {}
  __device__ void step(int, int) const {}
};

// pairfin: [npairs][48] (pair (a <= b) row-major over the upper triangle; entries 0..35 the block S_ab (row r of
// pose a, column cc of pose b; on a diagonal pair only cc <= r is read), 36..41 bp, 42..47 sum Y bl of the pose).
// pidx / np: the pose part of the LM scale runs over the problem's poses p < np (lane p) with pidx[p] >= 0, as the
// other solvers.  Writes x[0 .. 6K) and *sc_out, or sets *fail.  Launch: 1 workgroup of kSolveRegThreads,
// solve_reg_lds_bytes(K) of dynamic LDS, 10 < K <= kSolveRegMaxK.
template <class Stamp>
__device__ void solve_reg(const double* __restrict__ pairfin, int K, double lambda, double* __restrict__ x,
                          double* __restrict__ sc_out, int* fail, const int* pidx, int np, double* lds,
                          const Stamp& stamp) {
  const SolveRegLayout Ly(K);
  const int n = Ly.n, npairs = Ly.npairs;
  double* P = lds;
  double* R = lds + Ly.R;
  double* bpl = lds + Ly.bp;
  double* ybl = lds + Ly.ybl;
  double* rdg = lds + Ly.rd;
  double* ddg = lds + Ly.dd;
  double* Ldg = lds + Ly.ld;
  int* panel_ctr = reinterpret_cast<int*>(lds + Ly.flags);
  int* col_ctr = panel_ctr + K;
  int* abort_w = col_ctr + K;
  double* stg = lds;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  stamp.at(0);
  if (tid < 2 * K + 1) panel_ctr[tid] = 0;
  // ---- assembly: pairfin coalesced into the staging rows; bp and sum Y bl of the diagonal pairs ----
  {
    constexpr int kB = 15;
    const int nent = npairs * 48;
    for (int b0 = 0; b0 < nent; b0 += kB * kSolveRegThreads) {
      double va[kB];
#pragma unroll
      for (int u = 0; u < kB; u++) va[u] = pairfin[min(b0 + tid + kSolveRegThreads * u, nent - 1)];
#pragma unroll
      for (int u = 0; u < kB; u++) {
        const int idx = b0 + tid + kSolveRegThreads * u, pr = idx / 48, e = idx - 48 * pr;
        if (idx < nent && e < 36) stg[38 * pr + e] = va[u];
      }
    }
    if (tid < 12 * K) {
      const int a = tid / 12, e = tid - 12 * a;
      const double v = pairfin[48 * (a * K - a * (a - 1) / 2) + 36 + e];
      if (e < 6) bpl[6 * a + e] = v;
      else ybl[6 * a + e - 6] = v;
    }
  }
  if (*fail) return;  // uniform: a landmark block failed to invert (its flag is out with the sums)
  __syncthreads();
  // ---- bulk threads: one block each (column bc, row br; br == K: the rhs row), column-major ----
  const bool bulk = wv < kSrBulkWaves;
  int br = -1, bc = -1;
  if (bulk) {
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
  const bool own = bc >= 0, rhs = own && br == K;
  double T[6][6];
  {
    // off-diagonal pair (bc, br): T[a][b] = S(6 br + a, 6 bc + b) = entry (b, a) of the pair's block; diagonal:
    // T[a][b] = entry (a, b), b <= a, + lambda on the diagonal
    const int pr = own ? bc * K - bc * (bc - 1) / 2 + (rhs ? 0 : br - bc) : 0;
    const double* q = stg + 38 * pr;
    const bool off = br > bc;
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int b = 0; b < 6; b++) {
        const double t = q[off ? 6 * b + a : 6 * a + b];
        T[a][b] = own && !rhs && (off || b <= a) ? t + (!off && a == b ? lambda : 0.0) : 0.0;
      }
    if (rhs)
#pragma unroll
      for (int b = 0; b < 6; b++) T[0][b] = bpl[6 * bc + b] - ybl[6 * bc + b];
  }
  __syncthreads();  // the staging area becomes the panel store and R
  // block columns 0 and 1 as assembled (column c's rows 6 br + a at R[c & 1][row]; the rhs row at row n)
  auto publish = [&]() {
    double* Rc = R + (bc & 1) * 6 * (n + 1);
    if (rhs) {
      sr_st6(Rc + 6 * n, T[0]);
    } else {
#pragma unroll
      for (int a = 0; a < 6; a++) sr_st6(Rc + 6 * (6 * br + a), T[a]);
    }
  };
  if (own && bc < 2) publish();
  __syncthreads();
  stamp.at(1);
  if (bulk) {
    // ======== bulk waves ========
    int cmax = own ? bc : -1;  // the wave's last block column
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) cmax = max(cmax, __shfl_xor(cmax, o));
    for (int s = 0; s + 2 <= cmax; s++) {
      if (!sr_wait(panel_ctr + s, kSrPivWaves, abort_w, fail)) return;
      if (own && bc >= s + 2) {
        const double* Ps = P + sr_panel_off(s, n) - (6 * s + 6);  // entry (l, row): Ps[l * ld + row]
        const int pld = sr_panel_ld(s, n);
        const double* pk = Ps + 6 * bc;
        const double* pi = rhs ? Ps + n : Ps + 6 * br;
        // one l at a time, the next l's operands requested before this l's FMAs (register budget: 3 waves / SIMD)
        double xk[6], wi[6], xn[6], wn[6];
        sr_ld6(pk, xk);
        if (!rhs) sr_ld6(pi, wi);
        else wi[0] = pi[0];
#pragma unroll 1
        for (int l = 0; l < 6; l++) {
          const double dl = ddg[6 * s + l];
          if (l < 5) {
            sr_ld6(pk + (l + 1) * pld, xn);
            if (!rhs) sr_ld6(pi + (l + 1) * pld, wn);
            else wn[0] = pi[(l + 1) * pld];
          }
          if (!rhs) {
#pragma unroll
            for (int a = 0; a < 6; a++) {
              const double w = wi[a] * dl;
#pragma unroll
              for (int b = 0; b < 6; b++) T[a][b] -= w * xk[b];
            }
          } else {
            const double w = wi[0] * dl;
#pragma unroll
            for (int b = 0; b < 6; b++) T[0][b] -= w * xk[b];
          }
#pragma unroll
          for (int b = 0; b < 6; b++) {
            xk[b] = xn[b];
            wi[b] = wn[b];
          }
        }
      }
      if (s + 2 < K) {
        const bool mine = own && bc == s + 2;
        if (mine) publish();
        if (__ballot(mine)) sr_signal(col_ctr + s + 2);
      }
    }
    return;
  }
  // ======== pivot waves ========
  __builtin_amdgcn_s_setprio(2);
  const int g = wv - kSrBulkWaves;
  double* gdiag = lds + Ly.gd + 36 * g;
  double dprev[6];  // D of the previous pose step
  double L6[15], d6[6], r6[6];
  int base_c = 0;   // first bulk thread of column c
  for (int c = 0; c < K; c++) {
    const int c0 = 6 * c;
    // this lane's row of block column c: lanes 0..5 the pivot rows, lanes 6..63 rows below (and the rhs row n)
    const int row = lane < 6 ? c0 + lane : c0 + 6 + 58 * g + (lane - 6);
    const bool live = row <= n;
    if (c >= 2) {  // column c through panel c - 2, from the bulk waves that own it
      const int t1 = base_c + K - c;
      if (!sr_wait(col_ctr + c, (t1 >> 6) - (base_c >> 6) + 1, abort_w, fail)) return;
    }
    if (c >= 1 && !sr_wait(panel_ctr + c - 1, kSrPivWaves, abort_w, fail)) return;
    stamp.step(c, 0);
    double w[6];
    if (live) sr_ld6(R + (c & 1) * 6 * (n + 1) + 6 * row, w);
    else
#pragma unroll
      for (int b = 0; b < 6; b++) w[b] = 0.0;
    if (c >= 1 && live) {  // panel c - 1 (rows c0 - 0 .. n of it): w_b -= (X_row,l d_l) X_{c0 + b, l}
      const double* Ps = P + sr_panel_off(c - 1, n) - c0;
      const int pld = sr_panel_ld(c - 1, n);
#pragma unroll
      for (int l = 0; l < 6; l++) {
        double xk[6];
        sr_ld6(Ps + l * pld + c0, xk);
        const double wr = Ps[l * pld + row] * dprev[l];
#pragma unroll
        for (int b = 0; b < 6; b++) w[b] -= wr * xk[b];
      }
    }
    // the pivot block (lanes 0..5 of this wave) through LDS, factored by every lane
    if (lane < 6) sr_st6(gdiag + 6 * lane, w);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
      double a[6][6];
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int k = 0; k <= i; k++) a[i][k] = gdiag[6 * i + k];
      if (!sr_ldl6(a, L6, d6, r6)) {  // uniform: every pivot wave factors the same block
        if (lane == 0) {
          __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          atomicOr(fail, 1);
        }
        return;
      }
    }
    stamp.step(c, 1);
    if (g == 0 && lane < 16) {  // (the bulk waves read D after the panel counter; the substitution L and 1/D)
      if (lane < 15) Ldg[16 * c + lane] = L6[lane];
      if (lane < 6) {
        rdg[c0 + lane] = r6[lane];
        ddg[c0 + lane] = d6[lane];
      }
    }
    if (lane >= 6 && live) {  // panel row: X = w L^-T D^-1 (unit L: no divides)
#pragma unroll
      for (int k = 0, q = 0; k < 6; k++) {
#pragma unroll
        for (int l = 0; l < k; l++, q++) w[k] -= w[l] * L6[q];
      }
      double* Pc = P + sr_panel_off(c, n) - (c0 + 6);
      const int pld = sr_panel_ld(c, n);
#pragma unroll
      for (int k = 0; k < 6; k++) Pc[k * pld + row] = w[k] * r6[k];
    }
    sr_signal(panel_ctr + c);
    stamp.step(c, 2);
#pragma unroll
    for (int l = 0; l < 6; l++) dprev[l] = d6[l];
    base_c += K - c + 1;
  }
  if (g != 0) return;
  if (!sr_wait(panel_ctr + K - 1, kSrPivWaves, abort_w, fail)) return;
  stamp.at(2);
  // ---- backward substitution L^T x = y on this wave; row i: lane i % 64, slot i / 64 ----
  // L(6 st + l, i) for i < 6 st: panel s(i), entry (i - 6 s(i), 6 st + l); y_i: panel s(i)'s rhs row
  const double* Pi[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int i = min(lane + 64 * j, n - 1), si = i / 6;
    Pi[j] = P + sr_panel_off(si, n) + (i - 6 * si) * sr_panel_ld(si, n) - (6 * si + 6);
  }
  double zr[3];
#pragma unroll
  for (int j = 0; j < 3; j++) zr[j] = Pi[j][n];
  double Ac[3][6], Lc[15];
  auto fetch = [&](int st, double (&Ad)[3][6], double (&Ld)[15]) {
    const int c0 = 6 * st;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      if (lane + 64 * j < c0) sr_ld6(Pi[j] + c0, Ad[j]);  // (rows >= c0: never used)
      else
#pragma unroll
        for (int l = 0; l < 6; l++) Ad[j][l] = 0.0;
    }
#pragma unroll
    for (int q = 0; q < 15; q++) Ld[q] = Ldg[16 * st + q];
  };
  fetch(K - 1, Ac, Lc);
  for (int st = K - 1; st >= 0; st--) {
    const int c0 = 6 * st;
    double xb[6];
#pragma unroll
    for (int k = 5; k >= 0; k--) {
      const int i = c0 + k, sl = i >> 6;
      double v = sr_readlane64(sl == 0 ? zr[0] : sl == 1 ? zr[1] : zr[2], i & 63);
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
    if (st > 0) fetch(st - 1, Ac, Lc);
  }
  double* xs = ybl;  // x in LDS for the scale
#pragma unroll
  for (int j = 0; j < 3; j++)
    if (lane + 64 * j < n) {
      x[lane + 64 * j] = zr[j];
      xs[lane + 64 * j] = zr[j];
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  stamp.at(3);
  // the pose part of the LM scale x.(lambda x + bp) (lane = problem pose)
  const int pose_a = lane < np ? pidx[lane] : -1;
  double sc = 0;
  if (pose_a >= 0)
#pragma unroll
    for (int k = 0; k < 6; k++) sc += xs[6 * pose_a + k] * (lambda * xs[6 * pose_a + k] + bpl[6 * pose_a + k]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sc += __shfl_xor(sc, o);
  if (lane == 0) *sc_out = sc;
  stamp.at(4);
}

}  // namespace ba
}  // namespace rspl
