// Tracking pose optimisation, FrameOptimization (src/g2o_optimization/g2o_optimization.cc:256-398),
// as a single-launch fp64 Levenberg-Marquardt on gfx950: ONE workgroup (4 wavefronts; 1 with
// RSPL_FRAME_WAVES=1) owns one frame for the whole call -- 4 rounds x optimize(10) x trials -- so
// there is no host round trip and no grid synchronisation.  Each thread linearises a strided subset
// of the frame's unary edges; the 6x6 normal equations (21 + 6 + chi2 values) are all-reduced across
// each wave with DPP (quad swaps, half-row / row mirrors, then the four row results through
// readlane: a fixed tree, and because IEEE addition is commutative every lane ends with the
// bitwise-same sums), then the waves' sums are added in wave order through LDS.  Every thread then
// factors the same 6x6 system in registers, so the LM control (g2o
// OptimizationAlgorithmLevenberg: tau 1e-5, good-step scale clamp [1/3, 2/3], ni doubling,
// 10 trials, stop on qmax == 10 || rho == 0) is uniform and needs no broadcast.
// Latency bound by construction (a few hundred edges per frame): throughput comes from batching
// frames -- one workgroup each -- into one launch.  Same algorithm as the CPU restatement
// orc_frame_opt (oracle/ba.c).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <cstdlib>

#include "frame_kernels.hpp"
#include "se3_device.hpp"
#include "wave_reduce.hpp"

namespace rspl {
namespace frame {

using ba::SE3;
using wave::kNV;
using wave::rcp64;
using wave::wsum;
using wave::wsum_int;

__device__ __forceinline__ void huber(double e2, double delta, double& r0, double& r1) {
  const double dsqr = delta * delta;
  if (e2 <= dsqr) {
    r0 = e2;
    r1 = 1.0;
  } else {
    const double s = sqrt(e2);
    r0 = 2 * s * delta - dsqr;
    r1 = delta / s;
  }
}

struct Pose {  // T_cw with its rotation matrix
  SE3 T;
  double R[9];
  __device__ void set(const SE3& t) {
    T = t;
    ba::q_to_R(T.q, R);
  }
};

// e = obs - proj(T Xw) (+ the right-image u for stereo); returns Xc for the Jacobian
__device__ __forceinline__ void edge_error(const Edge& E, const Pose& P, double* Xc, double* e) {
  ba::mat3_vec(P.R, E.X, Xc);
  for (int i = 0; i < 3; i++) Xc[i] += P.T.t[i];
  const double iz = 1.0 / Xc[2];
  const double u = E.cam[0] * Xc[0] * iz + E.cam[2], v = E.cam[1] * Xc[1] * iz + E.cam[3];
  e[0] = E.obs[0] - u;
  e[1] = E.obs[1] - v;
  e[2] = E.stereo != 0.0 ? E.obs[2] - (u - E.cam[4] * iz) : 0.0;
}

__device__ __forceinline__ double chi2_of(const double* e) { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }

// One frame's per-edge state: the edge records, the last computed error, the level and the
// inlier flag -- staged in LDS for frames of <= kLdsEdges edges (one copy in, then every LM
// pass reads LDS instead of chasing L2 latency), in global scratch otherwise.
struct View {
  const Edge* E;
  double* err;   // [n][3]
  uint8_t* lev;
  uint8_t* inl;
  int n;
  double delta0, delta1;  // Huber deltas (mono, stereo): scalars, never indexed (no scratch)
};


#ifdef RSPL_FRAME_PROF  // experiment build only (tools/experiments): per-phase cycle sums of block 0, printed at exit
struct FProf {
  unsigned long long t[8];
  int n;
};
#define FP_DECL , FProf& pf
#define FP_ARG , pf
#define FP_NOW(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define FP_ADD(k, a, b) pf.t[k] += (b) - (a)
#else
#define FP_DECL
#define FP_ARG
#define FP_NOW(v)
#define FP_ADD(k, a, b)
#endif
using wave::block_sum_int;

// robust (Huber) or plain chi2 of an error, for the edge type
__device__ __forceinline__ double cost_of(const View& V, const double* ev, bool stereo, bool robust) {
  const double c2 = chi2_of(ev);
  if (!robust) return c2;
  double r0, r1;
  huber(c2, stereo ? V.delta1 : V.delta0, r0, r1);
  return r0;
}

__device__ __forceinline__ int hidx(int i, int j) { return i * 6 - i * (i - 1) / 2 + (j - i); }

// errors at T (stored) + robust chi2 + H / b (Huber IRLS weights), wave-reduced
template <int NW>
__device__ __forceinline__ void linearize(const View& V, const Pose& P, int lane, bool robust,
                                          double (&acc)[kNV] FP_DECL) {
  FP_NOW(l0);
#pragma unroll
  for (int k = 0; k < kNV; k++) acc[k] = 0.0;
  for (int e = lane; e < V.n; e += 64 * NW) {
    if (V.lev[e]) continue;
    const Edge E = V.E[e];
    double Xc[3], ev[3];
    edge_error(E, P, Xc, ev);
    double* er = V.err + 3 * e;
    er[0] = ev[0]; er[1] = ev[1]; er[2] = ev[2];
    const double c2 = chi2_of(ev);
    double w = 1.0;
    if (robust) {
      double r0, r1;
      huber(c2, E.stereo != 0.0 ? V.delta1 : V.delta0, r0, r1);
      acc[27] += r0;
      w = r1;
    } else {
      acc[27] += c2;
    }
    const double fx = E.cam[0], fy = E.cam[1], bf = E.cam[4];
    const double x = Xc[0], y = Xc[1], z = Xc[2], iz = 1.0 / z, iz2 = iz * iz;
    const double Dm[3][3] = {{fx * iz, 0, -fx * x * iz2}, {0, fy * iz, -fy * y * iz2},
                             {fx * iz, 0, -fx * x * iz2 + bf * iz2}};
    const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    double J[3][6];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) s += Dm[r][k] * SX[k * 3 + c];
        J[r][c] = s;
        J[r][3 + c] = -Dm[r][c];
      }
    const int rows = E.stereo != 0.0 ? 3 : 2;
    if (rows == 2)
#pragma unroll
      for (int c = 0; c < 6; c++) J[2][c] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const double g = J[0][i] * ev[0] + J[1][i] * ev[1] + J[2][i] * ev[2];
      acc[21 + i] += -w * g;
#pragma unroll
      for (int j = i; j < 6; j++) acc[hidx(i, j)] += w * (J[0][i] * J[0][j] + J[1][i] * J[1][j] + J[2][i] * J[2][j]);
    }
  }
  FP_NOW(l1);
  wave::block_allreduce28<NW>(acc, lane & 63);
  FP_NOW(l2);
  FP_NOW(l3);
  FP_ADD(2, l0, l1);
  FP_ADD(3, l1, l2);
  FP_ADD(4, l2, l3);
}

// (H + lambda I) x = b by Cholesky, in registers (every lane the same); false if not SPD.
// The factor keeps 1 / L[j][j] on its diagonal.
__device__ __forceinline__ bool solve6(const double (&acc)[kNV], double lambda, double (&x)[6]) {
  double L[6][6];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 6; j++) L[i][j] = j >= i ? acc[hidx(i, j)] : acc[hidx(j, i)];
#pragma unroll
  for (int i = 0; i < 6; i++) L[i][i] += lambda;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    double s = L[j][j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
    ok = ok && s > 0;
    const double r = rcp64(sqrt(s));  // 1 / pivot: multiplications instead of a divide chain
    L[j][j] = r;
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      double t = L[i][j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
      L[i][j] = t * r;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double s = acc[21 + i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i][k] * x[k];
    x[i] = s * L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; i--) {
    double s = x[i];
#pragma unroll
    for (int k = i + 1; k < 6; k++) s -= L[k][i] * x[k];
    x[i] = s * L[i][i];
  }
  return ok;
}

// SparseOptimizer::optimize(iters) with OptimizationAlgorithmLevenberg on the pose vertex
template <int NW>
__device__ __forceinline__ int optimize_pose(const View& V, Pose& P, int lane, bool robust, int iters,
                                             double& chi2_out FP_DECL) {
  // The linearisation at the current estimate that every iteration starts with is the one the accepted
  // candidate of the previous iteration already computed: each trial evaluates its candidate's errors, robust
  // cost AND normal equations in one pass over the edges (one 28-value reduction), and an accepted candidate's
  // system becomes the next iteration's -- the same operations on the same estimate as linearising it again
  // (g2o computes the candidate's errors, then re-linearises the accepted estimate), one edge pass and one
  // reduction fewer per iteration.
  double acc[kNV];
  double lambda = 0, ni = 2, currentChi = 0;
  int done = 0;
  if (iters > 0) linearize<NW>(V, P, lane, robust, acc FP_ARG);
  for (int it = 0; it < iters; it++) {
    currentChi = acc[27];
    if (it == 0) {  // computeLambdaInit: tau * max diagonal
      double mx = 0;
#pragma unroll
      for (int i = 0; i < 6; i++) mx = fmax(mx, fabs(acc[hidx(i, i)]));
      lambda = 1e-5 * mx;
      ni = 2;
    }
    double rho = 0;
    int qmax = 0;
    do {
      double x[6];
      FP_NOW(q0);
      const bool ok = solve6(acc, lambda, x);  // (uniform: every thread factors the same system)
      FP_NOW(q1);
      Pose C = P;
      double cacc[kNV];
      double tempChi = DBL_MAX;
      if (ok) {
        C.set(ba::se3_mul(ba::se3_exp(x), P.T));
        FP_NOW(q2);
        FP_ADD(1, q1, q2);
        linearize<NW>(V, C, lane, robust, cacc FP_ARG);  // the candidate's errors (stored), cost and system
        tempChi = cacc[27];
      } else {
        linearize<NW>(V, P, lane, robust, cacc FP_ARG);  // (as g2o: the errors recomputed at the unchanged estimate)
      }
      rho = currentChi - tempChi;
      double scale = 1.0;
      if (ok) {
        scale = 0;
#pragma unroll
        for (int i = 0; i < 6; i++) scale += x[i] * (lambda * x[i] + acc[21 + i]);
        scale += 1e-3;
      }
      rho /= scale;
      if (rho > 0 && isfinite(tempChi) && ok) {
        double alpha = 1. - ba::cube(2 * rho - 1);  // pow(2 rho - 1, 3)
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
        P = C;
#pragma unroll
        for (int k = 0; k < kNV; k++) acc[k] = cacc[k];
      } else {
        lambda *= ni;
        ni *= 2;
        if (!isfinite(lambda)) break;
      }
      qmax++;
      FP_NOW(q3);
      FP_ADD(0, q0, q1);
      FP_ADD(5, q0, q3);
#ifdef RSPL_FRAME_PROF
      pf.n++;
#endif
    } while (rho < 0 && qmax < 10);
    done++;
    if (qmax == 10 || rho == 0 || !isfinite(lambda)) break;
  }
  chi2_out = currentChi;
  return done;
}

// NW wavefronts per frame (1 or 4; the control is uniform over the workgroup: every thread holds the
// same sums); LDS: the frame's edges + errors + flags staged once (kLdsEdges cap)
template <bool LDS, int NW>
__global__ __launch_bounds__(64 * NW) void frame_opt_kernel(Args a, int batch) {
  extern __shared__ double smem[];
  constexpr int T = 64 * NW;
  const int f = blockIdx.x;
  const int lane = threadIdx.x;  // the thread's index in the frame's workgroup
  const Desc D = a.frames[f];
  View V;
  V.n = D.n;
  V.delta0 = D.delta[0];
  V.delta1 = D.delta[1];
  const double th0 = D.th[0], th1 = D.th[1];
  if constexpr (LDS) {
    Edge* Es = reinterpret_cast<Edge*>(smem);
    // 16-byte pieces, eight loads in flight per thread before their LDS stores: the source is the
    // host-mapped staging (PCIe round trips of ~1-2 us) for a single frame, device memory otherwise
    static_assert(sizeof(Edge) % 16 == 0, "edge records in 16-byte pieces");
    const uint4* src = reinterpret_cast<const uint4*>(a.edges + D.e0);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = D.n * (int)(sizeof(Edge) / 16);
    int k0 = lane;
    for (; k0 + 7 * T < n16; k0 += 8 * T) {  // whole batches: unconditional, register-resident
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = src[k0 + j * T];
#pragma unroll
      for (int j = 0; j < 8; j++) dst[k0 + j * T] = v[j];
    }
    for (; k0 < n16; k0 += T) dst[k0] = src[k0];  // the tail
    V.E = Es;
    V.err = smem + D.n * (sizeof(Edge) / 8);
    V.lev = reinterpret_cast<uint8_t*>(V.err + 3 * D.n);
    V.inl = V.lev + D.n;
  } else {
    V.E = a.edges + D.e0;
    V.err = a.err + 4 * (size_t)D.e0;
    V.lev = a.level + D.e0;
    V.inl = a.inl + D.e0;
  }
  for (int e = lane; e < D.n; e += T) {
    V.inl[e] = a.inl_in[D.e0 + e];
    V.lev[e] = 0;
  }
  __syncthreads();  // orders the LDS staging
  SE3 T0;
  for (int k = 0; k < 4; k++) T0.q[k] = D.T0[k];
  for (int k = 0; k < 3; k++) T0.t[k] = D.T0[4 + k];
  Pose P;
  P.set(T0);
  // per-round results in scalars (a loop-indexed array would live in scratch)
  double c2r[4] = {0, 0, 0, 0};
  int itr[4] = {0, 0, 0, 0};
  int rounds = 0;
  int num_outlier = 0;
#ifdef RSPL_FRAME_PROF
  FProf pf{};
  FP_NOW(k0);
#endif
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
    P.set(T0);  // setEstimate(SE3Quat(pose).inverse()) every round (:337)
    const bool robust = r < 3;  // setRobustKernel(0) after round 2's classification (:363)
    int act = 0;
    for (int e = lane; e < D.n; e += T) act += V.lev[e] == 0;
    act = block_sum_int<NW>(act);
    int its = 0;
    double chi = 0;
    if (act) its = optimize_pose<NW>(V, P, lane, robust, 10, chi FP_ARG);
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (k == r) {
        itr[k] = its;
        c2r[k] = chi;
      }
    int no = 0;
    __syncthreads();  // every thread's last errors are stored before any thread classifies
    for (int e = lane; e < D.n; e += T) {
      double* er = V.err + 3 * e;
      const Edge E = V.E[e];
      double ev[3];
      if (!V.inl[e]) {  // computeError() at the current estimate (:345-347)
        double Xc[3];
        edge_error(E, P, Xc, ev);
      } else {          // the last error the optimizer computed
        ev[0] = er[0]; ev[1] = er[1]; ev[2] = er[2];
      }
      const float c2 = (float)chi2_of(ev);  // const float chi2 = e->chi2() (:349)
      if (c2 > (E.stereo != 0.0 ? th1 : th0)) {
        V.inl[e] = 0;
        V.lev[e] = 1;
        no++;
      } else {
        V.inl[e] = 1;
        V.lev[e] = 0;
      }
    }
    num_outlier = block_sum_int<NW>(no);  // (its barriers also order the level writes before the next round)
    rounds = r + 1;
    if (D.n < 10) break;  // optimizer.edges().size() < 10 (:383)
  }
#ifdef RSPL_FRAME_PROF
  FP_NOW(k1);
  if (f == 0 && lane == 0 && pf.n)
    printf("fprof NW %d n %d trials %d: total %llu | per trial: solve6 %llu se3 %llu edges %llu wred %llu bcomb %llu "
           "trial %llu\n", NW, D.n, pf.n, k1 - k0, pf.t[0] / pf.n, pf.t[1] / pf.n, pf.t[2] / pf.n, pf.t[3] / pf.n,
           pf.t[4] / pf.n, pf.t[5] / pf.n);
#endif
  for (int e = lane; e < D.n; e += T) a.inl_out[D.e0 + e] = V.inl[e];
  if (lane == 0) {
    Out* o = a.out + f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o->T[k] = P.T.q[k];
      o->chi2[k] = c2r[k];
      o->iters[k] = itr[k];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) o->T[4 + k] = P.T.t[k];
    o->T[7] = 0;
    o->n_inliers = D.n - num_outlier;
    o->rounds = rounds;
  }
}

size_t lds_bytes(int n) { return (size_t)n * (sizeof(Edge) + 3 * sizeof(double) + 2); }

// waves per frame: 4 for latency (one frame per CU at 256 VGPRs) while the batch leaves CUs idle,
// 1 for throughput (two frames per SIMD) on large batches (profiles/r03_bench_frame.json).
// The wave count sets the summation order of H / b / chi2, so a frame's result depends on whether its
// batch exceeds 256 frames at the last-ulp level (agreement to the oracle tolerances either way:
// tests/test_gpu_frame.py::test_frame_alone_and_in_a_large_batch).
hipError_t optimize(const Args& a, int batch, int max_n, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  const bool one = batch > 256;
  if (max_n <= kLdsEdges) {
    if (one) frame_opt_kernel<true, 1><<<batch, 64, lds_bytes(max_n), s>>>(a, batch);
    else frame_opt_kernel<true, 4><<<batch, 256, lds_bytes(max_n), s>>>(a, batch);
  } else {
    if (one) frame_opt_kernel<false, 1><<<batch, 64, 0, s>>>(a, batch);
    else frame_opt_kernel<false, 4><<<batch, 256, 0, s>>>(a, batch);
  }
  return hipGetLastError();
}

}  // namespace frame
}  // namespace rspl
