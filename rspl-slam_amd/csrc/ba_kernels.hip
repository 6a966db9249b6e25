// Local bundle adjustment (LocalmapOptimization, src/g2o_optimization/g2o_optimization.cc:21-252)
// as an fp64 Levenberg-Marquardt on gfx950.  Same algorithm as the CPU restatement
// (oracle/ba.c, which restates the g2o pieces it relies on): SE3 left exp-map update,
// analytic point Jacobians, numeric (delta 1e-9) line Jacobians, Huber IRLS weights,
// Schur complement on marginalised points + lines, dense Cholesky of the reduced
// camera system.  Every reduction runs in a fixed order (CSR lists, fixed trees), so
// a call is bitwise reproducible.  Not a dense contraction: no MFMA; HBM/latency bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "ba_kernels.hpp"
#include "ba_solve_reg.hpp"
#include "se3_device.hpp"
#include "wave_reduce.hpp"


namespace rspl {
namespace ba {


__device__ __forceinline__ double n3(const double* v) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
}
__device__ __forceinline__ void cross3(const double* a, const double* b, double* o) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// g2o::Line3D::oplus (orthonormal 4-DoF update; vertex_line3d.h:26-29)
__device__ __forceinline__ void line_oplus(double* L, const double* v) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  const double* w = L;
  const double* d = L + 3;
  const double mx = n3(d), my = n3(w);
  const double wn = 1.0 / sqrt(mx * mx + my * my);
  const double Wm[4] = {my * wn, -mx * wn, mx * wn, my * wn};
  const double mn = 1.0 / my, dn = 1.0 / mx;
  double mdc[3];
  cross3(w, d, mdc);
  const double mdn = 1.0 / n3(mdc);
  const double U[9] = {w[0] * mn, d[0] * dn, mdc[0] * mdn, w[1] * mn, d[1] * dn, mdc[1] * mdn,
                       w[2] * mn, d[2] * dn, mdc[2] * mdn};
  const double cs = cos(v[3]), sn = sin(v[3]);
  const double Wu[4] = {cs, -sn, sn, cs};
  double q[4] = {sqrt(1 - (v[0] * v[0] + v[1] * v[1] + v[2] * v[2])), v[0], v[1], v[2]};
  const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int i = 0; i < 4; i++) q[i] /= qn;
  double Uu[9];
  q_to_R(q, Uu);
  double U2[9], W2[4];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += U[i * 3 + k] * Uu[k * 3 + j];
      U2[i * 3 + j] = s;
    }
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) W2[i * 2 + j] = Wm[i * 2 + 0] * Wu[0 * 2 + j] + Wm[i * 2 + 1] * Wu[1 * 2 + j];
  double out[6];
  for (int i = 0; i < 3; i++) {
    out[i] = W2[0] * U2[i * 3 + 0];
    out[3 + i] = W2[2] * U2[i * 3 + 1];
  }
  for (int rep = 0; rep < 2; rep++) {  // fromOrthonormal normalises, oplus normalises again
    const double s = 1.0 / n3(out + 3);
    for (int i = 0; i < 6; i++) out[i] *= s;
  }
  for (int i = 0; i < 6; i++) L[i] = out[i];
}

__device__ __forceinline__ SE3 load_T(const double* T) {
  SE3 r;
  for (int i = 0; i < 4; i++) r.q[i] = T[i];
  for (int i = 0; i < 3; i++) r.t[i] = T[4 + i];
  return r;
}

// Edge residual for pose estimate T and landmark values lm (point [3] or line [6]).
__device__ __forceinline__ void edge_error(int type, const double* cam, const double* obs, const SE3& T, const double* lm, double (&e)[4]) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  double R[9];
  q_to_R(T.q, R);
  if (type < 2) {  // EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ: e = obs - proj(T p)
    double Xc[3];
    mat3_vec(R, lm, Xc);
    for (int i = 0; i < 3; i++) Xc[i] += T.t[i];
    const double iz = 1.0 / Xc[2];
    const double u = cam[0] * Xc[0] * iz + cam[2];
    const double v = cam[1] * Xc[1] * iz + cam[3];
    e[0] = obs[0] - u;
    e[1] = obs[1] - v;
    if (type == 1) e[2] = obs[2] - (u - cam[4] * iz);
    return;
  }
  // EdgeSE3ProjectLine / EdgeStereoSE3ProjectLine (edge_project_line.cc:21-42, edge_project_stereo_line.cc:22-51)
  const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3];
  const double Kv0 = -fy * cx, Kv1 = -fx * cy, Kv2 = fx * fy;
  // both sides spelled out (every index of e / obs static: no scratch)
  auto side_err = [&](double tx0, const double* o, double& ea, double& eb) {
    const double t[3] = {tx0, T.t[1], T.t[2]};
    double Rw[3], Rd[3], tx[3];
    mat3_vec(R, lm, Rw);
    mat3_vec(R, lm + 3, Rd);
    cross3(t, Rd, tx);
    const double w0 = Rw[0] + tx[0], w1 = Rw[1] + tx[1], w2 = Rw[2] + tx[2];
    const double l0 = fy * w0, l1 = fx * w1, l2 = Kv0 * w0 + Kv1 * w1 + Kv2 * w2;
    const double nrm = sqrt(l0 * l0 + l1 * l1);
    ea = (o[0] * l0 + o[1] * l1 + l2) / nrm;
    eb = (o[2] * l0 + o[3] * l1 + l2) / nrm;
  };
  side_err(T.t[0], obs, e[0], e[1]);
  if (type == 3) side_err(T.t[0] - cam[4] / fx, obs + 4, e[2], e[3]);  // T_right(0,3) -= b, b = bf / fx
}

// Line-edge Jacobians, analytic (Problem::line_jac = 1): the delta -> 0 limit of g2o's central difference
// (truncation O(delta^2) ~ 1e-18 relative at delta 1e-9; the central difference itself carries ~1e-7 relative
// cancellation noise).  The same derivation and operation order as oracle/ba.c line_jac_analytic (FP
// contraction off: bit-identical to it): pose d wc / d omega = -[wc]x (+ [b]x [c]x on the right camera of a
// stereo edge, c = (bf / fx, 0, 0)), d wc / d upsilon = -[b]x with b = R d; line (Line3D::oplus at 0 after
// its |d| = 1 normalisation) d w / dv = [0, -2 rho u3, 2 rho u2, -(1 + rho^2) u1], d d / dv = [2 u3, 0, -2 u1, 0];
// error e_k = (o_k . l01 + l2) / |l01|, l = [fy wc0, fx wc1, Kv . wc].  Jp [4][6], Jl [4][4] (rows 2 / 4).
__device__ __forceinline__ void skew3(const double* v, double* S) {
  S[0] = 0; S[1] = -v[2]; S[2] = v[1];
  S[3] = v[2]; S[4] = 0; S[5] = -v[0];
  S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

__device__ __forceinline__ void line_jac_analytic(const double* cam, const SE3& T, const double* L, const double* obs,
                                                  bool stereo, double* Jp, double* Jl) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3], bf = cam[4];
  const double M[9] = {fy, 0, 0, 0, fx, 0, -fy * cx, -fx * cy, fx * fy};
  const double dn = n3(L + 3), wn = n3(L);
  double w[3], d[3], u1[3], u3[3], wxd[3];
  for (int i = 0; i < 3; i++) {
    w[i] = L[i] / dn;
    d[i] = L[3 + i] / dn;
    u1[i] = L[i] / wn;
  }
  cross3(L, L + 3, wxd);
  const double cn = n3(wxd);
  for (int i = 0; i < 3; i++) u3[i] = wxd[i] / cn;
  const double rho = wn / dn;
  double dw[4][3], dd[4][3];
  for (int i = 0; i < 3; i++) {
    dw[0][i] = 0;                dd[0][i] = 2 * u3[i];
    dw[1][i] = -2 * rho * u3[i]; dd[1][i] = 0;
    dw[2][i] = 2 * rho * d[i];   dd[2][i] = -2 * u1[i];
    dw[3][i] = -(1 + rho * rho) * u1[i]; dd[3][i] = 0;
  }
  double R[9], a[3], bb[3], Sb[9];
  q_to_R(T.q, R);
  mat3_vec(R, w, a);
  mat3_vec(R, d, bb);
  skew3(bb, Sb);
  for (int side = 0; side < (stereo ? 2 : 1); side++) {
    double t[3] = {T.t[0], T.t[1], T.t[2]};
    const double c[3] = {side == 1 ? bf / fx : 0.0, 0.0, 0.0};
    t[0] -= c[0];
    double txb[3], wc[3];
    cross3(t, bb, txb);
    for (int i = 0; i < 3; i++) wc[i] = a[i] + txb[i];
    double l[3];
    mat3_vec(M, wc, l);
    const double n = sqrt(l[0] * l[0] + l[1] * l[1]);
    double Sw[9], Sc[9], BC[9];
    skew3(wc, Sw);
    skew3(c, Sc);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += Sb[i * 3 + k] * Sc[k * 3 + j];
        BC[i * 3 + j] = s;
      }
    double Gp[3][6], Gl[3][4];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        Gp[i][j] = -Sw[i * 3 + j] + BC[i * 3 + j];
        Gp[i][3 + j] = -Sb[i * 3 + j];
      }
    for (int k = 0; k < 4; k++) {
      double Rw[3], Rd[3], tx[3];
      mat3_vec(R, dw[k], Rw);
      mat3_vec(R, dd[k], Rd);
      cross3(t, Rd, tx);
      for (int i = 0; i < 3; i++) Gl[i][k] = Rw[i] + tx[i];
    }
    for (int ep = 0; ep < 2; ep++) {
      const double* o = obs + 4 * side + 2 * ep;
      const double num = o[0] * l[0] + o[1] * l[1] + l[2];
      const double de_dl[3] = {o[0] / n - num * l[0] / (n * n * n), o[1] / n - num * l[1] / (n * n * n), 1.0 / n};
      double de_dwc[3];
      for (int j = 0; j < 3; j++) de_dwc[j] = de_dl[0] * M[0 * 3 + j] + de_dl[1] * M[1 * 3 + j] + de_dl[2] * M[2 * 3 + j];
      const int r = 2 * side + ep;
      for (int j = 0; j < 6; j++) Jp[r * 6 + j] = de_dwc[0] * Gp[0][j] + de_dwc[1] * Gp[1][j] + de_dwc[2] * Gp[2][j];
      for (int k = 0; k < 4; k++) Jl[r * 4 + k] = de_dwc[0] * Gl[0][k] + de_dwc[1] * Gl[1][k] + de_dwc[2] * Gl[2][k];
    }
  }
}

// a per-type constant of the kernel-argument structs with a select chain: a dynamic index would
// copy the whole by-value struct to scratch
__device__ __forceinline__ double pick4(const double (&a)[4], int t) {
  return t == 0 ? a[0] : t == 1 ? a[1] : t == 2 ? a[2] : a[3];
}

// per-edge Hpp records keep the upper triangle (21 doubles, row-major): the blocks are exactly
// symmetric (the same products summed in the same order for (a, b) and (b, a))
__host__ __device__ constexpr int pk6(int a, int b) { return a * 6 - a * (a - 1) / 2 + (b - a); }

// Hpl records: a point edge (positions [0, Ep)) 6 x 3 at 18 e (row stride 3), a line edge 6 x 4 at
// 18 Ep + 24 (e - Ep) (row stride 4) -- a point record carries no zero column (144 instead of 192 bytes,
// written once and read by the Schur chunks and the next update per trial)
__device__ __forceinline__ int hpl_off(int Ep, int e) { return e < Ep ? 18 * e : 18 * Ep + 24 * (e - Ep); }
// edge e's record as 6 x 4 (column 3 zero for a point edge); every load at a valid address, then selected
__device__ __forceinline__ void load_hpl4(const double* H, int Ep, int e, double (&B)[24]) {
  const int o = hpl_off(Ep, e), st = e < Ep ? 3 : 4;
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const double v = H[o + r * st + (c < st ? c : st - 1)];
      B[r * 4 + c] = c < st ? v : 0.0;
    }
}

__device__ __forceinline__ int edim(int t) { return t == 0 ? 2 : t == 1 ? 3 : t == 2 ? 2 : 4; }

// point edges only (t < 2), every index static: edge_error's point branch and its chi2 (info I)
__device__ __forceinline__ double point_error_R(int t, const double* cam, const double* obs, const double (&R)[9],
                                                const double* tt, const double* X, double (&e)[4]) {
  double Xc[3];
  mat3_vec(R, X, Xc);
  for (int i = 0; i < 3; i++) Xc[i] += tt[i];
  const double iz = 1.0 / Xc[2];
  const double u = cam[0] * Xc[0] * iz + cam[2];
  const double v = cam[1] * Xc[1] * iz + cam[3];
  e[0] = obs[0] - u;
  e[1] = obs[1] - v;
  e[2] = t == 1 ? obs[2] - (u - cam[4] * iz) : 0.0;
  e[3] = 0.0;
  double chi2 = 0;
  chi2 += e[0] * e[0];
  chi2 += e[1] * e[1];
  if (t == 1) chi2 += e[2] * e[2];
  return chi2 * 1.0;
}
__device__ __forceinline__ double point_error(int t, const double* cam, const double* obs, const SE3& T,
                                              const double* X, double (&e)[4]) {
  double R[9];
  q_to_R(T.q, R);
  return point_error_R(t, cam, obs, R, T.t, X, e);
}

// edge e's observation (type t): point edges [0, Ep) at stride 4 (u, v, u_r), line edges [Ep, E)
// at stride 8 after them (edges are in landmark-CSR order: point landmarks first)
__device__ __forceinline__ const double* obs_of(const Problem& P, int e, int t) {
  return t < 2 ? P.eobs + 4 * e : P.eobs + 4 * P.Ep + 8 * (e - P.Ep);
}
__device__ __forceinline__ int ldim(int t) { return t < 2 ? 3 : 4; }
__device__ __forceinline__ double einfo(int t) { return t < 2 ? 1.0 : 0.1; }

__device__ __forceinline__ const double* lm_ptr(const Problem& P, int g) {
  return g < P.nq ? P.X + 3 * g : P.L + 6 * (g - P.nq);
}

// Huber (RobustKernelHuber::robustify): rho0, rho1
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


// ---------------------------------------------------------------------------
// errors + robust chi2 per active edge.  The last block to finish (ticket counter)
// sums the block partials -- and the update kernel's scale partials -- in a fixed
// order, posts {chi2, scale, maxdiag, fail} + seq to the host-mapped mailbox and
// re-arms the device state (counter, fail flag, maxdiag) for the next trial.
// ---------------------------------------------------------------------------
// Mailbox post into fine-grained (uncached) host memory: the four values, then -- once they
// have completed (vmcnt) -- the sequence number the host spins on.  No release fence: a
// system/agent-scope release writes back the whole L2 (~3.5 us, MI355X_MICROARCH.md), once per
// LM trial on the critical path; the host reads only these uncached words.
__device__ __forceinline__ void post_mail(Mail* m, double v0, double v1, double v2, double v3, unsigned long long seq) {
  // vseq first (a reader that sees it change knows v is being rewritten), then v, then seq
  __hip_atomic_store(&m->vseq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&m->v[0], v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&m->v[1], v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&m->v[2], v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&m->v[3], v3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&m->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- device-side LM control (Sys::lm) ----
// Trial entry: false when the optimize() has already stopped (this trial is a no-op); else the
// damping, the current bank and whether the candidate's speculative linearisation is wanted
// (not in the last iteration).  Uniform scalar loads; the control was written by the previous
// trial's last kernel (kernel boundary = visibility).
struct LmView {
  double lambda;
  int cur, spec;
};
__device__ __forceinline__ bool lm_view(const Sys& S, LmView& v) {
  const LmCtrl* c = S.lm + S.lm_slot;
  if (c->stop) return false;
  v.lambda = c->lambda;
  v.cur = c->cur;
  v.spec = c->it + 1 < c->iters;
  return true;
}
template <typename T>
__device__ __forceinline__ void swp(T& a, T& b) {
  T t = a;
  a = b;
  b = t;
}
// bank 1 current: the host's candidate state / spare records are the current ones
__device__ __forceinline__ void bank_state(Problem& P) {
  swp(P.T, P.Tn);
  swp(P.X, P.Xn);
  swp(P.L, P.Ln);
}
__device__ __forceinline__ void bank_lin(Lin& L, Lin& Ls, Sys& S, Sys& Ss) {
  swp(L.Hpp, Ls.Hpp);
  swp(L.bp, Ls.bp);
  swp(L.Hll, Ls.Hll);
  swp(L.bl, Ls.bl);
  swp(L.Hpl, Ls.Hpl);
  swp(S.Hll, Ss.Hll);
  swp(S.bl, Ss.bl);
}
// One trial's verdict, g2o OptimizationAlgorithmLevenberg::solve as restated by ba.cpp optimize()
// (g2o_optimization.cc:172-210 runs optimize(10) / optimize(5)): rho test with the LM scale,
// damping update (accept: lambda *= max(1/3, min(2/3, 1 - (2 rho - 1)^3)), ni = 2; reject:
// lambda *= ni, ni *= 2), at most 10 trials per iteration, stop at qmax == 10 or rho == 0.
// Returns 1 when the optimize() is finished.
__device__ int lm_decide(const LmCtrl* c, LmCtrl* n, double chi2, double scale, double fail) {
  const bool ok = fail == 0.0;
  const double tempChi = ok ? chi2 : DBL_MAX;
  double rho = c->chi - tempChi;
  rho /= ok ? scale + 1e-3 : 1.0;
  double lambda = c->lambda, ni = c->ni;
  int qmax = c->qmax, it = c->it;
  bool brk = false;
  *n = *c;
  if (rho > 0 && isfinite(tempChi) && ok) {
    double alpha = 1. - cube(2 * rho - 1);  // pow(2 rho - 1, 3)
    alpha = fmin(alpha, 2. / 3.);
    lambda *= fmax(1. / 3., alpha);
    ni = 2;
    n->chi = tempChi;
    n->cur = c->cur ^ 1;
  } else {
    lambda *= ni;
    ni *= 2;
    brk = !isfinite(lambda);
  }
  if (!brk) qmax++;
  int stop = 0;
  if (brk || !(rho < 0 && qmax < 10)) {  // the iteration ends
    it++;
    if (qmax == 10 || rho == 0 || !isfinite(lambda) || it >= c->iters) stop = 1;
    else qmax = 0;
  }
  n->lambda = lambda;
  n->ni = ni;
  n->qmax = qmax;
  n->it = it;
  n->trials = c->trials + 1;
  n->stop = stop;
  return stop;
}

// Last-block ticket: this block's partials were stored device-coherent (relaxed agent-scope
// atomics, written through), so completing them (vmcnt) before a relaxed ticket increment is
// enough -- an acq_rel ticket would write back and invalidate the L2 in every block.
__device__ __forceinline__ unsigned ticket(unsigned* counter) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double block_sum256(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void errors_kernel(Problem P, Lin L, Active A, Sys S, int nb_scale,
                                                     unsigned long long seq) {
  __shared__ double red[256];
  __shared__ int last;
  const int i = blockIdx.x * 256 + threadIdx.x;
  double c = 0.0;
  if (i < A.Ea && (!A.elevel || !A.elevel[i])) {
    const int e = i;
    const int t = P.etype[e];
    const SE3 T = load_T(P.T + 8 * P.epose[e]);
    double er[4] = {0, 0, 0, 0};
    edge_error(t, P.cams + 5 * P.ecam[e], obs_of(P, e, t), T, lm_ptr(P, P.elm[e]), er);
    double chi2 = 0;
    for (int k = 0; k < edim(t); k++) chi2 += er[k] * er[k];
    chi2 *= einfo(t);
    for (int k = 0; k < 4; k++) L.err[4 * e + k] = er[k];
    if (A.robust) {
      double r1;
      huber(chi2, pick4(P.delta, t), c, r1);
    } else {
      c = chi2;
    }
  }
  const double bsum = block_sum256(c, red);
  if (threadIdx.x == 0) {
    __hip_atomic_store(S.partial + blockIdx.x, bsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned tk = ticket(S.counter);
    last = tk == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double c2 = 0, sc = 0;
  for (int k = threadIdx.x; k < (int)gridDim.x; k += 256)
    c2 += __hip_atomic_load(S.partial + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = threadIdx.x; k < nb_scale; k += 256) sc += S.partial2[k];
  const double chi2 = block_sum256(c2, red);
  const double scale = block_sum256(sc, red);
  if (threadIdx.x == 0) {
    const double f = (double)__hip_atomic_load(S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double mx = S.out[2];
    S.out[0] = chi2;
    S.out[1] = scale;
    S.out[3] = f;
    if (S.shard_out) {  // sharded: this rank's share goes to the all-reduce, shard_post posts
      S.shard_out[0] = chi2;
      S.shard_out[1] = scale;
      S.shard_out[2] = f;
      __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(S.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      S.out[2] = 0.0;
      return;
    }
    __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(S.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.out[2] = 0.0;
    if (seq) post_mail(S.mail, chi2, scale, mx, f, seq);  // seq 0: nobody waits (device-side LM)
  }
}

// mailbox post of the lambda-init statistic (max Hessian diagonal) after the first linearisation;
// with npd > 0 it first folds in the pose blocks: per pose, the npd block partials of
// pose_diag_kernel summed in order
__global__ __launch_bounds__(256) void post_kernel(Sys S, int K, int npd, unsigned long long seq, int lm_iters) {
  __shared__ double part[4][64];
  if (npd > 0) {  // entry q = 6 pose + diagonal index: 4 waves each sum every 4th block partial
    const int lane = threadIdx.x & 63, pt = threadIdx.x >> 6, nq6 = 6 * K;
    double mx = 0;
    for (int q0 = 0; q0 < nq6; q0 += 64) {
      const int q = q0 + lane;
      double sacc = 0;
      if (q < nq6) {
        const int pa = q / 6, i = q - 6 * pa;
        const double* src = S.partial2 + (size_t)pa * npd * 6 + i;
        for (int b = pt; b < npd; b += 4) sacc += src[(size_t)b * 6];
      }
      part[pt][lane] = sacc;
      __syncthreads();
      if (pt == 0 && q < nq6) mx = fmax(mx, fabs(((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]));
      __syncthreads();
    }
    if (pt == 0) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
      if (lane == 0) S.out[2] = fmax(S.out[2], mx);
    }
  }
  if (threadIdx.x != 0) return;
  if (S.lm && lm_iters > 0) {  // device-side LM: computeLambdaInit (tau = 1e-5 x max diagonal)
    LmCtrl* c = S.lm;  // slot 0: the first trial's
    c->lambda = 1e-5 * S.out[2];
    c->ni = 2;
    c->chi = S.out[0];
    c->cur = 0;
    c->it = 0;
    c->qmax = 0;
    c->stop = 0;
    c->iters = lm_iters;
    c->trials = 0;
    return;  // the host waits for the trials only
  }
  post_mail(S.mail, S.out[0], S.out[1], S.out[2],
            (double)__hip_atomic_load(S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), seq);
}

// ---------------------------------------------------------------------------
// per-edge Jacobians + weighted normal-equation contributions
// ---------------------------------------------------------------------------
// Writes the 86 contributions of one edge (Hll, bl, and -- for an optimised pose -- Hpp, bp, Hpl).
__device__ __forceinline__ double contrib(int o, int rows, int ld, double w, const double* er, const double* Jp,
                                          const double* Jl) {
  // o in [0, 86): 0..15 Hll (ld x ld), 16..19 bl, 20..55 Hpp, 56..61 bp, 62..85 Hpl (6 x 4)
  double s = 0;
  if (o < 16) {
    const int a = o / ld, b = o % ld;
    if (o >= ld * ld) return 0;
    for (int r = 0; r < rows; r++) s += Jl[r * 4 + a] * Jl[r * 4 + b];
    return w * s;
  }
  if (o < 20) {
    const int a = o - 16;
    if (a >= ld) return 0;
    for (int r = 0; r < rows; r++) s += Jl[r * 4 + a] * er[r];
    return -w * s;
  }
  if (o < 56) {
    const int a = (o - 20) / 6, b = (o - 20) % 6;
    for (int r = 0; r < rows; r++) s += Jp[r * 6 + a] * Jp[r * 6 + b];
    return w * s;
  }
  if (o < 62) {
    const int a = o - 56;
    for (int r = 0; r < rows; r++) s += Jp[r * 6 + a] * er[r];
    return -w * s;
  }
  const int a = (o - 62) / 4, b = (o - 62) % 4;
  if (b >= ld) return 0;
  for (int r = 0; r < rows; r++) s += Jp[r * 6 + a] * Jl[r * 4 + b];
  return w * s;
}

__device__ __forceinline__ void store_contrib(const Lin& L, int Ep, int e, int o, double v, bool pose_opt) {
  if (o < 16) L.Hll[16 * e + o] = v;
  else if (o < 20) L.bl[4 * e + o - 16] = v;
  else if (!pose_opt) return;
  else if (o < 56) {
    const int a = (o - 20) / 6, b = (o - 20) % 6;
    if (b >= a) L.Hpp[21 * e + pk6(a, b)] = v;
  }
  else if (o < 62) L.bp[6 * e + o - 56] = v;
  else L.Hpl[hpl_off(Ep, e) + o - 62] = v;  // (line edges: 6 x 4)
}

__device__ __forceinline__ double edge_weight_of(const Problem& P, const Active& A, const double* er, int t) {
  double w = einfo(t);
  if (A.robust) {
    double chi2 = 0;
    for (int k = 0; k < edim(t); k++) chi2 += er[k] * er[k];
    chi2 *= einfo(t);
    double r0, r1;
    huber(chi2, pick4(P.delta, t), r0, r1);
    w *= r1;  // robustInformation = rho'(chi2) * Omega
  }
  return w;
}

__device__ __forceinline__ double edge_weight(const Problem& P, const Lin& L, const Active& A, int e, int t) {
  return edge_weight_of(P, A, L.err + 4 * e, t);
}

// point edges: analytic Jacobians (g2o types_sba, EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::linearizeOplus).
// Mono edges carry a zero third row, so every index below is a compile-time constant (register resident, no
// scratch).
__device__ __forceinline__ void point_jac_R(int t, const double (&R)[9], const double* tt, const double* cam,
                                            const double* Xg, double (&Jp)[3][6], double (&Jl)[3][3]) {
  const double fx = cam[0], fy = cam[1], bf = cam[4];
  double Xc[3];
  mat3_vec(R, Xg, Xc);
#pragma unroll
  for (int k = 0; k < 3; k++) Xc[k] += tt[k];
  const double x = Xc[0], y = Xc[1], z = Xc[2], iz = 1.0 / z, iz2 = iz * iz;
  const bool st = t == 1;
  const double D[3][3] = {{fx * iz, 0, -fx * x * iz2},
                          {0, fy * iz, -fy * y * iz2},
                          {st ? fx * iz : 0.0, 0, st ? -fx * x * iz2 + bf * iz2 : 0.0}};
  const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      double s = 0, sl = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        s += D[r][k] * SX[k * 3 + c];
        sl += D[r][k] * R[k * 3 + c];
      }
      Jp[r][c] = s;            // -D * (-[Xc]x)
      Jp[r][3 + c] = -D[r][c]; // -D * I
      Jl[r][c] = -sl;          // -D * R
    }
}
__device__ __forceinline__ void point_jac(int t, const SE3& T, const double* cam, const double* Xg, double (&Jp)[3][6],
                                          double (&Jl)[3][3]) {
  double R[9];
  q_to_R(T.q, R);
  point_jac_R(t, R, T.t, cam, Xg, Jp, Jl);
}

// the pose block of one point edge: Hpp (upper triangle, pk6) = w Jp^T Jp, bp = -w Jp^T e
__device__ __forceinline__ void point_pose_terms(const double (&Jp)[3][6], double w, const double (&er)[3],
                                                 double (&Hp)[21], double (&bpv)[6]) {
#pragma unroll
  for (int a = 0; a < 6; a++) {
#pragma unroll
    for (int b = a; b < 6; b++) Hp[pk6(a, b)] = w * (Jp[0][a] * Jp[0][b] + Jp[1][a] * Jp[1][b] + Jp[2][a] * Jp[2][b]);
    bpv[a] = -w * (Jp[0][a] * er[0] + Jp[1][a] * er[1] + Jp[2][a] * er[2]);
  }
}

// Writes the pose-side records of point edge e (when its pose is optimised): Hpl, and -- only with PDIAG
// (the first linearisation of an optimize(), read by computeLambdaInit's pose_diag) -- the six diagonal
// entries of Hpp.  The pose block itself (Hpp, bp) is never stored for a point edge: the diagonal pose
// pair's Schur chunk recomputes it from the state (point_pose_block), which costs less than the 216 bytes
// per edge and trial of writing it and reading it back.  Accumulates the landmark side (Hll 3x3, bl 3) into
// hl / bv.  The operands in registers (pose T, camera, landmark, the edge's error er).
template <bool PDIAG>
__device__ __forceinline__ void point_edge_core(const Problem& P, const Lin& L, const Active& A, int e, int t,
                                                bool pose_opt, const SE3& T, const double* cam, const double* Xg,
                                                const double* er4, double (&hl)[9], double (&bv)[3],
                                                double* dg6 = nullptr) {
  double Jp[3][6], Jl[3][3];
  point_jac(t, T, cam, Xg, Jp, Jl);
  const bool st = t == 1;
  const double w = edge_weight_of(P, A, er4, t);
  const double er[3] = {er4[0], er4[1], st ? er4[2] : 0.0};
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) hl[a * 3 + b] += w * (Jl[0][a] * Jl[0][b] + Jl[1][a] * Jl[1][b] + Jl[2][a] * Jl[2][b]);
#pragma unroll
  for (int a = 0; a < 3; a++) bv[a] += -w * (Jl[0][a] * er[0] + Jl[1][a] * er[1] + Jl[2][a] * er[2]);
  if (!pose_opt) return;
  double* Hpl = L.Hpl + 18 * e;  // (hpl_off: a point edge)
#pragma unroll
  for (int a = 0; a < 6; a++) {
    if (PDIAG) {
      const double d = w * (Jp[0][a] * Jp[0][a] + Jp[1][a] * Jp[1][a] + Jp[2][a] * Jp[2][a]);
      L.Hpp[21 * e + pk6(a, a)] = d;
      if (dg6) dg6[a] = d;
    }
#pragma unroll
    for (int b = 0; b < 3; b++) Hpl[a * 3 + b] = w * (Jp[0][a] * Jl[0][b] + Jp[1][a] * Jl[1][b] + Jp[2][a] * Jl[2][b]);
  }
}

// The pose block (Hpp upper triangle, bp) of a live point edge of type t on an optimised pose at the state
// its records were linearised at (pose rotation R / translation tt, camera cam, observation ob, point Xg of
// the current bank): the error, the robust weight and the pose Jacobian formed again, exactly as
// point_edge_core's linearisation (same operations on the same operands).
__device__ __forceinline__ void point_pose_block(const Problem& P, const Active& A, int t, const double* Rt,
                                                 const double* cam, const double* ob, const double* Xg,
                                                 double (&Hp)[21], double (&bpv)[6]) {
  double R[9];
#pragma unroll
  for (int i = 0; i < 9; i++) R[i] = Rt[i];
  const double* tt = Rt + 9;
  double er4[4];
  point_error_R(t, cam, ob, R, tt, Xg, er4);
  double Jp[3][6], Jl[3][3];
  point_jac_R(t, R, tt, cam, Xg, Jp, Jl);
  const double w = edge_weight_of(P, A, er4, t);
  const double er[3] = {er4[0], er4[1], t == 1 ? er4[2] : 0.0};
  point_pose_terms(Jp, w, er, Hp, bpv);
}

// A diagonal pose pair's chunk: its pose (every e1 of its pairs is on it) and the cameras, for
// point_pose_block; the cameras in the chunk wave's LDS
struct DiagPose {
  const double* pose;  // R (9, row-major) and t (3) of the pose
  const double* cams;  // [ncam][5]
};

// (point edges: Hpl, and with PDIAG the Hpp diagonal pose_diag reads; see point_edge_core)
template <bool PDIAG>
__device__ __forceinline__ void zero_pose_records(const Lin& L, int e) {
  if (PDIAG)
#pragma unroll
    for (int k = 0; k < 6; k++) L.Hpp[21 * e + pk6(k, k)] = 0.0;
#pragma unroll
  for (int k = 0; k < 18; k++) L.Hpl[18 * e + k] = 0.0;
}

// point edges: analytic Jacobians (g2o types_sba).  Mono edges carry a zero third
// row, so every index below is a compile-time constant (register resident, no scratch).
// Writes the pose-side records of edge e (when its pose is optimised) and accumulates
// the landmark side (Hll 3x3, bl 3) into hl / bv.
__device__ __forceinline__ void point_edge(const Problem& P, const Lin& L, const Active& A, int e, bool pose_opt,
                                           const double* Tb, const double* Xg, double (&hl)[9], double (&bv)[3]) {
  if (A.elevel && A.elevel[e]) {  // outside this phase: exact-zero records, no contribution
    if (pose_opt) zero_pose_records<true>(L, e);
    return;
  }
  const int t = P.etype[e];
  point_edge_core<true>(P, L, A, e, t, pose_opt, load_T(Tb + 8 * P.epose[e]), P.cams + 5 * P.ecam[e], Xg, L.err + 4 * e, hl,
                  bv);
}

__device__ __forceinline__ void atomic_max_pos(double* addr, double v) {
  // non-negative doubles order like their bit patterns
  atomicMax(reinterpret_cast<unsigned long long*>(addr), (unsigned long long)__double_as_longlong(v));
}

// orders this wave's LDS writes before its later LDS reads (lanes exchange through LDS)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// sum over the kGroup lanes of a landmark group (fixed butterfly: deterministic; every
// lane of the wave takes part)
constexpr int kGroup = 8;
#ifndef RSPL_UE_WAVES
#define RSPL_UE_WAVES 4
#endif
constexpr int kUeWaves = RSPL_UE_WAVES;  // waves per update_errors workgroup that carry landmark groups
template <int N>
__device__ __forceinline__ void group_sum(double (&v)[N]) {
#pragma unroll
  for (int o = 1; o < kGroup; o <<= 1)
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += __shfl_xor(v[i], o);
}

// point landmarks: a group of kGroup lanes per landmark, lane j linearises edges j, j+8, ...
// of the landmark's CSR list; the group sums Hll / bl (no per-edge landmark records)
__device__ __forceinline__ void lin_point_landmarks(const Problem& P, const Lin& L, const Active& A, const Sys& S,
                                                    int t, bool maxd) {
  const int g = t / kGroup, j = t % kGroup;
  double hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bv[3] = {0, 0, 0};
  const bool in = g < P.nq;
  if (in) {
    const int k1 = A.lm_off[g + 1];
    for (int k = A.lm_off[g] + j; k < k1; k += kGroup)
      point_edge(P, L, A, (k), A.lm_pose[k] >= 0, P.T, P.X + 3 * g, hl, bv);
  }
  group_sum(hl);
  group_sum(bv);
  if (!in || j != 0 || !A.lm_act[g]) return;
  double* H = S.Hll + 16 * g;
#pragma unroll
  for (int i = 0; i < 9; i++) H[i] = hl[i];
#pragma unroll
  for (int i = 9; i < 16; i++) H[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 3; i++) S.bl[4 * g + i] = bv[i];
  S.bl[4 * g + 3] = 0.0;
  if (maxd) atomic_max_pos(S.out + 2, fmax(fabs(hl[0]), fmax(fabs(hl[4]), fabs(hl[8]))));
}

// Gauss-Jordan inverse with partial pivoting, fully unrolled (register resident).
// Progressive conditional row swaps select the same pivot as a max search.
template <int N>
__device__ __forceinline__ bool small_inv(const double* A, double* I) {
  double M[N][2 * N];
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++) {
      M[i][j] = A[i * N + j];
      M[i][N + j] = (i == j) ? 1.0 : 0.0;
    }
  bool ok = true;
#pragma unroll
  for (int c = 0; c < N; c++) {
#pragma unroll
    for (int r = c + 1; r < N; r++) {
      const bool sw = fabs(M[r][c]) > fabs(M[c][c]);
#pragma unroll
      for (int k = 0; k < 2 * N; k++) {
        const double a = M[c][k], b = M[r][k];
        M[c][k] = sw ? b : a;
        M[r][k] = sw ? a : b;
      }
    }
    ok = ok && (M[c][c] != 0.0);
    const double iv = 1.0 / M[c][c];
#pragma unroll
    for (int k = 0; k < 2 * N; k++) M[c][k] *= iv;
#pragma unroll
    for (int r = 0; r < N; r++)
      if (r != c) {
        const double f = M[r][c];
#pragma unroll
        for (int k = 0; k < 2 * N; k++) M[r][k] -= f * M[c][k];
      }
  }
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++) I[i * N + j] = M[i][N + j];
  return ok;
}

// (Hll_g + lambda I)^-1, zero-padded to 4x4 for points
__device__ __forceinline__ bool lm_dinv(const double* Hll, bool point, double lambda, double (&D)[16]) {
  if (point) {
    double H[9], Di[9];
#pragma unroll
    for (int i = 0; i < 9; i++) H[i] = Hll[i];
    H[0] += lambda;
    H[4] += lambda;
    H[8] += lambda;
    const bool ok = small_inv<3>(H, Di);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) D[i * 4 + j] = (i < 3 && j < 3) ? Di[i * 3 + j] : 0.0;
    return ok;
  }
  double H[16];
#pragma unroll
  for (int i = 0; i < 16; i++) H[i] = Hll[i];
#pragma unroll
  for (int i = 0; i < 4; i++) H[i * 5] += lambda;
  return small_inv<4>(H, D);
}

// line edges: g2o's numeric central difference (delta 1e-9).  A workgroup takes the
// <= kLineBlk = 8 edges of a run of whole line landmarks (A.ltab, CSR order) and splits the 20
// perturbed error evaluations of each by kind, so no
// wave diverges between the two transcendental paths: wave 0 evaluates the +-delta line
// perturbations of all 8 edges (Line3D::oplus, 8 lanes per edge), waves 1-2 the +-delta pose
// perturbations (SE3 exp, 12 lanes per edge).  The workgroup sums each landmark's edge
// records in CSR order into the landmark block itself; only a landmark with more than
// kLineBlk edges (split over workgroups) goes through per-edge records written through (sc1)
// and a last-edge ticket.
// MODE kLinSpec: the speculative linearisation (at the candidate P.Tn / candidate lines) inside
// update_errors_kernel, from the kernel's start: wave 0 forms the candidate of each of the block's
// line landmarks itself -- the same back-substitution as the landmark groups (8 lanes per
// landmark, the same butterfly, from the current records Lc / Sc) -- so it never waits for the
// groups; wave 3 evaluates each edge's own error at the candidate.
// MODE kLinSetup: the first pass of a device-LM optimize() (setup_kernel): wave 3 evaluates each
// edge's error at the current state (no separate error kernel), the block returns the robust cost of
// its edges (*chi_out, slot order) and, with cls (the second optimize), classifies its edges from
// their last computed errors itself (classify_edge) -- the landmark groups of the same launch write
// the levels, so none is read here.  The line edges' errors are not stored: the first trial's update
// rewrites every edge's error before anything reads them.
// candidate pose i of this trial (g2o VertexSE3Expmap::oplusImpl, the left update exp(xp) T):
// copied when the pose is not optimised or the solve failed
__device__ __forceinline__ void cand_pose(const Problem& P, const Active& A, const double* x, int i, bool failed,
                                          double (&o)[8]) {
  const int a = A.pidx[i];
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = P.T[8 * i + k];
  if (a < 0 || failed) return;
  double xp[6];
#pragma unroll
  for (int k = 0; k < 6; k++) xp[k] = x[6 * a + k];
  const SE3 r = se3_mul(se3_exp(xp), load_T(o));
#pragma unroll
  for (int k = 0; k < 4; k++) o[k] = r.q[k];
#pragma unroll
  for (int k = 0; k < 3; k++) o[4 + k] = r.t[k];
  o[7] = 0;
}

// outlier levels after the first optimize / final inlier flags (g2o_optimization.cc:176-231).
// Reads only fields that are NOT banked: L.err (swapped by neither bank_lin nor accept_swap) and the state
// P.T / P.X.  The speculative final kernel (SpecFinish, ba.cpp) reuses the Lin captured before optimize(5)
// and banks only the state; a classification that read a banked Lin field (Hpp, bp, Hll, bl, Hpl) would
// differ between that path and the host-ordered one (tests/test_gpu_ba.py test_ba_final_kernel_paths_agree).
__device__ __forceinline__ void edge_status(const Problem& P, const Lin& L, int e, double& chi2, bool& depth_ok) {
  const int t = P.etype[e];
  chi2 = 0;
  for (int k = 0; k < edim(t); k++) chi2 += L.err[4 * e + k] * L.err[4 * e + k];
  chi2 *= einfo(t);
  depth_ok = true;
  if (t < 2) {
    const SE3 T = load_T(P.T + 8 * P.epose[e]);
    double R[9], Xc[3];
    q_to_R(T.q, R);
    mat3_vec(R, P.X + 3 * P.elm[e], Xc);
    depth_ok = Xc[2] + T.t[2] > 0.0;
  }
}
constexpr int kLinPlain = 0, kLinSpec = 1, kLinSetup = 2;
// phase-2 level of edge e from its last computed error (classify_edge, g2o_optimization.cc:176-213)
__device__ __forceinline__ bool edge_outlier(const Problem& P, const Lin& L, int e) {
  double chi2;
  bool depth_ok;
  edge_status(P, L, e, chi2, depth_ok);
  return chi2 > pick4(P.th, P.etype[e]) || !depth_ok;
}
// line landmark g is active: it has an edge of level 0 (cls) / the phase's activity (A.lm_act)
__device__ __forceinline__ bool line_active(const Problem& P, const Lin& L, const Active& A, int g, bool cls) {
  if (!cls) return A.lm_act[g] != 0;
  for (int k = A.lm_off[g]; k < A.lm_off[g + 1]; k++)
    if (!edge_outlier(P, L, k)) return true;
  return false;
}
template <int MODE>
__device__ __forceinline__ void lin_lines(const Problem& P, const Lin& L, const Active& A, const Sys& S, int blk,
                                          bool maxd, const Lin* Lc = nullptr, const Sys* Sc = nullptr,
                                          double lambda = 0.0, bool failed = false,
                                          unsigned long long* stamp = nullptr, bool cls = false,
                                          double* chi_out = nullptr, double* pdg = nullptr, int pd_nb = 0,
                                          int pd_b = 0) {
  constexpr bool SPEC = MODE == kLinSpec, SETUP = MODE == kLinSetup, OWN_ERR = SPEC || SETUP;
  __shared__ double ev[kLineBlk][20][4];
  __shared__ double J[kLineBlk][4 * 6 + 4 * 4];
  __shared__ double Lsh[kLineBlk][6];
  __shared__ double es[kLineBlk][4];
  __shared__ int einfo_s[kLineBlk][4];  // edge id, type, flags (1 on, 2 live, 4 pose optimised), landmark
  __shared__ double cv[kLineBlk][20];   // landmark-side records (Hll 16, bl 4) of each edge
  __shared__ double Tsh[kLineBlk][8];   // SPEC: each edge's candidate pose
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int4 tb = A.ltab[blk];
  const int p0 = tb.x, cnt = tb.y & 0xff, gb = tb.z, ge = tb.w;
  const bool split = (tb.y >> 8) != 0;
  auto edge = [&](int slot, int& e, int& t, bool& on, bool& live) {
    e = einfo_s[slot][0];
    t = einfo_s[slot][1];
    on = einfo_s[slot][2] & 1;
    live = einfo_s[slot][2] & 2;
  };
  __shared__ double cand[kLineBlk][6];  // SPEC: the candidate line of landmark gb + m
  if (SPEC && wv == 0) {
    const int m = lane >> 3, j = lane & 7;
    const int g = gb + m;
    const bool in = g < ge;
    const int l = g - P.nq;
    const bool upd = in && A.lm_act[g] && !failed;
    double c[4] = {0, 0, 0, 0}, hb[20], lmv[6] = {0, 0, 0, 0, 0, 0};
    if (in) {  // the landmark-only operands in the first round trip
#pragma unroll
      for (int q = 0; q < 16; q++) hb[q] = Sc->Hll[16 * g + q];
#pragma unroll
      for (int q = 0; q < 4; q++) hb[16 + q] = Sc->bl[4 * g + q];
#pragma unroll
      for (int q = 0; q < 6; q++) lmv[q] = P.L[6 * l + q];
    }
    if (upd)
      for (int k = A.lm_off[g] + j; k < A.lm_off[g + 1]; k += kGroup) {
        const int a = A.lm_pose[k];
        if (a < 0) continue;
        const double* B = Lc->Hpl + hpl_off(P.Ep, k);  // (a line edge: 6 x 4)
        const double* xp = S.x + 6 * a;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          double sm = 0;
#pragma unroll
          for (int r = 0; r < 6; r++) sm += B[r * 4 + q] * xp[r];
          c[q] -= sm;
        }
      }
    group_sum(c);
    if (upd) {
#pragma unroll
      for (int q = 0; q < 4; q++) c[q] += hb[16 + q];
      double D[16];
      lm_dinv(hb, false, lambda, D);
      double xl[4];
#pragma unroll
      for (int r = 0; r < 4; r++) xl[r] = D[r * 4] * c[0] + D[r * 4 + 1] * c[1] + D[r * 4 + 2] * c[2] + D[r * 4 + 3] * c[3];
      line_oplus(lmv, xl);
    }
    if (in && j == 0)
#pragma unroll
      for (int q = 0; q < 6; q++) cand[m][q] = lmv[q];
  }
  // per edge (SPEC: wave 1, beside wave 0's candidate lines): its attributes and the current line
  // (SPEC: its candidate pose) into LDS
  const int es_ = SPEC ? tid - 64 : tid;
  if (es_ >= 0 && es_ < kLineBlk) {
    const int tid = es_;
    const bool on = tid < cnt;
    const int e = on ? (p0 + tid) : 0;
    const int t = on ? P.etype[e] : 2;
    // outside this phase: exact-zero records (setup: the level from the edge's last error)
    const bool live = on && !(SETUP ? (cls && edge_outlier(P, L, e)) : (A.elevel && A.elevel[e]));
    const bool popt = on && A.pidx[P.epose[e]] >= 0;
    einfo_s[tid][0] = e;
    einfo_s[tid][1] = t;
    einfo_s[tid][2] = (on ? 1 : 0) | (live ? 2 : 0) | (popt ? 4 : 0);
    einfo_s[tid][3] = on ? P.elm[e] : gb;
    if (live) {
      const int l = P.elm[e] - P.nq;
      if (SPEC) {
        double Tc[8];
        cand_pose(P, A, S.x, P.epose[e], failed, Tc);
#pragma unroll
        for (int k = 0; k < 8; k++) Tsh[tid][k] = Tc[k];
      } else {
        for (int k = 0; k < 6; k++) Lsh[tid][k] = P.L[6 * l + k];
      }
    }
  }
  __syncthreads();
  if (stamp && tid == 0) stamp[0] = wall_clock64();
  const double delta = 1e-9, scal = 1.0 / (2 * delta);
  {
    // this thread's evaluation: wave 0 line perturbations, waves 1-2 pose perturbations,
    // wave 3 (SPEC) the unperturbed error
    int slot = -1, m = 0;
    if (wv == 0) {
      slot = lane >> 3;
      m = lane & 7;  // ev row 2d + sign, d < 4
    } else if (wv < 3) {
      const int idx = (wv - 1) * 64 + lane;
      if (idx < 12 * kLineBlk) {
        slot = idx / 12;
        m = 8 + idx % 12;  // ev row 2d + sign, d = 4..9
      }
    } else if (OWN_ERR && lane < kLineBlk) {
      slot = lane;
      m = 20;
    }
    if (P.line_jac) {  // analytic: one lane per edge (wave 0), its error too (OWN_ERR)
      slot = (wv == 0 && lane < kLineBlk) ? lane : -1;
      m = OWN_ERR ? 20 : 21;
    }
    int e = 0, t = 2;
    bool on = false, live = false;
    if (slot >= 0) edge(slot, e, t, on, live);
    if (live && P.line_jac) {
      const SE3 T = load_T(SPEC ? &Tsh[slot][0] : P.T + 8 * P.epose[e]);
      const double* cam = P.cams + 5 * P.ecam[e];
      const double* obs = obs_of(P, e, t);
      double Lp[6];
      for (int k = 0; k < 6; k++) Lp[k] = SPEC ? cand[einfo_s[slot][3] - gb][k] : Lsh[slot][k];
      double Jp[24], Jl[16];
#pragma unroll
      for (int k = 0; k < 24; k++) Jp[k] = 0.0;
#pragma unroll
      for (int k = 0; k < 16; k++) Jl[k] = 0.0;
      line_jac_analytic(cam, T, Lp, obs, t == 3, Jp, Jl);
      // whole rows (static indices: no scratch); rows >= edim(t) are zero and never read
#pragma unroll
      for (int k = 0; k < 16; k++) J[slot][24 + k] = Jl[k];
#pragma unroll
      for (int k = 0; k < 24; k++) J[slot][k] = Jp[k];
      if (OWN_ERR) {
        double er[4] = {0, 0, 0, 0};
        edge_error(t, cam, obs, T, Lp, er);
        for (int k = 0; k < 4; k++) es[slot][k] = er[k];
      }
    } else if (live) {
      const int d = m >> 1;
      const double sgn = (m & 1) ? -delta : delta;
      const SE3 T = load_T(SPEC ? &Tsh[slot][0] : P.T + 8 * P.epose[e]);
      const double* cam = P.cams + 5 * P.ecam[e];
      const double* obs = obs_of(P, e, t);
      double Lp[6];
      for (int k = 0; k < 6; k++) Lp[k] = SPEC ? cand[einfo_s[slot][3] - gb][k] : Lsh[slot][k];
      double er[4] = {0, 0, 0, 0};
      if (wv == 0) {
        double v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = q == d ? sgn : 0.0;  // static indices: no scratch
        line_oplus(Lp, v);
        edge_error(t, cam, obs, T, Lp, er);
      } else if (wv < 3) {
        double u[6];
#pragma unroll
        for (int q = 0; q < 6; q++) u[q] = q == d - 4 ? sgn : 0.0;
        edge_error(t, cam, obs, se3_mul(se3_exp(u), T), Lp, er);
      } else {
        edge_error(t, cam, obs, T, Lp, er);
      }
      if (m < 20)
        for (int k = 0; k < 4; k++) ev[slot][m][k] = er[k];
      else
        for (int k = 0; k < 4; k++) es[slot][k] = er[k];
    }
  }
  __syncthreads();
  if (stamp && tid == 0) stamp[1] = wall_clock64();
  if (SETUP && tid == 0) {  // the robust cost of the block's edges at the current state, slot order
    double c = 0;
    for (int slot = 0; slot < cnt; slot++) {
      int e, t;
      bool on, live;
      edge(slot, e, t, on, live);
      if (!live) continue;
      double chi2 = 0;
      for (int k = 0; k < edim(t); k++) chi2 += es[slot][k] * es[slot][k];
      chi2 *= einfo(t);
      double cst = chi2;
      if (A.robust) {
        double r1;
        huber(chi2, pick4(P.delta, t), cst, r1);
      }
      c += cst;
    }
    *chi_out = c;
  }
  // J layout per edge: Jp [4][6] at 0, Jl [4][4] at 24 (the analytic path wrote it directly)
  // every J entry of every slot (rows >= edim(t) and slots that are not live: exact zeros), and each
  // slot's robust weight once (SPEC / SETUP: the slot's own error; else the edge's stored one)
  __shared__ double wsh[kLineBlk];
  for (int idx = tid; idx < (P.line_jac ? 0 : 40 * kLineBlk); idx += 256) {
    const int slot = idx / 40, rd = idx - 40 * slot, r = rd / 10, d = rd % 10;
    int e, t;
    bool on, live;
    edge(slot, e, t, on, live);
    const double v = (live && r < edim(t)) ? scal * (ev[slot][2 * d][r] - ev[slot][2 * d + 1][r]) : 0.0;
    if (d < 4) J[slot][24 + r * 4 + d] = v;
    else J[slot][r * 6 + (d - 4)] = v;
  }
  if (tid >= 192 && tid < 192 + kLineBlk) {
    const int slot = tid - 192;
    int e, t;
    bool on, live;
    edge(slot, e, t, on, live);
    const double* er = OWN_ERR ? &es[slot][0] : L.err + 4 * e;
    wsh[slot] = live ? edge_weight_of(P, A, er, t) : 0.0;
  }
  __syncthreads();
  // the 86 contributions per edge (contrib's layout: Hll, bl, Hpp, bp, Hpl), one kind per pass so that
  // a wave never diverges between kinds; four rows unrolled (the rows past edim(t) are zeros and add
  // exact zeros: the same sums, in the same order, as contrib()).  Hpp: the 21 upper entries stored.
  auto rowsum = [&](const double* x, int sx, const double* y, int sy) {
    double t0 = x[0], t1 = x[sx], t2 = x[2 * sx], t3 = x[3 * sx];
    double u0 = y[0], u1 = y[sy], u2 = y[2 * sy], u3 = y[3 * sy];
    double s = 0;
    s += t0 * u0;
    s += t1 * u1;
    s += t2 * u2;
    s += t3 * u3;
    return s;
  };
  auto slot_of = [&](int idx, int per, int& e, int& t, bool& live, bool& popt) {
    const int slot = idx / per;
    bool on;
    edge(slot, e, t, on, live);
    popt = (einfo_s[slot][2] & 4) != 0;
    return on ? slot : -1;
  };
  for (int idx = tid; idx < 20 * kLineBlk; idx += 256) {  // Hll (o < 16), bl
    int e, t;
    bool live, popt;
    const int slot = slot_of(idx, 20, e, t, live, popt);
    if (slot < 0) continue;
    const int o = idx - 20 * slot;
    const double* Jl = &J[slot][24];
    double v;
    if (o < 16) {
      v = live ? wsh[slot] * rowsum(Jl + o / 4, 4, Jl + o % 4, 4) : 0.0;
    } else {
      const double* er = OWN_ERR ? &es[slot][0] : L.err + 4 * e;
      double eb[4];
#pragma unroll
      for (int r = 0; r < 4; r++) eb[r] = r < edim(t) ? er[r] : 0.0;
      v = live ? -wsh[slot] * rowsum(Jl + (o - 16), 4, eb, 1) : 0.0;
    }
    cv[slot][o] = v;
    if (split)
      __hip_atomic_store(o < 16 ? L.Hll + 16 * e + o : L.bl + 4 * e + o - 16, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int idx = tid; idx < 21 * kLineBlk; idx += 256) {  // Hpp, upper triangle (pk6 order)
    int e, t;
    bool live, popt;
    const int slot = slot_of(idx, 21, e, t, live, popt);
    if (slot < 0 || !popt) continue;
    const int q = idx - 21 * slot;
    int a = 0, base = 0;
    while (q >= base + 6 - a) base += 6 - a++;
    const int b = a + (q - base);
    const double* Jp = &J[slot][0];
    L.Hpp[21 * e + q] = live ? wsh[slot] * rowsum(Jp + a, 6, Jp + b, 6) : 0.0;
  }
  for (int idx = tid; idx < 30 * kLineBlk; idx += 256) {  // bp (k < 6), Hpl (6 x 4)
    int e, t;
    bool live, popt;
    const int slot = slot_of(idx, 30, e, t, live, popt);
    if (slot < 0 || !popt) continue;
    const int k = idx - 30 * slot;
    const double* Jp = &J[slot][0];
    if (k < 6) {
      const double* er = OWN_ERR ? &es[slot][0] : L.err + 4 * e;
      double eb[4];
#pragma unroll
      for (int r = 0; r < 4; r++) eb[r] = r < edim(t) ? er[r] : 0.0;
      L.bp[6 * e + k] = live ? -wsh[slot] * rowsum(Jp + k, 6, eb, 1) : 0.0;
    } else {
      const int a = (k - 6) / 4, b = (k - 6) % 4;
      L.Hpl[hpl_off(P.Ep, e) + k - 6] = live ? wsh[slot] * rowsum(Jp + a, 6, &J[slot][24] + b, 4) : 0.0;
    }
  }
  if (SETUP && pdg)  // computeLambdaInit's pose-diagonal partials of this workgroup's edges (slot order), as
                    // the Hpp pass's diagonal entries (pose_diag_range's slots)
    for (int q = tid; q < 6 * A.K; q += 256) {
      const int j = q / 6, i = q - 6 * j;
      double sm = 0;
      for (int slot = 0; slot < cnt; slot++) {
        int e, t;
        bool on, live;
        edge(slot, e, t, on, live);
        if (!(einfo_s[slot][2] & 4) || A.pidx[P.epose[e]] != j) continue;
        const double* Jp = &J[slot][0];
        sm += live ? wsh[slot] * rowsum(Jp + i, 6, Jp + i, 6) : 0.0;
      }
      __hip_atomic_store(pdg + ((size_t)j * pd_nb + pd_b) * 6 + i, sm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (!split) {  // whole landmarks: their blocks from this workgroup's records, CSR (slot) order
    __syncthreads();
    if (tid < 20 * (ge - gb)) {
      const int g = gb + tid / 20, o = tid % 20;
      const int s0 = A.lm_off[g] - p0, s1 = A.lm_off[g + 1] - p0;
      if (s1 > s0) {
        double sm = 0;
        for (int q = s0; q < s1; q++) sm += cv[q][o];
        if (o < 16) S.Hll[16 * g + o] = sm;
        else S.bl[4 * g + o - 16] = sm;
        bool act = !SETUP && A.lm_act[g];
        if (SETUP)
          for (int q = s0; q < s1; q++) act = act || (einfo_s[q][2] & 2);
        if (maxd && o == 0 && act) {  // max |diagonal| of the block, as the ticket path
          double mx = 0;
          for (int dgi = 0; dgi < 16; dgi += 5) {
            double sd = 0;
            for (int q = s0; q < s1; q++) sd += cv[q][dgi];
            mx = fmax(mx, fabs(sd));
          }
          atomic_max_pos(S.out + 2, mx);
        }
      }
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // split landmark, per edge (32 lanes each): ticket; the last edge sums the landmark's records
  {
    const int slot = 2 * wv + (lane >> 5), ln = lane & 31;
    int e, t;
    bool on, live;
    edge(slot, e, t, on, live);
    if (on) {
      const int gl = einfo_s[slot][3], l = gl - P.nq;
      const int k0 = A.lm_off[gl], k1 = A.lm_off[gl + 1];
      unsigned tk = 0;
      if (ln == 0) tk = __hip_atomic_fetch_add(S.lm_ctr + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tk = __shfl(tk, lane & 32);
      if (tk == (unsigned)(k1 - k0 - 1)) {
        if (ln == 0) __hip_atomic_store(S.lm_ctr + l, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        double sm = 0;
        if (ln < 20) {
          const double* base = ln < 16 ? L.Hll + ln : L.bl + (ln - 16);
          const int str = ln < 16 ? 16 : 4;
          for (int k = k0; k < k1; k++)
            sm += __hip_atomic_load(base + (size_t)str * (k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (ln < 16) S.Hll[16 * gl + ln] = sm;
          else S.bl[4 * gl + ln - 16] = sm;
        }
        double mx = (ln < 16 && ln % 5 == 0) ? fabs(sm) : 0.0;
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
        if (maxd && ln == 0 && (SETUP ? line_active(P, L, A, gl, cls) : A.lm_act[gl] != 0)) atomic_max_pos(S.out + 2, mx);
      }
    }
  }
}

// one launch for both landmark families: blocks [0, nbq) point landmarks (kGroup lanes
// each), blocks [nbq, ...) line edges (one wave each).  maxd: contribute the landmark
// diagonals to S.out[2] (computeLambdaInit); speculative passes leave it alone.
__global__ __launch_bounds__(256) void linearize_kernel(Problem P, Lin L, Active A, Sys S, int nbq, int maxd) {
  if ((int)blockIdx.x < nbq) lin_point_landmarks(P, L, A, S, blockIdx.x * 256 + threadIdx.x, maxd != 0);
  else lin_lines<kLinPlain>(P, L, A, S, blockIdx.x - nbq, maxd != 0);
}

// deterministic block reduction of NV values per thread: wave shuffles, then waves in order
template <int NV>
__device__ __forceinline__ void block_reduce(double (&acc)[NV], double* lds /* [nwaves][NV] */) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    acc[i] = wave::xsum64(acc[i]);  // (the xor butterfly's sums, on lane moves)
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; i++) lds[wv * NV + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0;
    for (int w = 0; w < nw; w++) s += lds[w * NV + threadIdx.x];
    lds[threadIdx.x] = s;  // result in lds[0..NV)
  }
  __syncthreads();
}

// max diagonal of the pose blocks (computeLambdaInit), first iteration only.  Block b sums
// the Hpp diagonals of its 256 edges per reduced pose (fixed tree) into partial[a][b]; the
// post kernel sums each pose's partials in block order and takes
// the max.  wt: the partials are written through (read by the last block of the same launch).
__device__ __forceinline__ void pose_diag_block(const Problem& P, const Lin& L, const Active& A, const Sys& S, bool wt) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  int a = -1;
  double d[6] = {0, 0, 0, 0, 0, 0};
  if (e < A.Ea) {
    a = A.pidx[P.epose[e]];
    if (a >= 0) {
      const double* H = L.Hpp + 21 * e;
#pragma unroll
      for (int i = 0; i < 6; i++) d[i] = H[pk6(i, i)];
    }
  }
  // per pose: each wave's butterfly (poses absent from the wave skipped), then the 4 wave sums in
  // wave order -- no block barrier per pose
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ double wsum[4][32][6];
  for (int p0 = 0; p0 < A.K; p0 += 32) {
    const int pn = min(32, A.K - p0);
    for (int j = 0; j < pn; j++) {
      const int pa = p0 + j;
      double acc[6];
#pragma unroll
      for (int i = 0; i < 6; i++) acc[i] = a == pa ? d[i] : 0.0;
      if (__ballot(a == pa)) {  // wave-uniform
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
          for (int i = 0; i < 6; i++) acc[i] += __shfl_xor(acc[i], o);
      }
      if (lane < 6) wsum[wv][j][lane] = acc[lane];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 6 * pn; q += 256) {
      const int j = q / 6, i = q - 6 * j;
      const double v = ((wsum[0][j][i] + wsum[1][j][i]) + wsum[2][j][i]) + wsum[3][j][i];
      double* dst = S.partial2 + ((size_t)(p0 + j) * gridDim.x + blockIdx.x) * 6 + i;
      if (wt) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else *dst = v;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void pose_diag_kernel(Problem P, Lin L, Active A, Sys S) {
  pose_diag_block(P, L, A, S, false);
}

// pose_diag_block over the edge range [e0, e1) (a setup block's own edges, any length; rounds of 256
// summed per wave in round order): partial b of nb into dst[(a * nb + b) * 6 + i], written through.
// The block's record stores must be complete and visible (s_waitcnt + barrier) before the call.
__device__ __forceinline__ void pose_diag_range(const Problem& P, const Lin& L, const Active& A, double* dst, int nb,
                                                int b, int e0, int e1) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ double wsum[4][32][6];
  for (int p0 = 0; p0 < A.K; p0 += 32) {
    const int pn = min(32, A.K - p0);
    for (int j = 0; j < pn; j++)
      if (lane < 6) wsum[wv][j][lane] = 0.0;
    for (int eb = e0; eb < e1; eb += 256) {  // block-uniform
      const int e = eb + threadIdx.x;
      int a = -1;
      double d[6] = {0, 0, 0, 0, 0, 0};
      if (e < e1) {
        a = A.pidx[P.epose[e]];
        if (a >= 0) {
          const double* H = L.Hpp + 21 * e;
#pragma unroll
          for (int i = 0; i < 6; i++) d[i] = H[pk6(i, i)];
        }
      }
      for (int j = 0; j < pn; j++) {
        const int pa = p0 + j;
        double acc[6];
#pragma unroll
        for (int i = 0; i < 6; i++) acc[i] = a == pa ? d[i] : 0.0;
        if (__ballot(a == pa)) {  // wave-uniform
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
            for (int i = 0; i < 6; i++) acc[i] += __shfl_xor(acc[i], o);
        }
        if (lane < 6) wsum[wv][j][lane] += acc[lane];
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 6 * pn; q += 256) {
      const int j = q / 6, i = q - 6 * j;
      const double v = ((wsum[0][j][i] + wsum[1][j][i]) + wsum[2][j][i]) + wsum[3][j][i];
      __hip_atomic_store(dst + ((size_t)(p0 + j) * nb + b) * 6 + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

// pose_diag_range from the per-edge diagonals a landmark block staged in LDS (pd / pa: the block's n CSR edges,
// pose index or -1): wave w sums its quarter of the edges per (pose, entry) in edge order, the four quarters
// then in wave order -- no wait for the block's record stores, no reload
constexpr int kPdCap = 512;  // edges per landmark block staged (more: pose_diag_range)
__device__ __forceinline__ void pose_diag_lds(const Active& A, const double (*pd)[6], const int* pa, int n, double* dst,
                                              int nb, int b) {
  __shared__ double ws[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l0 = (n * wv) / 4, l1 = (n * (wv + 1)) / 4, nq = 6 * A.K;
  for (int q0 = 0; q0 < nq; q0 += 64) {
    const int q = q0 + lane, j = q / 6, i = q - 6 * j;
    double sm = 0;
    if (q < nq)
      for (int l = l0; l < l1; l += 8) {  // eight LDS reads in flight, summed in edge order
        int pv[8];
        double dv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const bool ok = l + u < l1;
          pv[u] = ok ? pa[l + u] : -1;
          dv[u] = ok ? pd[l + u][i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) sm += pv[u] == j ? dv[u] : 0.0;
      }
    ws[wv][lane] = sm;
    __syncthreads();
    if (wv == 0 && q < nq)
      __hip_atomic_store(dst + ((size_t)j * nb + b) * 6 + i, ((ws[0][lane] + ws[1][lane]) + ws[2][lane]) + ws[3][lane],
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------
// Schur complement for damping lambda
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Schur complement for damping lambda
// ---------------------------------------------------------------------------
// Edge-pair lists, built once per call on the device.  Chunk c = (pose pair pr, landmark
// range lb) owns the segment [pp_off[c], pp_off[c+1]) of the (e1, e2) lists; within it the
// pairs follow landmark order, then i, then j (deterministic).  Lane l of round r handles
// landmark lb * lmchunk + 64 r + l; its matches are found from bit masks over batches of 8
// CSR entries (independent loads) and placed by a wave prefix sum in lane order.
template <bool FILL>
__device__ __forceinline__ void pair_scan(const Active& A, int c, int* pp_cnt, const int* pp_off, int4* pp) {
  const int lane = threadIdx.x & 63;
  int pr, g0, g1, nr;
  if (A.dsub <= 1) {  // (every pair nchk ranges of lmchunk)
    pr = c / A.nchk;
    g0 = (c - pr * A.nchk) * A.lmchunk;
    g1 = A.nL;
    nr = A.lmchunk / 64;
  } else {
    const ChunkGeo cg = chunk_geo(A, c);
    pr = cg.pr;
    g0 = cg.g0;
    g1 = cg.g1;
    nr = (cg.g1 - cg.g0 + 63) / 64;
  }
  const int pa = A.pairs[2 * pr], pb = A.pairs[2 * pr + 1];
  int base = FILL ? pp_off[c] : 0;
  // four landmark rounds at a time: their CSR ranges, then the first eight edge poses of each (a landmark's
  // whole edge list when it has <= 8 edges, the common case), every load of a group in flight at once
  for (int r0 = 0; r0 < nr; r0 += 4) {
    int k0[4], k1[4], pz[4][8];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int g = g0 + 64 * (r0 + u) + lane;
      const bool in = r0 + u < nr && g < g1;
      const int o0 = in ? A.lm_off[g] : 0, o1 = in ? A.lm_off[g + 1] : 0;
      const bool act = in && A.lm_act[g];
      k0[u] = act ? o0 : 0;
      k1[u] = act ? o1 : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int v = 0; v < 8; v++) pz[u][v] = k1[u] > k0[u] ? A.lm_pose[min(k0[u] + v, k1[u] - 1)] : -1;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (r0 + u >= nr) break;  // uniform
      const int g = g0 + 64 * (r0 + u) + lane;
      const int e0 = k0[u], e1 = k1[u];
      int cnt = 0;
      unsigned ma1 = 0, mb1 = 0;  // the masks when the landmark has <= 8 edges (one block each)
      if (e1 - e0 <= 8) {
        unsigned ma = 0, mb = 0;
#pragma unroll
        for (int v = 0; v < 8; v++) {
          ma |= (e0 + v < e1 && pz[u][v] == pa) ? 1u << v : 0u;
          mb |= (e0 + v < e1 && pz[u][v] == pb) ? 1u << v : 0u;
        }
        cnt = ma ? __popc(ma) * __popc(mb) : 0;
        ma1 = ma;
        mb1 = mb;
      } else {
        for (int ib = e0; ib < e1; ib += 8) {  // i blocks
          unsigned ma = 0;
          for (int v = 0; v < 8 && ib + v < e1; v++) ma |= A.lm_pose[ib + v] == pa ? 1u << v : 0u;
          if (!ma) continue;
          for (int jb = e0; jb < e1; jb += 8) {  // j blocks
            unsigned mb = 0;
            for (int v = 0; v < 8 && jb + v < e1; v++) mb |= A.lm_pose[jb + v] == pb ? 1u << v : 0u;
            cnt += __popc(ma) * __popc(mb);
          }
        }
      }
      // wave exclusive prefix of the per-lane counts (lane order)
      int pre = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(pre, o);
        if (lane >= o) pre += t;
      }
      const int total = __shfl(pre, 63);
      if (FILL && cnt && e1 - e0 <= 8) {  // emit from the masks: i ascending, then j ascending
        int q = base + pre - cnt;
        for (unsigned ma = ma1; ma; ma &= ma - 1) {
          const int ea = (e0 + __ffs(ma) - 1);
          for (unsigned mb = mb1; mb; mb &= mb - 1) pp[q++] = make_int4(ea, (e0 + __ffs(mb) - 1), g, 0);
        }
      } else if (FILL && cnt) {
        int q = base + pre - cnt;
        for (int ib = e0; ib < e1; ib++) {
          if (A.lm_pose[ib] != pa) continue;
          for (int jb = e0; jb < e1; jb++) {
            if (A.lm_pose[jb] != pb) continue;
            pp[q] = make_int4(ib, jb, g, 0);
            q++;
          }
        }
      }
      base += total;
    }
  }
  if (!FILL && lane == 0) __hip_atomic_store(pp_cnt + c, base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void pair_count_kernel(Active A, int* pp_cnt) {
  pair_scan<false>(A, blockIdx.x, pp_cnt, nullptr, nullptr);
}
__global__ __launch_bounds__(64) void pair_fill_kernel(Active A, const int* pp_off, int4* pp) {
  pair_scan<true>(A, blockIdx.x, nullptr, pp_off, pp);
}
// exclusive scan of the chunk counts (one workgroup; n = npairs * nchk + 1 offsets)
__global__ __launch_bounds__(1024) void pair_offsets_kernel(const int* cnt, int* off, int n) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (n + 1023) / 1024, b0 = min(tid * per, n), b1 = min(b0 + per, n);
  int s = 0;
  for (int i = b0; i < b1; i++) s += cnt[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the partials
    const int t = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += t;
    __syncthreads();
  }
  int run = part[tid] - s;
  for (int i = b0; i < b1; i++) {
    off[i] = run;
    run += cnt[i];
  }
  if (tid == 1023) off[n] = part[1023];
}

// ---------------------------------------------------------------------------
// The first pass of a device-LM optimize() in one launch (was: errors, [classify,
// landmark_active,] linearize, pose_diag, post; build_pairs' count and scan in the first optimize).
//   setup_kernel -- blocks [0, nbq): kGroup lanes per landmark (every landmark).  With `level` (the
//     second optimize) the outlier levels of the landmark's edges from their last computed errors
//     (classify_edge, g2o_optimization.cc:176-213) and its activity (landmark_active); for point
//     landmarks the errors and robust cost at the current state and the linearisation (edge records,
//     Hll / bl, the landmark diagonal maximum).  Blocks [nbq, nbq + n_lblk): the line workgroups
//     (lin_lines<kLinSetup>: classification, cost and linearisation of their own edges).  The cost of
//     block b goes to S.partial[b], its edges' pose-diagonal sums to pdg.  Then the last block of the
//     launch (ticket): the cost, the maximum diagonal and the LM control (computeLambdaInit).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double setup_landmark(const Problem& P, const Lin& L, const Active& A, const Sys& S, int t,
                                                 uint8_t* level, uint8_t* lm_act2, double (*pd)[6] = nullptr,
                                                 int* pa = nullptr, int pe0 = 0) {
  const int g = t / kGroup, j = t % kGroup;
  const bool in = g < A.nL, point = g < P.nq;
  double hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bv[3] = {0, 0, 0}, chi = 0;
  int live = 0;
  if (in) {
    const int k1 = A.lm_off[g + 1];
    const double* Xg = P.X + 3 * g;
    for (int k = A.lm_off[g] + j; k < k1; k += kGroup) {
      bool lev = false;
      if (level && edge_outlier(P, L, k)) {
        lev = true;
        level[k] = 1;
      }
      live |= lev ? 0 : 1;
      if (!point) continue;  // line edges: the line workgroups
      const bool pose_opt = A.lm_pose[k] >= 0;
      if (pd) pa[k - pe0] = pose_opt ? A.lm_pose[k] : -1;  // (the block's edges: its pose-diagonal partials)
      if (lev) {  // outside this phase: exact-zero records, no cost, error kept
        if (pose_opt) zero_pose_records<true>(L, k);
        if (pd)
#pragma unroll
          for (int i = 0; i < 6; i++) pd[k - pe0][i] = 0.0;
        continue;
      }
      const int te = P.etype[k];
      const SE3 T = load_T(P.T + 8 * P.epose[k]);
      const double* cm = P.cams + 5 * P.ecam[k];
      double er[4];
      const double chi2 = point_error(te, cm, obs_of(P, k, te), T, Xg, er);
#pragma unroll
      for (int q = 0; q < 4; q++) L.err[4 * k + q] = er[q];
      double cst = chi2;
      if (A.robust) {
        double r1;
        huber(chi2, pick4(P.delta, te), cst, r1);
      }
      chi += cst;
      double dg6[6] = {0, 0, 0, 0, 0, 0};
      point_edge_core<true>(P, L, A, k, te, pose_opt, T, cm, Xg, er, hl, bv, dg6);
      if (pd)
#pragma unroll
        for (int i = 0; i < 6; i++) pd[k - pe0][i] = dg6[i];
    }
  }
#pragma unroll
  for (int o = 1; o < kGroup; o <<= 1) live |= __shfl_xor(live, o);
  const bool act = level ? live != 0 : (in && A.lm_act[g] != 0);
  if (level && in && j == 0) lm_act2[g] = act ? 1 : 0;
  group_sum(hl);
  group_sum(bv);
  if (in && point && j == 0 && act) {
    double* H = S.Hll + 16 * g;
#pragma unroll
    for (int i = 0; i < 9; i++) H[i] = hl[i];
#pragma unroll
    for (int i = 9; i < 16; i++) H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; i++) S.bl[4 * g + i] = bv[i];
    S.bl[4 * g + 3] = 0.0;
    atomic_max_pos(S.out + 2, fmax(fabs(hl[0]), fmax(fabs(hl[4]), fabs(hl[8]))));
  }
  return chi;
}

__device__ __forceinline__ void prof_stamp(const Sys& S, int slot) {
  if (S.prof) S.prof[slot] = wall_clock64();
}
__device__ __forceinline__ void prof_max(const Sys& S, int slot) {  // latest over the blocks
  if (S.prof) atomicMax(S.prof + slot, (unsigned long long)wall_clock64());
}

// The first pass in ONE launch: blocks [0, nbq) landmark groups, [nbq, nb_lm) line workgroups,
// [nb_lm, ...) pair counting; every landmark / line block then sums the pose diagonals of its own
// edges (pose_diag_range -> pdg) and every block takes a ticket; the last block sums the cost
// partials and the pose-diagonal partials in block order, scans the pair counts and writes the LM
// control (round 3 did this in a second launch; one launch measured neutral, four per call instead of six).
__global__ __launch_bounds__(256) void setup_kernel(Problem P, Lin L, Active A, Sys S, int nbq, int nb_lm,
                                                    uint8_t* level, uint8_t* lm_act2, int* pp_cnt, int* pp_off,
                                                    double* pdg, int lm_iters, int gate, Lin Ls, Sys Ss) {
  __shared__ double red[4];
  __shared__ double part[4][64];
  __shared__ int last;
  if (gate >= 0) {  // queued behind the previous optimize()'s trials: only once it has stopped, on its bank
    const LmCtrl* c = S.lm + gate;
    if (!c->stop) return;
    if (c->cur) {
      bank_state(P);
      bank_lin(L, Ls, S, Ss);
    }
  }
  const int b = blockIdx.x;
  if (b == 0 && threadIdx.x == 0) prof_stamp(S, 9);
  if (b >= nb_lm) {  // the first optimize: edge pairs per Schur chunk, one wave per chunk
    const int c = (b - nb_lm) * 4 + (threadIdx.x >> 6);
    if (c < chunk_count(A)) pair_scan<false>(A, c, pp_cnt, nullptr, nullptr);
    if (threadIdx.x == 0) prof_max(S, kProfX + 4);
  } else if (b >= nbq) {
    double c = 0.0;  // set in thread 0
    lin_lines<kLinSetup>(P, L, A, S, b - nbq, true, nullptr, nullptr, 0.0, false, nullptr, level != nullptr, &c, pdg,
                         nb_lm, b);  // (its edges' pose-diagonal partials too)
    if (threadIdx.x == 0) __hip_atomic_store(S.partial + b, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) prof_max(S, kProfX + 2);
  } else {
    // this block's point landmarks' edges: one CSR range; their pose diagonals staged in LDS when they fit
    __shared__ double pd[kPdCap][6];
    __shared__ int pa[kPdCap];
    const int g0 = min(b * (256 / kGroup), P.nq), g1 = min(b * (256 / kGroup) + 256 / kGroup, P.nq);
    const int e0 = A.lm_off[g0], e1 = A.lm_off[g1];
    const bool staged = e1 - e0 <= kPdCap;
    double acc[1] = {setup_landmark(P, L, A, S, b * 256 + threadIdx.x, level, lm_act2, staged ? pd : nullptr, pa, e0)};
    block_reduce<1>(acc, red);  // (its barriers also order the staged diagonals)
    if (threadIdx.x == 0) __hip_atomic_store(S.partial + b, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) prof_max(S, kProfX + 0);
    if (staged) {
      pose_diag_lds(A, pd, pa, e1 - e0, pdg, nb_lm, b);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      pose_diag_range(P, L, A, pdg, nb_lm, b, e0, e1);
    }
    if (threadIdx.x == 0) prof_max(S, kProfX + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = ticket(S.counter) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // ---- the last block ----
  if (threadIdx.x == 0) prof_stamp(S, 10);
  double cs[1] = {0.0};  // the cost: the landmark / line blocks' partials, fixed order
  for (int k = threadIdx.x; k < nb_lm; k += 256) cs[0] += __hip_atomic_load(S.partial + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  block_reduce<1>(cs, red);
  const double chi2 = red[0];
  if (pp_cnt) {  // exclusive scan of the chunks' edge-pair counts -> pp_off
    __shared__ int sc[256];
    const int tid = threadIdx.x, nc = chunk_count(A);
    const int per = (nc + 255) / 256, b0 = min(tid * per, nc), b1 = min(b0 + per, nc);
    int sm = 0;
    for (int i = b0; i < b1; i++) sm += __hip_atomic_load(pp_cnt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sc[tid] = sm;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
      const int t = tid >= o ? sc[tid - o] : 0;
      __syncthreads();
      sc[tid] += t;
      __syncthreads();
    }
    int run = sc[tid] - sm;
    for (int i = b0; i < b1; i++) {
      pp_off[i] = run;
      run += __hip_atomic_load(pp_cnt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 255) pp_off[nc] = sc[255];
  }
  if (threadIdx.x == 0) prof_stamp(S, 11);
  // per pose and diagonal entry q = 6 pose + i: 4 waves each sum every 4th block partial
  const int lane = threadIdx.x & 63, pt = threadIdx.x >> 6, nq6 = 6 * A.K, npd = nb_lm;
  double mx = 0;
  for (int q0 = 0; q0 < nq6; q0 += 64) {
    const int q = q0 + lane;
    double sacc = 0;
    if (q < nq6) {
      const int pa = q / 6, i = q - 6 * pa;
      const double* src = pdg + (size_t)pa * npd * 6 + i;
      for (int b0 = pt; b0 < npd; b0 += 4 * 16) {  // 16 write-through loads in flight, summed in block order
        double t[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int bb = b0 + 4 * u;
          t[u] = bb < npd ? __hip_atomic_load(src + (size_t)bb * 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) sacc += t[u];
      }
    }
    part[pt][lane] = sacc;
    __syncthreads();
    if (pt == 0 && q < nq6) mx = fmax(mx, fabs(((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]));
    __syncthreads();
  }
  if (pt != 0) return;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (lane != 0) return;
  __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prof_stamp(S, 12);
  // the landmark diagonal maximum (atomic max of the landmark blocks: performed device-coherently)
  const double md = fmax(__hip_atomic_load(S.out + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), mx);
  S.out[0] = chi2;
  S.out[2] = md;
  LmCtrl* ctl = S.lm;  // slot 0: the first trial's (computeLambdaInit: tau = 1e-5 x max diagonal)
  ctl->lambda = 1e-5 * md;
  ctl->ni = 2;
  ctl->chi = chi2;
  ctl->cur = 0;
  ctl->it = 0;
  ctl->qmax = 0;
  ctl->stop = 0;
  ctl->iters = lm_iters;
  ctl->trials = 0;
}

// Schur complement, stage 1: one wave per chunk (pose pair, landmark range) walks its
// segment of the edge-pair lists, forming Y = Hpl_e1 Dinv_g on the fly:
//   [0,36)  [e1==e2] Hpp_e1 - Y Hpl_e2^T,   [36,42) [e1==e2] bp_e1,   [42,48) [e1==e2] Y bl_g
// then the wave sums its 64 lanes in lane order (LDS transpose).

// larger systems, stage 2: one thread per (pose pair, entry) scatters the pair sums.
//   S_ab = [a==b] lambda I + pair sum,  bp_a,  bs_a = bp_a - sum Y bl  (solved in place in x)
__global__ __launch_bounds__(256) void pair_final_kernel(Active A, Sys S, double lambda) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= A.npairs * 42) return;
  const int pr = idx / 42, v = idx - 42 * pr;
  const int a = A.pairs[2 * pr], b = A.pairs[2 * pr + 1], n = 6 * A.K;
  const double s = S.pairfin[48 * pr + v];
  if (v < 36) {
    const int r = v / 6, cc = v - 6 * r;
    const double val = s + ((a == b && r == cc) ? lambda : 0.0);
    S.S[(size_t)(6 * a + r) * n + 6 * b + cc] = val;
    if (a != b) S.S[(size_t)(6 * b + cc) * n + 6 * a + r] = val;
  } else if (a == b) {
    const int r = v - 36;
    S.bp[6 * a + r] = s;
    S.x[6 * a + r] = s - S.pairfin[48 * pr + v + 6];
  }
}

// ---------------------------------------------------------------------------
// Reduced camera system: Schur assembly + dense LDL^T + solve in one 256-thread workgroup,
// matrix in LDS (odd row stride), n = 6K <= kCholLdsMax.
//   assembly: S_ab = [a==b] lambda I + the pair's chunk sum (reduced by its last chunk),
//             written straight into the lower triangle; bp_a alongside, and bs as an extra
//             bordered row n;
//   factor:   blocked by the 6x6 pose blocks, K steps of LDL^T (pivots need a reciprocal
//             only: v_rcp_f64 + Newton, no sqrt / divide chains):
//             (1) wave 0 factors the diagonal block in registers (every lane, uniform),
//             (2) panel rows solve x L_dd^T = a (one lane per row, the rhs row included:
//                 it ends as z = D^-1 L^-1 bs, so there is no forward substitution),
//             (3) rank-6 update of the trailing lower triangle (16x16 thread grid);
//   solve:    backward substitution L^T x = z in wave 0, LDS-resident;
//   poses:    the candidate T <- exp(xp) T and the pose part of the LM scale.
// ---------------------------------------------------------------------------
constexpr int kCholLdsMax = 192;  // packed lower triangle (n+1)(n+2)/2 + 3n + 15 n/6 doubles <= 160 KB of LDS

// packed row-major lower triangle: element (r, c <= r)
__device__ __forceinline__ int pk(int r, int c) { return r * (r + 1) / 2 + c; }

// 1/d to full precision: v_rcp_f64 + two Newton steps (no divide sequence on the chain)
__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

// LDL^T of the 6x6 SPD diagonal block at (c0, c0) of the packed lower triangle Al: unit L
// (strictly-lower, packed row-major into L6), D (d6) and 1/D (r6); false unless every pivot is > 0
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


// pose pair index -> (a, b), a <= b, row-major upper triangle of K poses
__device__ __forceinline__ void pair_of(int pr, int K, int& a, int& b) {
  int base = 0;
  a = 0;
  while (pr >= base + (K - a)) {
    base += K - a;
    a++;
  }
  b = a + (pr - base);
}

__global__ __launch_bounds__(256) void schur_solve_kernel(Problem P, Active A, Sys S, int n, double lambda) {
  extern __shared__ double Al[];     // rows 0..n, packed lower triangle: the matrix + the bordered rhs row n
  __shared__ int bad;
  if (S.lm) {  // device-side LM: damping and bank from the control
    LmView v;
    if (!lm_view(S, v)) return;
    lambda = v.lambda;
    if (v.cur) bank_state(P);
  }
  const int K = n / 6;
  double* z = Al + pk(n, 0);         // row n: bs -> z = D^-1 L^-1 bs -> solution x
  double* rdg = Al + pk(n + 1, 0);   // [n] 1/D
  double* ddg = rdg + n;                    // [n] D
  double* Ldg = ddg + n;                    // [K][15] strictly-lower parts of the (unit) diagonal blocks
  double* bpl = Ldg + 15 * K;               // [n] pose gradient bp (for the LM scale)
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  const int pose_a = tid < P.np ? A.pidx[tid] : -1;  // the pose part of the LM scale (lane = pose)
  if (tid == 0) prof_stamp(S, 0);
  // assembly: every thread issues its pairfin loads (8 at a time) before writing LDS; the
  // fail flag is checked after them (it would otherwise gate every load)
  const int nent = A.npairs * 42;
  for (int q0 = tid; q0 < nent; q0 += 8 * 256) {
    double v1[8], v2[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = q0 + u * 256;
      const int pr = idx / 42, v = idx - 42 * pr;
      v1[u] = idx < nent ? S.pairfin[48 * pr + v] : 0.0;
      v2[u] = (idx < nent && v >= 36) ? S.pairfin[48 * pr + v + 6] : 0.0;
    }
    if (*S.fail) return;  // uniform: a landmark block failed to invert
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = q0 + u * 256;
      if (idx >= nent) break;
      const int pr = idx / 42, v = idx - 42 * pr;
      int pa, pb;
      pair_of(pr, K, pa, pb);
      if (v < 36) {
        const int r = v / 6, cc = v - 6 * r;
        if (pa == pb) {
          if (cc <= r) Al[pk(6 * pa + r, 6 * pa + cc)] = v1[u] + (r == cc ? lambda : 0.0);
        } else {
          Al[pk(6 * pb + cc, 6 * pa + r)] = v1[u];
        }
      } else if (pa == pb) {
        const int r = v - 36;
        bpl[6 * pa + r] = v1[u];
        z[6 * pa + r] = v1[u] - v2[u];
      }
    }
  }
  __syncthreads();
  if (tid == 0) prof_stamp(S, 1);
  // factor: blocked by the 6x6 pose blocks; the rhs row n is factored along (its panel rows
  // become z = D^-1 L^-1 bs: no separate forward substitution)
  const int wv = tid >> 6, lane = tid & 63, fy = tid >> 4, fx = tid & 15;
  for (int s = 0; s < K; s++) {
    const int c0 = 6 * s, r0 = c0 + 6;
    if (wv == 0) {  // (1) diagonal block (every lane, uniform) + (2) panel rows, one per lane
      double L6[15], d6[6], r6[6];
      const bool ok = ldl6(Al, c0, L6, d6, r6);
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 15; q++) Ldg[15 * s + q] = L6[q];
#pragma unroll
        for (int k = 0; k < 6; k++) {
          rdg[c0 + k] = r6[k];
          ddg[c0 + k] = d6[k];
        }
        if (!ok) bad = 1;
      }
      for (int i = r0 + lane; i <= n; i += 64) {  // x = a L_dd^-T D^-1 (unit L: no divides)
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
    __syncthreads();
    if (tid == 0 && s < 2) prof_stamp(S, 5 + 2 * s);  // step s: pivot block + panel done
    if (bad) {  // LDS flag after the barrier: uniform
      if (tid == 0) atomicOr(S.fail, 1);
      return;
    }
    for (int i = r0 + fy; i <= n; i += 16) {  // (3) trailing update A22 -= X D X^T (+ the rhs row)
      double wi[6];
#pragma unroll
      for (int l = 0; l < 6; l++) wi[l] = Al[pk(i, c0 + l)] * ddg[c0 + l];
      const int kmax = min(i, n - 1);
      for (int k = r0 + fx; k <= kmax; k += 16) {
        const double* xk = Al + pk(k, c0);
        double t = Al[pk(i, k)];
#pragma unroll
        for (int l = 0; l < 6; l++) t -= wi[l] * xk[l];
        Al[pk(i, k)] = t;
      }
    }
    __syncthreads();
    if (tid == 0 && s < 2) prof_stamp(S, 6 + 2 * s);  // step s: trailing update done
  }
  if (wv != 0) return;
  if (tid == 0) prof_stamp(S, 2);
  // backward substitution L^T x = z in wave 0 (LDS in program order within the wave)
  for (int s = K - 1; s >= 0; s--) {
    const int c0 = 6 * s;
    double xb[6];
#pragma unroll
    for (int k = 5; k >= 0; k--) {
      double v = z[c0 + k];
#pragma unroll
      for (int l = k + 1; l < 6; l++) v -= Ldg[15 * s + l * (l - 1) / 2 + k] * xb[l];
      xb[k] = v;
    }
    for (int i = lane; i < c0; i += 64) {
      double v = z[i];
#pragma unroll
      for (int l = 0; l < 6; l++) v -= Al[pk(c0 + l, i)] * xb[l];
      z[i] = v;
    }
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 6; k++) z[c0 + k] = xb[k];
  }
  for (int i = lane; i < n; i += 64) S.x[i] = z[i];
  if (tid == 0) prof_stamp(S, 3);
  // the pose part of the LM scale x.(lambda x + bp) (lane = pose; the candidate poses are formed
  // by update_errors_kernel)
  double sc = 0;
  if (lane < P.np && pose_a >= 0)
#pragma unroll
    for (int k = 0; k < 6; k++) sc += z[6 * pose_a + k] * (lambda * z[6 * pose_a + k] + bpl[6 * pose_a + k]);
  sc = wave::xsum64(sc);
  if (lane == 0) S.out[4] = sc;
  if (tid == 0) prof_stamp(S, 4);
}


// ---------------------------------------------------------------------------
// 10 < K <= kRegMaxK (C5's 30-keyframe window, n = 174): rspl::ba::solve_reg (ba_solve_reg.hpp) -- the matrix as
// fp64 MFMA accumulator tiles on SIMDs 1..3, the pivot chain alone on SIMD 0, look-ahead between the two, one
// 768-thread workgroup.  (Replaced the round-5 block-per-thread register kernel: 108 -> 95 us per solve at K = 29 in
// tools/experiments/solve_bench.hip, results within 1e-14 of it.)
// ---------------------------------------------------------------------------
// lane l's double, read by every lane (l uniform)
__device__ __forceinline__ double readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

constexpr int kRegMaxK = kSolveRegMaxK;

struct BaSolveStamp {  // RSPL_BA_PROF slots of the solve (ba.cpp report_prof)
  const Sys& S;
  __device__ void at(int slot) const {
    if (threadIdx.x == 0) prof_stamp(S, slot);
  }
  __device__ void step(int s, int) const {
    if (threadIdx.x == 0 && s < 2) prof_stamp(S, 5 + 2 * s);
  }
  __device__ void wave(int, int) const {}
};

__global__ __launch_bounds__(kSolveRegThreads) void schur_reg_kernel(Problem P, Active A, Sys S, int n, double lambda) {
  extern __shared__ double lds_sr[];
  if (S.lm) {  // device-side LM: damping from the control
    LmView v;
    if (!lm_view(S, v)) return;
    lambda = v.lambda;
  }
  solve_reg(S.pairfin, n / 6, lambda, S.x, S.out + 4, S.fail, A.pidx, P.np, lds_sr, BaSolveStamp{S});
}

// ---------------------------------------------------------------------------
// Reduced camera system for n = 6K <= 60 (K <= kWaveSolveMaxK optimised poses: the C3 window)
// in ONE wavefront, no workgroup barrier.  Lane i owns row i of S in registers (a[0, N): only
// k <= i is meaningful) and the bordered rhs entry z_i.  Right-looking LDL^T column by column:
//   pivot d_j = a_jj by readlane (every lane, uniform), l_ij = a_ij / d_j (lanes i > j),
//   column j's unscaled entries w_kj broadcast through LDS, a_ik -= l_ij w_kj for every k > j
//   (entries above the diagonal are never read), z_i -= l_ij z_j (forward substitution fused);
// then y = D^-1 z and the backward substitution L^T x = y, column i of L read back from LDS into
// registers so the dependent chain is readlane + fma per row.  Assembly reads the pose-pair sums
// (pairfin) straight into the rows; the candidate poses and the pose part of the LM scale follow.
// Returns false (nothing written) when the landmark inversion failed upstream or a pivot is <= 0.
// ---------------------------------------------------------------------------
constexpr int kWaveSolveMaxK = 10;


struct WaveSolveLds {
  double W[2][64][6];  // the panel's unscaled column entries w_ij of row i, double-buffered by block parity
  double Lm[60][61];   // Lm[j][i] = l_ij (column j of L); odd stride
};

// pose pair index of (c, a), c <= a, row-major upper triangle of K poses
__device__ __forceinline__ int pair_index(int c, int a, int K) { return c * K - c * (c - 1) / 2 + (a - c); }

template <int N>
__device__ __forceinline__ void solve_wave(Problem P, const Active& A, const Sys& S, double lambda, WaveSolveLds& w,
                                           bool coherent) {
  constexpr int K = N / 6;
  const int lane = threadIdx.x & 63;
  const int pa = lane / 6, r = lane - 6 * pa;
  const bool row = lane < N;
  auto ld = [&](int idx) {
    return coherent ? __hip_atomic_load(S.pairfin + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : S.pairfin[idx];
  };
  double a[N];
  double z = 0.0, bpl = 0.0;
  {
    const int dg = 48 * pair_index(pa, pa, K);
    // branch-free: every lane issues all N loads (lanes / entries outside the lower triangle read
    // slot 0 and discard it), so the loads go out back to back without exec-mask branches
#pragma unroll
    for (int k = 0; k < N; k++) {
      const int c = k / 6, cc = k - 6 * (k / 6);
      const bool valid = row && k <= lane;  // then c <= pa
      int idx = c == pa ? dg + r * 6 + cc : 48 * pair_index(c, pa, K) + cc * 6 + r;
      idx = valid ? idx : 0;
      const double v = ld(idx);
      a[k] = valid ? v : 0.0;
    }
    if (row) {
      bpl = ld(dg + 36 + r);
      z = bpl - ld(dg + 42 + r);
    }
  }
  const int failed = coherent ? __hip_atomic_load(S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *S.fail;
  if (failed) return;  // uniform: a landmark block failed to invert
  if (lane == 0) prof_stamp(S, 1);
  // damping on the diagonal (a[k] with k == lane: select, static register index)
#pragma unroll
  for (int k = 0; k < N; k++) a[k] += (k == lane) ? lambda : 0.0;
  // Right-looking LDL^T blocked by the 6x6 pose blocks.  Panel b (pivots j = 6b .. 6b + 5): each lane
  // updates its own row's panel entries, the column entries of the panel's later rows broadcast by
  // readlane (no LDS on the pivot chain); then the lane's unscaled panel entries w_ij go to LDS once
  // (one wave_sync per pose block instead of per pivot) and every lane applies the rank-6 update
  // a_ik -= sum_j l_ij w_kj to its later columns k, j ascending -- the same FMAs in the same order as
  // the unblocked elimination.
  bool ok = true;
#pragma unroll
  for (int b = 0; b < K; b++) {
    double l6[6], w6[6];
#pragma unroll
    for (int jj = 0; jj < 6; jj++) {
      const int j = 6 * b + jj;
      const double dj = readlane64(a[j], j);
      ok = ok && dj > 0.0;
      const double rj = rcp64(dj);
      const double wij = a[j];
      const double l = lane > j ? wij * rj : 0.0;
      w6[jj] = wij;
      l6[jj] = l;
      w.Lm[j][lane] = l;
      const double zj = readlane64(z, j);
      z = fma(-l, zj, z);
#pragma unroll
      for (int c = j + 1; c < 6 * b + 6; c++) a[c] = fma(-l, readlane64(wij, c), a[c]);
    }
    if (b + 1 < K) {
#pragma unroll
      for (int jj = 0; jj < 6; jj++) w.W[b & 1][lane][jj] = w6[jj];
      wave_sync();
#pragma unroll
      for (int kb = b + 1; kb < K; kb++) {  // one later pose block (6 columns) at a time
        double wk[6][6];
#pragma unroll
        for (int c = 0; c < 6; c++)
#pragma unroll
          for (int jj = 0; jj < 6; jj++) wk[c][jj] = w.W[b & 1][6 * kb + c][jj];
#pragma unroll
        for (int c = 0; c < 6; c++)
#pragma unroll
          for (int jj = 0; jj < 6; jj++) a[6 * kb + c] = fma(-l6[jj], wk[c][jj], a[6 * kb + c]);
      }
    }
  }
  if (!ok) {
    if (lane == 0) atomicOr(S.fail, 1);
    return;
  }
  if (lane == 0) prof_stamp(S, 2);
  // y = D^-1 z; backward L^T x = y (lane i: y_i -= L_ki x_k for k > i, k descending)
  double dgl = 1.0;
#pragma unroll
  for (int k = 0; k < N; k++) dgl = k == lane ? a[k] : dgl;
  double y = z * rcp64(dgl);
  double lt[N];
#pragma unroll
  for (int k = 0; k < N; k++) lt[k] = row && k > lane ? w.Lm[lane][k] : 0.0;
#pragma unroll
  for (int k = N - 1; k >= 0; k--) {
    const double xk = readlane64(y, k);
    y = fma(-lt[k], xk, y);  // lt[k] == 0 for k <= lane
  }
  const double x = y;
  if (lane == 0) prof_stamp(S, 3);
  if (row) S.x[lane] = x;
  // the pose part of the LM scale x.(lambda x + bp) (the candidate poses: update_errors_kernel)
  double sc = row ? x * (lambda * x + bpl) : 0.0;
  sc = wave::xsum64(sc);
  if (lane == 0) S.out[4] = sc;
}

// standalone single-wave solve (sharded path: after the pairfin all-reduce)
template <int N>
__global__ __launch_bounds__(64) void schur_wave_kernel(Problem P, Active A, Sys S, double lambda) {
  __shared__ WaveSolveLds w;
  if (S.lm) {
    LmView v;
    if (!lm_view(S, v)) return;
    lambda = v.lambda;
    if (v.cur) bank_state(P);
  }
  solve_wave<N>(P, A, S, lambda, w, false);
}

// one edge pair's Schur terms with D = (Hll_g + lambda I)^-1, landmark dimension LD (3: points, 4: lines
// or a mixed range; 6 x 4 operands, the 4th column of a point's Hpl is zero): Y = Hpl_e1 D,
// acc -= Y Hpl_e2^T; diag (e1 == e2) adds Hpp_e1, bp_e1 and Y bl_g.  LOWER (a diagonal pose pair):
// only the block's lower triangle (cc <= r) -- the only part any solver reads of a diagonal block.
// Same products in the same order as the zero-padded 4-dim form.
template <int LD, bool LOWER>
__device__ __forceinline__ void schur_pair(const double (&H1)[6 * LD], const double (&B)[6 * LD], bool diag,
                                           const double (&Hp)[21], const double (&bpv)[6], const double (&blv)[LD],
                                           const double (&D)[LD * LD], double (&acc)[48]) {
#pragma unroll
  for (int r = 0; r < 6; r++) {
    double y[LD];
#pragma unroll
    for (int q = 0; q < LD; q++) {
      double t = H1[r * LD] * D[q];
#pragma unroll
      for (int c = 1; c < LD; c++) t += H1[r * LD + c] * D[c * LD + q];
      y[q] = t;
    }
#pragma unroll
    for (int cc = 0; cc < (LOWER ? r + 1 : 6); cc++) {
      double t = y[0] * B[cc * LD];
#pragma unroll
      for (int q = 1; q < LD; q++) t += y[q] * B[cc * LD + q];
      acc[r * 6 + cc] -= t;
    }
    if (LOWER && diag) {
#pragma unroll
      for (int cc = 0; cc <= r; cc++) acc[r * 6 + cc] += Hp[pk6(cc, r)];
      acc[36 + r] += bpv[r];
      double t = y[0] * blv[0];
#pragma unroll
      for (int q = 1; q < LD; q++) t += y[q] * blv[q];
      acc[42 + r] += t;
    }
  }
}

// A chunk's walk over its edge-pair segment [beg, end), lane-strided, software-pipelined: the pair
// indices two passes ahead and every operand of the next pass are requested before this pass's
// arithmetic (ping-pong operand sets), so a wave waits on one memory round trip per segment rather than
// per pass.  LD 3: a range of point landmarks only (3x3 D, 6x3 Hpl); 4: a range holding lines.  LOWER: a
// diagonal pose pair (e1 == e2 pairs add Hpp / bp / Y bl; lower triangle only).
// Register budget: only the off-diagonal point chunks (most of them) keep the PairOps operand set; the
// diagonal chunks take e1 == e2 without a copy of H1, and line ranges invert the landmark block before
// their edge operands are requested, so the kernel fits 256 VGPRs with no AGPRs (was 255 + 52): a
// chunk wave then fits on a SIMD beside one front-end wave (a fp16 conv or GNN layer wave, <= 224
// registers) instead of waiting for the SIMD to drain.  The same FMAs in the same order as before.
template <int LD>
struct PairOps {
  double D[LD * LD], H1[6 * LD], H2[6 * LD], Hp[21], bpv[6], blv[LD];  // D: Hll of the landmark
  bool diag, live, pt;
};

template <int LD, bool LOWER>
__device__ __forceinline__ void load_pair(const Lin& L, const Active& A, const Sys& S, int nq, int4 q,
                                          PairOps<LD>& o) {
  static_assert(!LOWER && LD == 3, "off-diagonal pose pairs of point ranges only (chunk_loop takes the others)");
  const int e1 = q.x, e2 = q.y, g = q.z;
  o.diag = false;
  o.live = !(A.elevel && (A.elevel[e1] | A.elevel[e2]));  // else zero records: no contribution
  const double* dg = S.Hll + 16 * g;  // the landmark block (inverted in use_pair)
#pragma unroll
  for (int i = 0; i < LD * LD; i++) o.D[i] = dg[i];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c < LD; c++) {
      o.H1[r * LD + c] = L.Hpl[18 * e1 + r * 3 + c];
      o.H2[r * LD + c] = L.Hpl[18 * e2 + r * 3 + c];
    }
  o.pt = g < nq;
}

template <int LD, bool LOWER>
__device__ __forceinline__ void use_pair(const PairOps<LD>& o, double lambda, bool& bad, double (&acc)[48]) {
  if (!o.live) return;
  double D[LD * LD];  // (Hll + lambda I)^-1 (Gauss-Jordan, partial pivoting; points 3x3, lines 4x4)
  if constexpr (LD == 3) {
    double Hd[9];
#pragma unroll
    for (int i = 0; i < 9; i++) Hd[i] = o.D[i] + ((i % 4 == 0) ? lambda : 0.0);
    bad |= !small_inv<3>(Hd, D);
  } else {
    bad |= !lm_dinv(o.D, o.pt, lambda, D);
  }
  // one call site with B = H2 (a copy of H1 on the diagonal): two call sites on H1 / H2 were merged
  // by the compiler into one through a selected pointer, which put both arrays in scratch memory
  schur_pair<LD, LOWER>(o.H1, o.H2, o.diag, o.Hp, o.bpv, o.blv, D, acc);
}

template <int LD, bool LOWER>
__device__ __forceinline__ void chunk_loop(const Problem& P, const Lin& L, const Active& A, const Sys& S,
                                           const DiagPose& dp, int nq, int beg, int end, int4 qn, double lambda,
                                           bool& bad, double (&acc)[48]) {
  const int lane = threadIdx.x & 63;
  for (int k = beg + lane; k < end; k += 64) {
    const int4 q = qn;
    if (k + 64 < end) qn = A.pp[k + 64];
    if constexpr (LD == 4 && LOWER) {
      // diagonal pose pairs over line ranges (a few chunks per trial): the landmark inverse first, the
      // edge operands after it (no operand in flight across the 4x4 Gauss-Jordan) -- this path otherwise
      // sets the kernel's register budget above 256 (one wave per SIMD, none beside a front-end wave)
      const int e1 = q.x, e2 = q.y, g = q.z;
      const bool live = !(A.elevel && (A.elevel[e1] | A.elevel[e2]));
      double Hd[16], D[16];
#pragma unroll
      for (int i = 0; i < 16; i++) Hd[i] = S.Hll[16 * g + i];
      bad |= live && !lm_dinv(Hd, g < nq, lambda, D);
      asm volatile("" ::: "memory");
      if (live && e1 == e2) {  // the edge with itself: H1 twice, + Hp / bp / Y bl
        double H1[24], Hp[21], bpv[6], blv[4];
        // a point edge's pose block from the state (point_pose_block; its operands requested with H1 at
        // clamped addresses), a line edge's from its records
        const bool pt = g < nq;
        const int te = P.etype[e1], ci = P.ecam[e1];
        const double* obp = pt ? P.eobs + 4 * e1 : P.eobs;
        const double* xgp = pt ? P.X + 3 * g : P.cams;
        const double ob[3] = {obp[0], obp[1], obp[2]}, Xg[3] = {xgp[0], xgp[1], xgp[2]};
        load_hpl4(L.Hpl, P.Ep, e1, H1);
#pragma unroll
        for (int i = 0; i < 4; i++) blv[i] = S.bl[4 * g + i];
        if (pt) {
          point_pose_block(P, A, te, dp.pose, dp.cams + 5 * ci, ob, Xg, Hp, bpv);
        } else {
#pragma unroll
          for (int i = 0; i < 21; i++) Hp[i] = L.Hpp[21 * e1 + i];
#pragma unroll
          for (int i = 0; i < 6; i++) bpv[i] = L.bp[6 * e1 + i];
        }
        schur_pair<LD, LOWER>(H1, H1, true, Hp, bpv, blv, D, acc);
      } else if (live) {  // two edges of one landmark on the same pose (rare)
        double H1[24], H2[24], Hp[21], bpv[6], blv[4];
        load_hpl4(L.Hpl, P.Ep, e1, H1);
        load_hpl4(L.Hpl, P.Ep, e2, H2);
        schur_pair<LD, LOWER>(H1, H2, false, Hp, bpv, blv, D, acc);
      }
    } else if constexpr (LD == 4) {  // off-diagonal pose pairs over line ranges: the inverse first as well
      const int e1 = q.x, e2 = q.y, g = q.z;
      const bool live = !(A.elevel && (A.elevel[e1] | A.elevel[e2]));
      double Hd[16], D[16];
#pragma unroll
      for (int i = 0; i < 16; i++) Hd[i] = S.Hll[16 * g + i];
      bad |= live && !lm_dinv(Hd, g < nq, lambda, D);
      asm volatile("" ::: "memory");
      if (live) {
        double H1[24], H2[24], Hp[21], bpv[6], blv[4];
        load_hpl4(L.Hpl, P.Ep, e1, H1);
        load_hpl4(L.Hpl, P.Ep, e2, H2);
        schur_pair<LD, LOWER>(H1, H2, false, Hp, bpv, blv, D, acc);
      }
    } else if constexpr (LOWER) {  // diagonal pose pairs over point ranges: e1 == e2 without an H2 copy
      // every operand in one round trip, unconditionally (the edge's pose block is formed from the state by
      // point_pose_block: the pose and cameras in dp, the edge's type / camera / observation and the point
      // requested here with the records)
      const int e1 = q.x, e2 = q.y, g = q.z;
      const bool live = !(A.elevel && (A.elevel[e1] | A.elevel[e2]));
      double Hd[9], D[9], H1[18], Hp[21], bpv[6], blv[3], ob[3], Xg[3];
#pragma unroll
      for (int i = 0; i < 9; i++) Hd[i] = S.Hll[16 * g + i];
#pragma unroll
      for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) H1[r * 3 + c] = L.Hpl[18 * e1 + r * 3 + c];
      const int te = P.etype[e1], ci = P.ecam[e1];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        blv[i] = S.bl[4 * g + i];
        ob[i] = P.eobs[4 * e1 + i];
        Xg[i] = P.X[3 * g + i];
      }
      if (live) {
#pragma unroll
        for (int i = 0; i < 9; i++) Hd[i] += (i % 4 == 0) ? lambda : 0.0;
        bad |= !small_inv<3>(Hd, D);
        if (e1 == e2) {
          point_pose_block(P, A, te, dp.pose, dp.cams + 5 * ci, ob, Xg, Hp, bpv);
          schur_pair<LD, LOWER>(H1, H1, true, Hp, bpv, blv, D, acc);
        } else {
          double H2[18];
#pragma unroll
          for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) H2[r * 3 + c] = L.Hpl[18 * e2 + r * 3 + c];
          schur_pair<LD, LOWER>(H1, H2, false, Hp, bpv, blv, D, acc);
        }
      }
    } else {
      PairOps<LD> o;
      load_pair<LD, LOWER>(L, A, S, nq, q, o);
      use_pair<LD, LOWER>(o, lambda, bad, acc);
    }
  }
}

// One Schur chunk (pose pair, landmark range) on one wave: walks its segment of the edge-pair
// lists, sums its 64 lanes in lane order (LDS transpose in red[64 * 49], this wave's own) and hands
// the partial off write-through to whichever chunk of the pose pair finishes last; that one sums the
// pair's chunks in chunk order (deterministic) into pairfin (write-through when `wt`: a solver in the
// same launch reads it).  vb is the chunk's virtual workgroup id (XCD-aware order).  Returns true in
// the wave that completed a pose pair.
// The chunk of virtual workgroup vb and its pair-list segment (bank-independent: requested before the
// LM control is read).  XCD-aware chunk order: workgroups go round-robin over the 8 XCDs (blockIdx % 8),
// so landmark range lb runs on XCD lb % 8 for every pose pair -- each XCD's L2 then holds only its
// ranges' records (~1/8 of them), which its ~k_g pose pairs per landmark re-read.
struct ChunkSeg {
  int c, lb, beg, end;
  int pr, c0, c1;  // its pose pair and that pair's chunks
  bool pts;        // a range of point landmarks only
  int4 q0;         // the lane's first pair
};
__device__ __forceinline__ bool chunk_seg(const Active& A, int nq, int vb, ChunkSeg& cs) {
  const int lane = threadIdx.x & 63;
  if (A.nchk >= 8) {  // (dsub == 1)
    const int xcd = vb & 7, slot = vb >> 3, rpx = (A.nchk + 7) >> 3;
    cs.lb = (slot % rpx) * 8 + xcd;
    cs.pr = slot / rpx;
    if (cs.lb >= A.nchk || cs.pr >= A.npairs) return false;
    cs.c = cs.pr * A.nchk + cs.lb;
    cs.c0 = cs.pr * A.nchk;
    cs.c1 = cs.c0 + A.nchk;
    cs.pts = (cs.lb + 1) * A.lmchunk <= nq;
  } else {  // fewer ranges than XCDs (many pose pairs, wide chunks): plain order, every XCD busy
    if (vb >= chunk_count(A)) return false;
    cs.c = vb;
    const ChunkGeo cg = chunk_geo(A, cs.c);
    cs.lb = cg.lb;
    cs.pr = cg.pr;
    cs.c0 = cg.c0;
    cs.c1 = cg.c1;
    cs.pts = cg.gend <= nq;
  }
  cs.beg = A.pp_off[cs.c];
  cs.end = A.pp_off[cs.c + 1];
  cs.q0 = cs.beg + lane < cs.end ? A.pp[cs.beg + lane] : make_int4(0, 0, 0, 0);
  return true;
}

__device__ __forceinline__ bool chunk_wave(const Problem& P, const Lin& L, const Active& A, const Sys& S,
                                           double lambda, const ChunkSeg& cs, double* red, bool wt) {
  const int lane = threadIdx.x & 63;
  const int c = cs.c, beg = cs.beg, end = cs.end;
  if (lane == 0 && c < 4096) prof_stamp(S, kProfPc + 4 * c);
  const int pr = cs.pr;
  double acc[48];
#pragma unroll
  for (int v = 0; v < 48; v++) acc[v] = 0.0;
  // a range of point landmarks only
  // (all but the last range or two) takes the 3-dim loops, off-diagonal pose pairs without the e1 == e2 terms
  const bool pts = cs.pts;
  const int pa = A.pairs[2 * pr];
  const bool dpp = pa == A.pairs[2 * pr + 1];
  DiagPose dp;
  if (dpp) {  // a diagonal pose pair: its pose's rotation / translation and the cameras, in this wave's LDS
    const unsigned long long m = __ballot(lane < P.np && A.pidx[lane] == pa);
    if (lane == 0) {
      const SE3 T = load_T(P.T + 8 * (__ffsll((long long)m) - 1));
      double R[9];
      q_to_R(T.q, R);
#pragma unroll
      for (int i = 0; i < 9; i++) red[i] = R[i];
#pragma unroll
      for (int i = 0; i < 3; i++) red[9 + i] = T.t[i];
    }
    for (int i = lane; i < 5 * P.ncam; i += 64) red[12 + i] = P.cams[i];
    dp.pose = red;
    dp.cams = red + 12;
    wave_sync();
  }
  bool bad = false;
  if (pts && !dpp) chunk_loop<3, false>(P, L, A, S, dp, P.nq, beg, end, cs.q0, lambda, bad, acc);
  else if (pts) chunk_loop<3, true>(P, L, A, S, dp, P.nq, beg, end, cs.q0, lambda, bad, acc);
  else if (!dpp) chunk_loop<4, false>(P, L, A, S, dp, P.nq, beg, end, cs.q0, lambda, bad, acc);
  else chunk_loop<4, true>(P, L, A, S, dp, P.nq, beg, end, cs.q0, lambda, bad, acc);
  if (bad) atomicOr(S.fail, 1);
  wave_sync();  // (the cameras' LDS reads before the transpose below overwrites them)
  if (lane == 0 && c < 4096) prof_stamp(S, kProfPc + 4 * c + 1);
#pragma unroll
  for (int v = 0; v < 48; v++) red[lane * 49 + v] = acc[v];
  wave_sync();
  if (lane < 48) {  // 8 independent partial sums, combined in a fixed order
    double p8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int l = 0; l < 64; l++) p8[l & 7] += red[l * 49 + lane];
    const double s = ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
    __hip_atomic_store(S.chunk + 48 * c + lane, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int c0 = cs.c0, c1 = cs.c1;
  unsigned tk = 0;
  if (lane == 0) tk = __hip_atomic_fetch_add(S.pair_ctr + pr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tk = __shfl(tk, 0);
  if (tk != (unsigned)(c1 - c0 - 1)) {
    if (lane == 0 && c < 4096) prof_stamp(S, kProfPc + 4 * c + 2);
    return false;
  }
  if (lane == 0) __hip_atomic_store(S.pair_ctr + pr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane < 48) {
    double s = 0;
    for (int cb = c0; cb < c1; cb += 16) {  // 16 write-through loads in flight, summed in chunk order
      double t[16];
#pragma unroll
      for (int u = 0; u < 16; u++)
        t[u] = cb + u < c1 ? __hip_atomic_load(S.chunk + 48 * (cb + u) + lane, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
#pragma unroll
      for (int u = 0; u < 16; u++) s += t[u];
    }
    if (wt) __hip_atomic_store(S.pairfin + 48 * pr + lane, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else S.pairfin[48 * pr + lane] = s;
  }
  if (lane == 0 && c < 4096) prof_stamp(S, kProfPc + 4 * c + 3);
  return true;
}

// second ticket over the pose pairs (re-armed by its winner): true in the wave that finished the
// last pose pair -- every pair sum is then out (write-through)
__device__ __forceinline__ bool last_pair(const Sys& S, int npairs) {
  const int lane = threadIdx.x & 63;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned tp = 0;
  if (lane == 0) tp = __hip_atomic_fetch_add(S.solve_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tp = __shfl(tp, 0);
  if (tp != (unsigned)(npairs - 1)) return false;
  if (lane == 0) __hip_atomic_store(S.solve_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// N > 0 (6K <= 60): the pose pair finished last solves the reduced system in the same wave
// (solve_wave<N>), so the trial needs no separate solve launch.
template <int N>
__global__ __launch_bounds__(64) void pair_chunk_kernel(Problem P, Lin L, Active A, Sys S, double lambda, Lin Ls,
                                                        Sys Ss) {
  constexpr int kRedLen = 64 * 49, kSolveLen = (int)(sizeof(WaveSolveLds) / sizeof(double));
  __shared__ double smem[N > 0 && kSolveLen > kRedLen ? kSolveLen : kRedLen];
  ChunkSeg cs;
  if (!chunk_seg(A, P.nq, blockIdx.x, cs)) return;  // in flight while the control is read
  if (S.lm) {  // device-side LM: damping and bank from the control
    LmView v;
    if (!lm_view(S, v)) return;
    lambda = v.lambda;
    if (v.cur) {  // (the state too: the diagonal chunks form their point edges' pose blocks from it)
      bank_lin(L, Ls, S, Ss);
      bank_state(P);
    }
  }
  if (!chunk_wave(P, L, A, S, lambda, cs, smem, N > 0)) return;
  if constexpr (N > 0) {
    if (!last_pair(S, A.npairs)) return;
    wave_sync();  // red[] is dead: the LDS becomes the solver's
    if (threadIdx.x == 0) prof_stamp(S, 0);
    solve_wave<N>(P, A, S, lambda, *reinterpret_cast<WaveSolveLds*>(smem), true);
    if (threadIdx.x == 0) prof_stamp(S, 4);
  }
}


// larger systems: one workgroup on global memory

__global__ __launch_bounds__(256) void cholesky_kernel(Sys S, int n) {
  __shared__ double red[256];
  __shared__ int bad;
  double* A = S.S;
  double* x = S.x;
  const int tid = threadIdx.x;
  if (tid == 0) bad = *S.fail;
  __syncthreads();
  if (bad) return;
  for (int j = 0; j < n; j++) {
    if (tid == 0) {
      const double v = A[(size_t)j * n + j];
      if (!(v > 0)) bad = 1;
      else A[(size_t)j * n + j] = sqrt(v);
    }
    __syncthreads();
    if (bad) {
      if (tid == 0) atomicOr(S.fail, 1);
      return;
    }
    const double d = A[(size_t)j * n + j];
    for (int i = j + 1 + tid; i < n; i += 256) A[(size_t)i * n + j] /= d;
    __syncthreads();
    const int m = n - j - 1;
    for (int idx = tid; idx < m * m; idx += 256) {
      const int i = j + 1 + idx / m, k = j + 1 + idx % m;
      if (k <= i) A[(size_t)i * n + k] -= A[(size_t)i * n + j] * A[(size_t)k * n + j];
    }
    __syncthreads();
  }
  for (int i = 0; i < n; i++) {
    double s = 0;
    for (int k = tid; k < i; k += 256) s += A[(size_t)i * n + k] * x[k];
    red[tid] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (tid < st) red[tid] += red[tid + st];
      __syncthreads();
    }
    if (tid == 0) x[i] = (x[i] - red[0]) / A[(size_t)i * n + i];
    __syncthreads();
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = 0;
    for (int k = i + 1 + tid; k < n; k += 256) s += A[(size_t)k * n + i] * x[k];
    red[tid] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (tid < st) red[tid] += red[tid + st];
      __syncthreads();
    }
    if (tid == 0) x[i] = (x[i] - red[0]) / A[(size_t)i * n + i];
    __syncthreads();
  }
}

// Back-substitution xl = Dinv (bl - sum_e Hpl_e^T xp) fused with the candidate state
// (poses T <- exp(xp) T, points += xl, lines oplus(xl); inactive vertices copied: ping-pong
// buffers) and the LM scale x.(lambda x + b) per block.
__global__ __launch_bounds__(256) void update_kernel(Problem P, Lin L, Active A, Sys S, double lambda) {
  __shared__ double red[256];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool failed = *S.fail != 0;
  double sc = 0;
  if (i < P.np) {
    const double* Tp = P.T + 8 * i;
    double* Tq = P.Tn + 8 * i;
    const int a = A.pidx[i];
    if (a >= 0 && !failed) {
      const double* xp = S.x + 6 * a;
      const SE3 r = se3_mul(se3_exp(xp), load_T(Tp));
      for (int k = 0; k < 4; k++) Tq[k] = r.q[k];
      for (int k = 0; k < 3; k++) Tq[4 + k] = r.t[k];
      Tq[7] = 0;
      if (S.pose_scale)
        for (int k = 0; k < 6; k++) sc += xp[k] * (lambda * xp[k] + S.bp[6 * a + k]);
    } else {
      for (int k = 0; k < 8; k++) Tq[k] = Tp[k];
    }
  } else if (i < P.np + P.nq + P.nl) {
    const int g = i - P.np;
    const bool point = g < P.nq;
    const bool upd = A.lm_act[g] && !failed;
    double xl[4] = {0, 0, 0, 0};
    if (upd) {
      double c[4];
      for (int k = 0; k < 4; k++) c[k] = S.bl[4 * g + k];
      const int k0 = A.lm_off[g], k1 = A.lm_off[g + 1];
      for (int kb = k0; kb < k1; kb += 4) {
        int es[4], as[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int k = min(kb + u, k1 - 1);
          es[u] = (k);
          as[u] = kb + u < k1 ? A.lm_pose[k] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          double B[24];
          load_hpl4(L.Hpl, P.Ep, es[u], B);
          const double* xp = S.x + 6 * max(as[u], 0);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            double s = 0;
#pragma unroll
            for (int r = 0; r < 6; r++) s += B[r * 4 + j] * xp[r];
            c[j] -= as[u] >= 0 ? s : 0.0;
          }
        }
      }
      double D[16];
      if (!lm_dinv(S.Hll + 16 * g, point, lambda, D)) atomicOr(S.fail, 1);
#pragma unroll
      for (int r = 0; r < 4; r++) xl[r] = D[r * 4] * c[0] + D[r * 4 + 1] * c[1] + D[r * 4 + 2] * c[2] + D[r * 4 + 3] * c[3];
#pragma unroll
      for (int k = 0; k < 4; k++) sc += xl[k] * (lambda * xl[k] + S.bl[4 * g + k]);
    }
    if (point) {
      for (int k = 0; k < 3; k++) P.Xn[3 * g + k] = P.X[3 * g + k] + xl[k];
    } else {
      const int l = g - P.nq;
      double Lv[6];
      for (int k = 0; k < 6; k++) Lv[k] = P.L[6 * l + k];
      if (upd) line_oplus(Lv, xl);
      for (int k = 0; k < 6; k++) P.Ln[6 * l + k] = Lv[k];
    }
  }
  const double s = block_sum256(sc, red);
  if (threadIdx.x == 0) S.partial2[blockIdx.x] = s;
}

// Fast-path trial tail (after schur_solve has written the candidate poses and the pose
// part of the scale): per landmark a group of kGroup lanes does the back-substitution
// xl = Dinv (bl - sum_e Hpl_e^T xp) (edges split over the lanes, group sum), the candidate
// landmark (points += xl, lines oplus; copied when inactive: ping-pong), the scale term, and
// then the robust cost of the landmark's edges against the candidate poses.  The last block
// (ticket) sums the block partials in order and posts {chi2, scale, maxdiag, fail} + seq.
// Spec: the speculative linearisation of the candidate fused into update_errors_kernel
// (records into the spare set Ls / Ss).  Blocks [0, nbu) are the landmark groups: besides the
// update and the errors, a point group linearises its landmark's edges at the candidate from
// the errors in its registers, and a line group writes the candidate line.  Blocks [nbu, ...) are
// line-edge workgroups (lin_lines<kLinSpec>) that form their landmarks' candidates themselves, so
// they run from the kernel's start.  The mailbox ticket counts only the group blocks, so the
// host decides while the line workgroups still run.
template <bool SPEC>
__global__ __launch_bounds__(256) void update_errors_kernel(Problem P, Lin L, Active A, Sys S, double lambda,
                                                            unsigned long long seq, Lin Ls, Sys Ss, int nbu) {
  __shared__ double red[4 * 2];
  __shared__ int last;
  const bool stamp = threadIdx.x == 0 && blockIdx.x < 4096;
  if (stamp) prof_stamp(S, kProfUe + 4 * blockIdx.x);
  bool spec = SPEC;  // the candidate's speculative linearisation (device LM: not in the last iteration)
  if (SPEC && (int)blockIdx.x >= nbu) {  // line workgroups
    if (S.lm) {
      LmView v;
      if (!lm_view(S, v)) return;
      lambda = v.lambda;
      spec = v.spec;
      if (v.cur) {
        bank_state(P);
        bank_lin(L, Ls, S, Ss);
      }
    }
    if (!spec) return;
    lin_lines<kLinSpec>(P, Ls, A, Ss, blockIdx.x - nbu, false, &L, &S, lambda, *S.fail != 0,
                    S.prof ? S.prof + kProfUe + 4 * blockIdx.x + 1 : nullptr);
    if (stamp) prof_stamp(S, kProfUe + 4 * blockIdx.x + 3);
    return;
  }
  if (!SPEC) nbu = gridDim.x;
  // the candidate poses, cameras and pose steps of this trial go to LDS once per block, in the same
  // round trip as each group's landmark-only operands; the group's first edge per lane is fetched
  // in the next (every later access to them is LDS or registers: two dependent round trips).  The
  // landmark-only operands of BOTH banks are requested before the LM control is read (the control
  // picks the current bank), so that read is not a round trip of its own.
  __shared__ double sT[64 * 8], scam[16 * 5], sx[6 * 32];
  const int tid = threadIdx.x;
  // kUeWaves of the 4 waves carry landmark groups: fewer landmarks per workgroup spread the groups over
  // more CUs (the others only stage the block's poses and take part in the barriers)
  // the landmark block: with A.ue_bpr the workgroups of Schur chunk range lb (its lmchunk landmarks) go to
  // the XCD that ran the range's chunks (lb % 8, chunk_seg): their records are in that XCD's L2
  int ub = blockIdx.x;
  if (SPEC && A.ue_bpr > 0) {
    const int b = blockIdx.x, x = b & 7, sl = b >> 3, r = sl / A.ue_bpr, lb = 8 * r + x;
    constexpr int per = 64 * kUeWaves / kGroup;  // landmarks per workgroup (as set_update_geometry)
    ub = lb < A.nchk ? lb * A.ue_bpr + (sl - r * A.ue_bpr) : (A.nL + per - 1) / per + 1;  // (else: no landmark)
  }
  const int t = ub * (64 * kUeWaves) + tid, g = t / kGroup, j = t % kGroup;
  const bool in = tid < 64 * kUeWaves && g < A.nL;
  const bool point = g < P.nq;
  int k0 = 0, k1 = 0;
  bool act = false;
  double dl[16], blg[4], lm[6] = {0, 0, 0, 0, 0, 0};  // dl: Hll of the landmark (inverted below)
  double dl2[16], blg2[4], lm2[6] = {0, 0, 0, 0, 0, 0};  // the other bank's
#pragma unroll
  for (int q = 0; q < 16; q++) dl[q] = dl2[q] = 0.0;
#pragma unroll
  for (int q = 0; q < 4; q++) blg[q] = blg2[q] = 0.0;
  if (in) {
    k0 = A.lm_off[g];
    k1 = A.lm_off[g + 1];
    act = A.lm_act[g] != 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      dl[q] = point && q >= 9 ? 0.0 : S.Hll[16 * g + q];
      dl2[q] = point && q >= 9 ? 0.0 : Ss.Hll[16 * g + q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      blg[q] = S.bl[4 * g + q];
      blg2[q] = Ss.bl[4 * g + q];
    }
    if (point) {
#pragma unroll
      for (int q = 0; q < 3; q++) {
        lm[q] = P.X[3 * g + q];
        lm2[q] = P.Xn[3 * g + q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        lm[q] = P.L[6 * (g - P.nq) + q];
        lm2[q] = P.Ln[6 * (g - P.nq) + q];
      }
    }
  }
  if (S.lm) {
    LmView v;
    if (!lm_view(S, v)) {  // stopped: carry the control over to the next trial's slot
      if (blockIdx.x == 0 && threadIdx.x == 0) S.lm[S.lm_slot ^ 1] = S.lm[S.lm_slot];
      return;
    }
    lambda = v.lambda;
    spec = SPEC && v.spec;
    if (v.cur) {
      bank_state(P);
      bank_lin(L, Ls, S, Ss);
#pragma unroll
      for (int q = 0; q < 16; q++) dl[q] = dl2[q];
#pragma unroll
      for (int q = 0; q < 4; q++) blg[q] = blg2[q];
#pragma unroll
      for (int q = 0; q < 6; q++) lm[q] = lm2[q];
    }
  }
  const bool failed = *S.fail != 0;
  for (int q = tid; q < 5 * P.ncam; q += 256) scam[q] = P.cams[q];
  for (int q = tid; q < 6 * A.K; q += 256) sx[q] = S.x[q];
  // the lane's first edge (most landmarks have <= kGroup edges): everything it needs in one round trip
  const int kf = k0 + j;
  const bool has = in && kf < k1;
  int af = -1, tf = 0, pf = 0, cf = 0, lvf = 0;
  double Bf[24], of[8];
  if (has) {
    af = A.lm_pose[kf];
    tf = P.etype[kf];
    pf = P.epose[kf];
    cf = P.ecam[kf];
    lvf = A.elevel ? A.elevel[kf] : 0;
    load_hpl4(L.Hpl, P.Ep, kf, Bf);
    const double* o = obs_of(P, kf, point ? 0 : 2);
#pragma unroll
    for (int q = 0; q < 8; q++) of[q] = (q < 3 || !point) ? o[q] : 0.0;
  }
  // the candidate poses (np <= 64) while the first edges are in flight; block 0 publishes them
  // for the verdict and the next trial
  if (tid < P.np) {
    double Tc[8];
    cand_pose(P, A, S.x, tid, failed, Tc);
#pragma unroll
    for (int k = 0; k < 8; k++) sT[8 * tid + k] = Tc[k];
    if (blockIdx.x == 0)
#pragma unroll
      for (int k = 0; k < 8; k++) P.Tn[8 * tid + k] = Tc[k];
  }
  __syncthreads();
  if (stamp) prof_stamp(S, kProfUe + 4 * blockIdx.x + 1);  // operands loaded
  const bool upd = in && act && !failed;
  // back-substitution xl = Dinv (bl - sum_e Hpl_e^T xp): the first edge from registers, any later
  // ones (landmarks with more than kGroup edges) from memory
  double c[4] = {0, 0, 0, 0};
  if (upd) {
    if (has && af >= 0) {
      const double* xp = sx + 6 * af;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < 6; r++) s += Bf[r * 4 + q] * xp[r];
        c[q] -= s;
      }
    }
    for (int k = kf + kGroup; k < k1; k += kGroup) {
      const int a = A.lm_pose[k];
      if (a < 0) continue;
      double B[24];
      load_hpl4(L.Hpl, P.Ep, k, B);
      const double* xp = sx + 6 * a;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < 6; r++) s += B[r * 4 + q] * xp[r];
        c[q] -= s;
      }
    }
  }
  group_sum(c);
  double xl[4] = {0, 0, 0, 0};
  double sc = 0, chi = 0;
  if (upd) {
#pragma unroll
    for (int q = 0; q < 4; q++) c[q] += blg[q];
    {
      double D[16];
      if (!lm_dinv(dl, point, lambda, D) && j == 0) atomicOr(S.fail, 1);
#pragma unroll
      for (int q = 0; q < 16; q++) dl[q] = point ? (q < 9 ? D[4 * (q / 3) + q % 3] : 0.0) : D[q];
    }
    if (point) {
#pragma unroll
      for (int r = 0; r < 3; r++) xl[r] = dl[r * 3] * c[0] + dl[r * 3 + 1] * c[1] + dl[r * 3 + 2] * c[2];
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++)
        xl[r] = dl[r * 4] * c[0] + dl[r * 4 + 1] * c[1] + dl[r * 4 + 2] * c[2] + dl[r * 4 + 3] * c[3];
    }
    if (j == 0)
#pragma unroll
      for (int q = 0; q < 4; q++) sc += xl[q] * (lambda * xl[q] + blg[q]);
  }
  const bool lin_pts = SPEC && spec && in && point;  // linearise the point edges at the candidate
  double hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bv[3] = {0, 0, 0};
  if (in) {
    if (point) {
#pragma unroll
      for (int q = 0; q < 3; q++) lm[q] += xl[q];
      if (j == 0)
#pragma unroll
        for (int q = 0; q < 3; q++) P.Xn[3 * g + q] = lm[q];
    } else {
      const int l = g - P.nq;
      if (upd) line_oplus(lm, xl);
      if (j == 0)
#pragma unroll
        for (int q = 0; q < 6; q++) P.Ln[6 * l + q] = lm[q];
    }
    // robust cost of the landmark's edges at the candidate (+ the point edges' linearisation)
    auto edge_cost = [&](int k, int te, int pose, int cam, int lev, const double (&ob)[8], int a) {
      if (lev) {
        if (lin_pts && a >= 0) zero_pose_records<false>(Ls, k);
        return;
      }
      const SE3 T = load_T(sT + 8 * pose);
      const double* cm = scam + 5 * cam;
      double er[4] = {0, 0, 0, 0};
      double chi2;
      if (point) {
        chi2 = point_error(te, cm, ob, T, lm, er);
      } else {
        edge_error(te, cm, ob, T, lm, er);
        chi2 = 0;
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (q < edim(te)) chi2 += er[q] * er[q];
        chi2 *= einfo(te);
      }
#pragma unroll
      for (int q = 0; q < 4; q++) L.err[4 * k + q] = er[q];
      double cst = chi2;
      if (A.robust) {
        double r1;
        huber(chi2, pick4(P.delta, te), cst, r1);
      }
      chi += cst;
      if (lin_pts) point_edge_core<false>(P, Ls, A, k, te, a >= 0, T, cm, lm, er, hl, bv);
    };
    if (has) edge_cost(kf, tf, pf, cf, lvf, of, af);
    for (int k = kf + kGroup; k < k1; k += kGroup) {
      const int te = P.etype[k];
      const double* o = obs_of(P, k, te);
      double ob[8];
#pragma unroll
      for (int q = 0; q < 8; q++) ob[q] = (q < 3 || !point) ? o[q] : 0.0;
      edge_cost(k, te, P.epose[k], P.ecam[k], A.elevel ? A.elevel[k] : 0, ob, A.lm_pose[k]);
    }
  }
  if (SPEC && spec) {  // point landmarks: the landmark blocks of the candidate's linearisation
    group_sum(hl);
    group_sum(bv);
    if (in && point && j == 0 && act) {
      double* H = Ss.Hll + 16 * g;
#pragma unroll
      for (int i = 0; i < 9; i++) H[i] = hl[i];
#pragma unroll
      for (int i = 9; i < 16; i++) H[i] = 0.0;
#pragma unroll
      for (int i = 0; i < 3; i++) Ss.bl[4 * g + i] = bv[i];
      Ss.bl[4 * g + 3] = 0.0;
    }
  }
  if (stamp) prof_stamp(S, kProfUe + 4 * blockIdx.x + 2);
  double acc[2] = {chi, sc};
  block_reduce<2>(acc, red);
  if (threadIdx.x == 0) {
    __hip_atomic_store(S.partial + blockIdx.x, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(S.partial2 + blockIdx.x, red[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned tk = ticket(S.counter);
    last = tk == (unsigned)nbu - 1;
  }
  __syncthreads();
  if (stamp) prof_stamp(S, kProfUe + 4 * blockIdx.x + 3);
  if (!last) return;
  double f2[2] = {0, 0};
  for (int k = threadIdx.x; k < nbu; k += 256) {
    f2[0] += __hip_atomic_load(S.partial + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f2[1] += __hip_atomic_load(S.partial2 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  block_reduce<2>(f2, red);
  if (threadIdx.x == 0) {
    const double chi2 = red[0], scale = red[1] + S.out[4];
    const double f = (double)__hip_atomic_load(S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double mx = S.out[2];
    S.out[0] = chi2;
    S.out[1] = scale;
    S.out[3] = f;
    if (S.shard_out) {  // sharded: landmark part only; shard_post adds the pose part S.out[4] once
      S.shard_out[0] = chi2;
      S.shard_out[1] = red[1];
      S.shard_out[2] = f;
      __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(S.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      S.out[2] = 0.0;
      return;
    }
    __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(S.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.out[2] = 0.0;
    if (S.lm) {  // device-side LM: decide here; the host reads the outcome only at the end
      LmCtrl* c = S.lm + (S.lm_slot ^ 1);
      const double lam0 = S.lm[S.lm_slot].lambda, chi0 = S.lm[S.lm_slot].chi;
      const int stop = lm_decide(S.lm + S.lm_slot, c, chi2, scale, f);
      if (S.lm_trace && c->trials <= 64) {
        double* t = S.lm_trace + 8 * (c->trials - 1);
        t[0] = chi2; t[1] = scale; t[2] = f; t[3] = lam0; t[4] = chi0; t[5] = c->cur; t[6] = c->it; t[7] = c->qmax;
      }
      // system-scope stores into host memory, each waited for: only when the host reads them
      if (stop || S.lm_post) post_mail(S.mail, c->chi, (double)c->it, (double)c->cur, (double)stop, seq);
      return;
    }
    post_mail(S.mail, chi2, scale, mx, f, seq);
  }
}

__global__ __launch_bounds__(256) void landmark_active_kernel(Active A, const uint8_t* level, uint8_t* lm_act) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.nL) return;
  uint8_t on = 0;
  for (int k = A.lm_off[g]; k < A.lm_off[g + 1]; k++) on |= level[(k)] == 0;
  lm_act[g] = on;
}

__device__ __forceinline__ bool edge_inlier(const Problem& P, const Lin& L, int e) {
  double chi2;
  bool depth_ok;
  edge_status(P, L, e, chi2, depth_ok);
  return chi2 <= pick4(P.th, P.etype[e]) && depth_ok;
}
__device__ __forceinline__ void classify_edge(const Problem& P, const Lin& L, int e, uint8_t* level, uint8_t* inlier,
                                              int final_pass) {
  if (final_pass) {
    inlier[e] = edge_inlier(P, L, e) ? 1 : 0;
    return;
  }
  double chi2;
  bool depth_ok;
  edge_status(P, L, e, chi2, depth_ok);
  if (chi2 > pick4(P.th, P.etype[e]) || !depth_ok) level[e] = 1;
}

__global__ __launch_bounds__(256) void classify_kernel(Problem P, Lin L, int E, uint8_t* level, uint8_t* inlier,
                                                       int final_pass) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) classify_edge(P, L, e, level, inlier, final_pass);
}

// end of a call: final inlier flags + the final T / X / L written straight into host-mapped
// memory; the last block (ticket) posts the mailbox once every block's writes are out
__global__ __launch_bounds__(256) void finish_kernel(Problem P, Lin L, int E, const int* gmap, uint8_t* inl, double* Th,
                                                     double* Xh, double* Lh, Sys S, unsigned long long seq) {
  __shared__ int last;
  if (S.lm) {  // queued behind the last optimize()'s trials (S.lm_slot: the control after the last one):
               // a no-op unless that optimize() has stopped; the current bank from its control
    const LmCtrl* c = S.lm + S.lm_slot;
    if (!c->stop) return;
    if (c->cur) bank_state(P);
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < E) inl[gmap[i]] = edge_inlier(P, L, i) ? 1 : 0;
  if (i < 8 * P.np) Th[i] = P.T[i];
  if (i < 3 * P.nq) Xh[i] = P.X[i];
  if (i < 6 * P.nl) Lh[i] = P.L[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(S.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == gridDim.x - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&S.mail->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// landmark sharding (rspl_ba_set_shard): the pieces between the host's all-reduces
// ---------------------------------------------------------------------------
__global__ void shard_fail_stage_kernel(Sys S, double* slot) {
  *slot = (double)__hip_atomic_load(S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void shard_fail_adopt_kernel(Sys S, const double* slot) {
  __hip_atomic_store(S.fail, *slot != 0.0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// this rank's pose-diagonal sums (block partials of pose_diag_kernel in block order) and its
// landmark maximum, laid out for the sum all-reduce
__global__ __launch_bounds__(256) void shard_fold_kernel(Sys S, double* red, int K, int npd, int rank, int nranks) {
  const int n6 = 6 * K;
  for (int q = threadIdx.x; q < n6; q += 256) {
    double acc = 0;
    if (npd > 0) {
      const int pa = q / 6, i = q - 6 * pa;
      const double* src = S.partial2 + (size_t)pa * npd * 6 + i;
      for (int b = 0; b < npd; b++) acc += src[(size_t)b * 6];
    }
    red[q] = acc;
  }
  for (int r = threadIdx.x; r < nranks; r += 256) red[n6 + r] = r == rank ? S.out[2] : 0.0;
}

__global__ void shard_post_kernel(Sys S, const double* red, int n6, int nranks, int mode, int add_pose_scale,
                                  unsigned long long seq) {
  __shared__ double mxs[64];
  const double* so = red + n6 + nranks;  // summed {chi2, scale, fail}
  double mx = 0;
  if (mode == 0) {
    for (int q = threadIdx.x; q < n6; q += 64) mx = fmax(mx, fabs(red[q]));
    for (int r = threadIdx.x; r < nranks; r += 64) mx = fmax(mx, red[n6 + r]);
  }
  mxs[threadIdx.x] = mx;
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int k = 1; k < 64; k++) mx = fmax(mx, mxs[k]);
  const double chi2 = so[0], scale = so[1] + (add_pose_scale ? S.out[4] : 0.0), f = so[2] != 0.0 ? 1.0 : 0.0;
  if (mode == 0) S.out[2] = mx;
  S.out[0] = chi2;
  S.out[1] = scale;
  S.out[3] = f;
  post_mail(S.mail, chi2, scale, mode == 0 ? mx : S.out[2], f, seq);
}

// G = [X (owned points) | L (owned lines) | inlier flag at the global edge id of each local edge]
__global__ __launch_bounds__(256) void shard_gather_kernel(Problem P, Lin L, int E, const int* gmap, int rank,
                                                           int nranks, double* G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nq3 = 3 * P.nq, nl6 = 6 * P.nl;
  if (i < E) {
    G[nq3 + nl6 + gmap[i]] = edge_inlier(P, L, i) ? 1.0 : 0.0;
  }
  if (i < nq3 && (i / 3) % nranks == rank) G[i] = P.X[i];
  if (i < nl6 && (P.nq + i / 6) % nranks == rank) G[nq3 + i] = P.L[i];
}

__global__ __launch_bounds__(256) void shard_finish_kernel(Problem P, int E, const double* G, uint8_t* inl,
                                                           double* Th, double* Xh, double* Lh, Sys S,
                                                           unsigned long long seq) {
  __shared__ int last;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nq3 = 3 * P.nq, nl6 = 6 * P.nl;
  if (i < E) inl[i] = G[nq3 + nl6 + i] != 0.0;
  if (i < 8 * P.np) Th[i] = P.T[i];
  if (i < nq3) Xh[i] = G[i];
  if (i < nl6) Lh[i] = G[nq3 + i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(S.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == gridDim.x - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __hip_atomic_store(S.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&S.mail->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int shard_red_len(int K, int nranks) { return 6 * K + nranks + 3; }
bool fast_path(int K) { return 6 * K > 0 && 6 * K <= kCholLdsMax; }
bool wave_path(int K) { return K > 0 && K <= kWaveSolveMaxK; }
// reduced-system solver for K <= 10: the single-wave LDL^T fused into the last Schur chunk (two launches per
// trial); a 4-wave blocked LDL^T as a third launch lost in the pipeline (788 vs 772 frames/s, four alternating runs
// on two boxes, profiles/r03_experiments.md) and was removed in round 6.  K > 10: the LDS / register solves.
// ---------------------------------------------------------------------------
int errors_blocks(int Ea) { return Ea > 0 ? (Ea + 255) / 256 : 1; }
int update_blocks(const Problem& P) {
  const int nv = P.np + P.nq + P.nl;
  return nv > 0 ? (nv + 255) / 256 : 1;
}

hipError_t compute_errors(const Problem& P, const Lin& L, const Active& A, Sys& S, unsigned long long seq,
                          hipStream_t s) {
  hipLaunchKernelGGL(errors_kernel, dim3(errors_blocks(A.Ea)), dim3(256), 0, s, P, L, A, S, 0, seq);
  return hipGetLastError();
}

int update_errors_blocks(const Active& A) {
  if (A.ue_bpr > 0) return 8 * ((A.nchk + 7) / 8) * A.ue_bpr;
  return A.nL > 0 ? (A.nL * kGroup + 64 * kUeWaves - 1) / (64 * kUeWaves) : 1;
}

void set_update_geometry(Active& A) {
  constexpr int per = 64 * kUeWaves / kGroup;  // landmarks per update workgroup
  A.ue_bpr = A.nchk >= 8 && A.lmchunk % per == 0 ? A.lmchunk / per : 0;
}

hipError_t linearize(const Problem& P, const Lin& L, const Active& A, const Sys& S, bool with_maxdiag,
                     hipStream_t s) {
  const int nbq = (P.nq * kGroup + 255) / 256, nbl = A.n_lblk;
  if (nbq + nbl > 0)
    hipLaunchKernelGGL(linearize_kernel, dim3(nbq + nbl), dim3(256), 0, s, P, L, A, S, nbq, with_maxdiag ? 1 : 0);
  if (with_maxdiag && A.K > 0 && A.Ea > 0)
    hipLaunchKernelGGL(pose_diag_kernel, dim3((A.Ea + 255) / 256), dim3(256), 0, s, P, L, A, S);
  return hipGetLastError();
}

int setup_pdg_len(const Active& A) {
  const int nbq = A.nL > 0 ? (A.nL * kGroup + 255) / 256 : 0;
  return 6 * A.K * (nbq + A.n_lblk) + 6;
}

hipError_t setup_dev(const Problem& P, const Lin& L, const Active& A, Sys& S, uint8_t* level, uint8_t* lm_act2,
                     int lm_iters, int* pp_cnt, int* pp_off, int4* pp, double* pdg, hipStream_t s, int gate,
                     const Lin* Ls, const Sys* Ss) {
  if (gate >= 0 && (!Ls || !Ss || pp_cnt)) return hipErrorInvalidValue;
  if (!S.lm || lm_iters <= 0) return hipErrorInvalidValue;
  Active A0 = A;
  A0.elevel = nullptr;  // the levels are written by this launch (level != null), never read by it
  const int nc = chunk_count(A);
  if (nc == 0) pp_cnt = nullptr;
  const int nbq = A.nL > 0 ? (A.nL * kGroup + 255) / 256 : 0, nb = nbq + A.n_lblk;
  const int nbp = pp_cnt ? (nc + 3) / 4 : 0;
  // at least one block: the last one writes the LM control
  hipLaunchKernelGGL(setup_kernel, dim3(std::max(nb + nbp, 1)), dim3(256), 0, s, P, L, A0, S, nbq, nb, level, lm_act2,
                     pp_cnt, pp_off, pdg, lm_iters, gate, Ls ? *Ls : L, Ss ? *Ss : S);
  if (pp_cnt) hipLaunchKernelGGL(pair_fill_kernel, dim3(nc), dim3(64), 0, s, A, pp_off, pp);
  return hipGetLastError();
}

hipError_t post(Sys& S, unsigned long long seq, hipStream_t s, const Active* A, int lm_iters) {
  const int npd = (A && A->K > 0 && A->Ea > 0) ? (A->Ea + 255) / 256 : 0;
  hipLaunchKernelGGL(post_kernel, dim3(1), dim3(256), 0, s, S, A ? A->K : 0, npd, seq, lm_iters);
  return hipGetLastError();
}

size_t schur_lds_bytes(int n) { return sizeof(double) * ((size_t)(n + 1) * (n + 2) / 2 + 3 * n + 15 * (n / 6)); }

hipError_t ensure_schur_attr() {
  static bool attr = false;
  if (attr) return hipSuccess;
  hipError_t e = hipFuncSetAttribute((const void*)schur_solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)schur_lds_bytes(kCholLdsMax));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)schur_reg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)solve_reg_lds_bytes(kRegMaxK));
  if (e == hipSuccess) attr = true;
  return e;
}

// the LDS-resident blocked LDL^T of the reduced system (K > kWaveSolveMaxK): the register-resident kernel for
// K <= kRegMaxK, the packed-LDS one beyond
static void launch_lds_solve(const Problem& P, const Active& A, const Sys& S, double lambda, hipStream_t s) {
  const int n = 6 * A.K;
  if (A.K > kRegMaxK)
    hipLaunchKernelGGL(schur_solve_kernel, dim3(1), dim3(256), schur_lds_bytes(n), s, P, A, S, n, lambda);
  else
    hipLaunchKernelGGL(schur_reg_kernel, dim3(1), dim3(kSolveRegThreads), solve_reg_lds_bytes(A.K), s, P, A, S, n,
                       lambda);
}

// pair_chunk grid: 8 XCD lanes x (landmark ranges per XCD) x pose pairs (idle slots exit)
static int pair_chunk_blocks(const Active& A) {
  return A.nchk >= 8 ? 8 * ((A.nchk + 7) / 8) * A.npairs : chunk_count(A);
}

// Schur chunks; with fused = true (wave path) the last pose pair also solves (solve_wave<6K>)
static void launch_chunks(const Problem& P, const Lin& L, const Active& A, const Sys& S, double lambda, const Lin& Ls,
                          const Sys& Ss, bool fused, hipStream_t s) {
  const dim3 g(pair_chunk_blocks(A)), b(64);
  switch (fused ? A.K : 0) {
#define RSPL_CHUNK_CASE(k) \
  case k: hipLaunchKernelGGL(pair_chunk_kernel<6 * k>, g, b, 0, s, P, L, A, S, lambda, Ls, Ss); break;
    RSPL_CHUNK_CASE(1) RSPL_CHUNK_CASE(2) RSPL_CHUNK_CASE(3) RSPL_CHUNK_CASE(4) RSPL_CHUNK_CASE(5)
    RSPL_CHUNK_CASE(6) RSPL_CHUNK_CASE(7) RSPL_CHUNK_CASE(8) RSPL_CHUNK_CASE(9) RSPL_CHUNK_CASE(10)
#undef RSPL_CHUNK_CASE
    default: hipLaunchKernelGGL(pair_chunk_kernel<0>, g, b, 0, s, P, L, A, S, lambda, Ls, Ss); break;
  }
}

static void launch_wave_solve(const Problem& P, const Active& A, const Sys& S, double lambda, hipStream_t s) {
  switch (A.K) {
#define RSPL_SOLVE_CASE(k) \
  case k: hipLaunchKernelGGL(schur_wave_kernel<6 * k>, dim3(1), dim3(64), 0, s, P, A, S, lambda); break;
    RSPL_SOLVE_CASE(1) RSPL_SOLVE_CASE(2) RSPL_SOLVE_CASE(3) RSPL_SOLVE_CASE(4) RSPL_SOLVE_CASE(5)
    RSPL_SOLVE_CASE(6) RSPL_SOLVE_CASE(7) RSPL_SOLVE_CASE(8) RSPL_SOLVE_CASE(9) RSPL_SOLVE_CASE(10)
#undef RSPL_SOLVE_CASE
    default: break;
  }
}

hipError_t trial(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, unsigned long long seq,
                 hipStream_t s, const Spec* spec, bool* fused) {
  *fused = false;
  const bool wave = wave_path(A.K);
  if (chunk_count(A) > 0) launch_chunks(P, L, A, S, lambda, L, S, wave, s);
  const int n = 6 * A.K;
  if (fast_path(A.K)) {
    if (!wave) {
      hipError_t e = ensure_schur_attr();
      if (e != hipSuccess) return e;
      launch_lds_solve(P, A, S, lambda, s);
    }
    const int nbu = update_errors_blocks(A);
    if (spec) {
      const int nbl = A.n_lblk;
      hipLaunchKernelGGL(update_errors_kernel<true>, dim3(nbu + nbl), dim3(256), 0, s, P, L, A, S, lambda, seq,
                         spec->Ls, spec->Ss, nbu);
      *fused = true;
    } else {
      hipLaunchKernelGGL(update_errors_kernel<false>, dim3(nbu), dim3(256), 0, s, P, L, A, S, lambda, seq, L, S, 0);
    }
    return hipGetLastError();
  }
  if (n > 0) {  // larger systems: Schur sums + global-memory Cholesky
    hipLaunchKernelGGL(pair_final_kernel, dim3((A.npairs * 42 + 255) / 256), dim3(256), 0, s, A, S, lambda);
    hipLaunchKernelGGL(cholesky_kernel, dim3(1), dim3(256), 0, s, S, n);
  }
  const int nbu = update_blocks(P);
  hipLaunchKernelGGL(update_kernel, dim3(nbu), dim3(256), 0, s, P, L, A, S, lambda);
  Problem Pn = P;  // cost of the candidate state
  Pn.T = P.Tn; Pn.X = P.Xn; Pn.L = P.Ln;
  hipLaunchKernelGGL(errors_kernel, dim3(errors_blocks(A.Ea)), dim3(256), 0, s, Pn, L, A, S, nbu, seq);
  return hipGetLastError();
}

hipError_t trial_dev(const Problem& P, const Lin& L, const Active& A, Sys& S, unsigned long long seq, hipStream_t s,
                     const Spec& spec, hipEvent_t* ev) {
  if (!S.lm || !fast_path(A.K)) return hipErrorInvalidValue;
  const bool wave = wave_path(A.K);
  if (ev) (void)hipEventRecord(ev[0], s);
  if (chunk_count(A) > 0) launch_chunks(P, L, A, S, 0.0, spec.Ls, spec.Ss, wave, s);
  if (!wave) {
    hipError_t e = ensure_schur_attr();
    if (e != hipSuccess) return e;
    launch_lds_solve(P, A, S, 0.0, s);
  }
  const int nbu = update_errors_blocks(A), nbl = A.n_lblk;
  if (ev) (void)hipEventRecord(ev[1], s);
  hipLaunchKernelGGL(update_errors_kernel<true>, dim3(nbu + nbl), dim3(256), 0, s, P, L, A, S, 0.0, seq, spec.Ls,
                     spec.Ss, nbu);
  if (ev) (void)hipEventRecord(ev[2], s);
  return hipGetLastError();
}

hipError_t finish(const Problem& P, const Lin& L, int E, const int* gmap, uint8_t* inl, double* Th, double* Xh,
                  double* Lh, Sys& S, unsigned long long seq, hipStream_t s) {
  const int n = std::max(std::max(E, 8 * P.np), std::max(3 * P.nq, 6 * P.nl));
  hipLaunchKernelGGL(finish_kernel, dim3(std::max((n + 255) / 256, 1)), dim3(256), 0, s, P, L, E, gmap, inl, Th, Xh,
                     Lh, S, seq);
  return hipGetLastError();
}

hipError_t build_pairs(const Active& A, int* pp_cnt, int* pp_off, int4* pp, hipStream_t s) {
  const int nc = chunk_count(A);
  if (nc == 0) return hipSuccess;
  hipLaunchKernelGGL(pair_count_kernel, dim3(nc), dim3(64), 0, s, A, pp_cnt);
  hipLaunchKernelGGL(pair_offsets_kernel, dim3(1), dim3(1024), 0, s, pp_cnt, pp_off, nc);
  hipLaunchKernelGGL(pair_fill_kernel, dim3(nc), dim3(64), 0, s, A, pp_off, pp);
  return hipGetLastError();
}

hipError_t landmark_active(const Active& A, const uint8_t* level, uint8_t* lm_act, hipStream_t s) {
  if (A.nL > 0) hipLaunchKernelGGL(landmark_active_kernel, dim3((A.nL + 255) / 256), dim3(256), 0, s, A, level, lm_act);
  return hipGetLastError();
}

hipError_t classify(const Problem& P, const Lin& L, int E, uint8_t* level, uint8_t* inlier, int final_pass,
                    hipStream_t s) {
  if (E > 0) hipLaunchKernelGGL(classify_kernel, dim3((E + 255) / 256), dim3(256), 0, s, P, L, E, level, inlier,
                                final_pass);
  return hipGetLastError();
}

hipError_t trial_chunks(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s) {
  if (chunk_count(A) > 0) launch_chunks(P, L, A, S, lambda, L, S, false, s);
  hipLaunchKernelGGL(shard_fail_stage_kernel, dim3(1), dim3(1), 0, s, S, S.pairfin + (size_t)A.npairs * 48);
  return hipGetLastError();
}

hipError_t trial_solve(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s) {
  hipLaunchKernelGGL(shard_fail_adopt_kernel, dim3(1), dim3(1), 0, s, S, S.pairfin + (size_t)A.npairs * 48);
  const int n = 6 * A.K;
  if (fast_path(A.K)) {
    if (wave_path(A.K)) {
      launch_wave_solve(P, A, S, lambda, s);
    } else {
      hipError_t e = ensure_schur_attr();
      if (e != hipSuccess) return e;
      launch_lds_solve(P, A, S, lambda, s);
    }
    hipLaunchKernelGGL(update_errors_kernel<false>, dim3(update_errors_blocks(A)), dim3(256), 0, s, P, L, A, S, lambda,
                       0ull, L, S, 0);
    return hipGetLastError();
  }
  if (n > 0) {
    hipLaunchKernelGGL(pair_final_kernel, dim3((A.npairs * 42 + 255) / 256), dim3(256), 0, s, A, S, lambda);
    hipLaunchKernelGGL(cholesky_kernel, dim3(1), dim3(256), 0, s, S, n);
  }
  const int nbu = update_blocks(P);
  hipLaunchKernelGGL(update_kernel, dim3(nbu), dim3(256), 0, s, P, L, A, S, lambda);
  Problem Pn = P;
  Pn.T = P.Tn; Pn.X = P.Xn; Pn.L = P.Ln;
  hipLaunchKernelGGL(errors_kernel, dim3(errors_blocks(A.Ea)), dim3(256), 0, s, Pn, L, A, S, nbu, 0ull);
  return hipGetLastError();
}

hipError_t shard_fold(const Active& A, Sys& S, double* red, int rank, int nranks, hipStream_t s) {
  const int npd = (A.K > 0 && A.Ea > 0) ? (A.Ea + 255) / 256 : 0;
  hipLaunchKernelGGL(shard_fold_kernel, dim3(1), dim3(256), 0, s, S, red, A.K, npd, rank, nranks);
  return hipGetLastError();
}

hipError_t shard_post(Sys& S, const double* red, int n6, int nranks, int mode, int add_pose_scale,
                      unsigned long long seq, hipStream_t s) {
  hipLaunchKernelGGL(shard_post_kernel, dim3(1), dim3(64), 0, s, S, red, n6, nranks, mode, add_pose_scale, seq);
  return hipGetLastError();
}

hipError_t shard_gather(const Problem& P, const Lin& L, int E, const int* gmap, int rank, int nranks, double* G,
                        hipStream_t s) {
  const int n = std::max(E, std::max(3 * P.nq, 6 * P.nl));
  if (n > 0)
    hipLaunchKernelGGL(shard_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, P, L, E, gmap, rank, nranks, G);
  return hipGetLastError();
}

hipError_t shard_finish(const Problem& P, int E_global, const double* G, uint8_t* inl, double* Th, double* Xh,
                        double* Lh, Sys& S, unsigned long long seq, hipStream_t s) {
  const int n = std::max(std::max(E_global, 8 * P.np), std::max(3 * P.nq, 6 * P.nl));
  hipLaunchKernelGGL(shard_finish_kernel, dim3(std::max((n + 255) / 256, 1)), dim3(256), 0, s, P, E_global, G, inl,
                     Th, Xh, Lh, S, seq);
  return hipGetLastError();
}

}  // namespace ba
}  // namespace rspl
