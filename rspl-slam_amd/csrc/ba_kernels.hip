// Local bundle adjustment (LocalmapOptimization, src/g2o_optimization/g2o_optimization.cc:21-252)
// as an fp64 Levenberg-Marquardt on gfx950.  Same algorithm as the CPU restatement
// (oracle/ba.c, which restates the g2o pieces it relies on): SE3 left exp-map update,
// analytic point Jacobians, numeric (delta 1e-9) line Jacobians, Huber IRLS weights,
// Schur complement on marginalised points + lines, dense Cholesky of the reduced
// camera system.  Every reduction runs in a fixed order (CSR lists, fixed trees), so
// a call is bitwise reproducible.  Not a dense contraction: no MFMA; HBM/latency bound.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "ba_kernels.hpp"

namespace rspl {
namespace ba {

struct SE3 {
  double q[4];  // w x y z
  double t[3];
};

__device__ __forceinline__ void q_to_R(const double* q, double* R) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ void mat3_vec(const double* R, const double* v, double* o) {
  o[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  o[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  o[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
}

__device__ __forceinline__ void se3_normalize(SE3& T) {
  if (T.q[0] < 0)
    for (int i = 0; i < 4; i++) T.q[i] = -T.q[i];
  const double n = sqrt(T.q[0] * T.q[0] + T.q[1] * T.q[1] + T.q[2] * T.q[2] + T.q[3] * T.q[3]);
  for (int i = 0; i < 4; i++) T.q[i] /= n;
}

__device__ __forceinline__ void R_to_q(const double* m, double* q) {
  const double t = m[0] + m[4] + m[8];
  if (t > 0) {
    double s = sqrt(t + 1.0);
    q[0] = 0.5 * s;
    s = 0.5 / s;
    q[1] = (m[7] - m[5]) * s;
    q[2] = (m[2] - m[6]) * s;
    q[3] = (m[3] - m[1]) * s;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[i * 3 + i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double s = sqrt(m[i * 3 + i] - m[j * 3 + j] - m[k * 3 + k] + 1.0);
    double v[3];
    v[i] = 0.5 * s;
    s = 0.5 / s;
    q[0] = (m[k * 3 + j] - m[j * 3 + k]) * s;
    v[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
    v[k] = (m[k * 3 + i] + m[i * 3 + k]) * s;
    q[1] = v[0]; q[2] = v[1]; q[3] = v[2];
  }
}

__device__ __forceinline__ SE3 se3_mul(const SE3& a, const SE3& b) {
  SE3 r;
  double R[9], t[3];
  q_to_R(a.q, R);
  mat3_vec(R, b.t, t);
  for (int i = 0; i < 3; i++) r.t[i] = a.t[i] + t[i];
  r.q[0] = a.q[0] * b.q[0] - a.q[1] * b.q[1] - a.q[2] * b.q[2] - a.q[3] * b.q[3];
  r.q[1] = a.q[0] * b.q[1] + a.q[1] * b.q[0] + a.q[2] * b.q[3] - a.q[3] * b.q[2];
  r.q[2] = a.q[0] * b.q[2] - a.q[1] * b.q[3] + a.q[2] * b.q[0] + a.q[3] * b.q[1];
  r.q[3] = a.q[0] * b.q[3] + a.q[1] * b.q[2] - a.q[2] * b.q[1] + a.q[3] * b.q[0];
  se3_normalize(r);
  return r;
}

// SE3Quat::exp, update = [omega; upsilon]
__device__ SE3 se3_exp(const double* u) {
  const double* w = u;
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double O2[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += O[i * 3 + k] * O[k * 3 + j];
      O2[i * 3 + j] = s;
    }
  double a, b, c, d;
  if (th < 1e-5) {
    a = 1.0; b = 0.5; c = 0.5; d = 1.0 / 6.0;
  } else {
    a = sin(th) / th;
    b = (1 - cos(th)) / (th * th);
    c = b;
    d = (th - sin(th)) / (th * th * th);
  }
  double R[9], V[9];
  for (int i = 0; i < 9; i++) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    R[i] = I + a * O[i] + b * O2[i];
    V[i] = I + c * O[i] + d * O2[i];
  }
  SE3 r;
  R_to_q(R, r.q);
  mat3_vec(V, u + 3, r.t);
  se3_normalize(r);
  return r;
}

__device__ __forceinline__ double n3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
__device__ __forceinline__ void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// g2o::Line3D::oplus (orthonormal 4-DoF update; vertex_line3d.h:26-29)
__device__ void line_oplus(double* L, const double* v) {
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
__device__ void edge_error(int type, const double* cam, const double* obs, const SE3& T, const double* lm, double* e) {
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
  const int sides = type == 3 ? 2 : 1;
  for (int side = 0; side < sides; side++) {
    double t[3] = {T.t[0], T.t[1], T.t[2]};
    if (side == 1) t[0] -= cam[4] / fx;  // T_right(0,3) -= b, b = bf / fx
    double Rw[3], Rd[3], tx[3];
    mat3_vec(R, lm, Rw);
    mat3_vec(R, lm + 3, Rd);
    cross3(t, Rd, tx);
    const double w0 = Rw[0] + tx[0], w1 = Rw[1] + tx[1], w2 = Rw[2] + tx[2];
    const double l0 = fy * w0, l1 = fx * w1, l2 = Kv0 * w0 + Kv1 * w1 + Kv2 * w2;
    const double nrm = sqrt(l0 * l0 + l1 * l1);
    const double* o = obs + 4 * side;
    e[2 * side + 0] = (o[0] * l0 + o[1] * l1 + l2) / nrm;
    e[2 * side + 1] = (o[2] * l0 + o[3] * l1 + l2) / nrm;
  }
}

__device__ __forceinline__ int edim(int t) { return t == 0 ? 2 : t == 1 ? 3 : t == 2 ? 2 : 4; }
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
// errors + robust chi2 per active edge; block partial sums (fixed tree)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void errors_kernel(Problem P, Lin L, Active A, double* partial) {
  __shared__ double red[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  double c = 0.0;
  if (i < A.Ea) {
    const int e = A.edges[i];
    const int t = P.etype[e];
    const SE3 T = load_T(P.T + 8 * P.epose[e]);
    double er[4] = {0, 0, 0, 0};
    edge_error(t, P.cams + 5 * P.ecam[e], P.eobs + 8 * e, T, lm_ptr(P, P.elm[e]), er);
    double chi2 = 0;
    for (int k = 0; k < edim(t); k++) chi2 += er[k] * er[k];
    chi2 *= einfo(t);
    for (int k = 0; k < 4; k++) L.err[4 * e + k] = er[k];
    if (A.robust) {
      double r1;
      huber(chi2, P.delta[t], c, r1);
    } else {
      c = chi2;
    }
    L.rho0[e] = c;
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------
// per-edge Jacobians + weighted normal-equation contributions
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void linearize_kernel(Problem P, Lin L, Active A) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.Ea) return;
  const int e = A.edges[i];
  const int t = P.etype[e], rows = edim(t), ld = ldim(t);
  const int pose = P.epose[e], g = P.elm[e];
  const double* cam = P.cams + 5 * P.ecam[e];
  const double* obs = P.eobs + 8 * e;
  const SE3 T = load_T(P.T + 8 * pose);
  double Jp[4][6], Jl[4][4];
  if (t < 2) {  // analytic (g2o types_sba), J = -dproj/dXc * dXc/dparam
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    const double* X = P.X + 3 * g;
    double R[9], Xc[3];
    q_to_R(T.q, R);
    mat3_vec(R, X, Xc);
    for (int k = 0; k < 3; k++) Xc[k] += T.t[k];
    const double x = Xc[0], y = Xc[1], z = Xc[2], iz = 1.0 / z, iz2 = iz * iz;
    const double D[3][3] = {{fx * iz, 0, -fx * x * iz2}, {0, fy * iz, -fy * y * iz2}, {fx * iz, 0, -fx * x * iz2 + bf * iz2}};
    const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int r = 0; r < rows; r++)
      for (int c = 0; c < 3; c++) {
        double s = 0, sl = 0;
        for (int k = 0; k < 3; k++) {
          s += D[r][k] * SX[k * 3 + c];
          sl += D[r][k] * R[k * 3 + c];
        }
        Jp[r][c] = s;
        Jp[r][3 + c] = -D[r][c];
        Jl[r][c] = -sl;
      }
  } else {  // numeric central difference, delta 1e-9 (g2o BaseBinaryEdge::linearizeOplus)
    const double delta = 1e-9, scal = 1.0 / (2 * delta);
    const double* L0 = P.L + 6 * (g - P.nq);
    double ep[4], em[4], Lp[6];
    for (int d = 0; d < 4; d++) {
      double v[4] = {0, 0, 0, 0};
      v[d] = delta;
      for (int k = 0; k < 6; k++) Lp[k] = L0[k];
      line_oplus(Lp, v);
      edge_error(t, cam, obs, T, Lp, ep);
      v[d] = -delta;
      for (int k = 0; k < 6; k++) Lp[k] = L0[k];
      line_oplus(Lp, v);
      edge_error(t, cam, obs, T, Lp, em);
      for (int r = 0; r < rows; r++) Jl[r][d] = scal * (ep[r] - em[r]);
    }
    for (int d = 0; d < 6; d++) {
      double u[6] = {0, 0, 0, 0, 0, 0};
      u[d] = delta;
      SE3 Tp = se3_mul(se3_exp(u), T);
      edge_error(t, cam, obs, Tp, L0, ep);
      u[d] = -delta;
      Tp = se3_mul(se3_exp(u), T);
      edge_error(t, cam, obs, Tp, L0, em);
      for (int r = 0; r < rows; r++) Jp[r][d] = scal * (ep[r] - em[r]);
    }
  }
  const double* er = L.err + 4 * e;
  double w = einfo(t);
  if (A.robust) {
    double chi2 = 0;
    for (int k = 0; k < rows; k++) chi2 += er[k] * er[k];
    chi2 *= einfo(t);
    double r0, r1;
    huber(chi2, P.delta[t], r0, r1);
    w *= r1;  // robustInformation = rho'(chi2) * Omega
  }
  double* Hll = L.Hll + 16 * e;
  double* bl = L.bl + 4 * e;
  for (int a = 0; a < ld; a++) {
    double s = 0;
    for (int r = 0; r < rows; r++) s += Jl[r][a] * er[r];
    bl[a] = -w * s;
    for (int b = 0; b < ld; b++) {
      double h = 0;
      for (int r = 0; r < rows; r++) h += Jl[r][a] * Jl[r][b];
      Hll[a * ld + b] = w * h;
    }
  }
  if (A.pidx[pose] >= 0) {
    double* Hpp = L.Hpp + 36 * e;
    double* bp = L.bp + 6 * e;
    double* Hpl = L.Hpl + 24 * e;
    for (int a = 0; a < 6; a++) {
      double s = 0;
      for (int r = 0; r < rows; r++) s += Jp[r][a] * er[r];
      bp[a] = -w * s;
      for (int b = 0; b < 6; b++) {
        double h = 0;
        for (int r = 0; r < rows; r++) h += Jp[r][a] * Jp[r][b];
        Hpp[a * 6 + b] = w * h;
      }
      for (int b = 0; b < ld; b++) {
        double h = 0;
        for (int r = 0; r < rows; r++) h += Jp[r][a] * Jl[r][b];
        Hpl[a * 4 + b] = w * h;
      }
    }
  }
}

__device__ __forceinline__ void atomic_max_pos(double* addr, double v) {
  // non-negative doubles order like their bit patterns
  atomicMax(reinterpret_cast<unsigned long long*>(addr), (unsigned long long)__double_as_longlong(v));
}

// landmark blocks: Hll = sum_e Hll_e, bl = sum_e bl_e (edge order of the CSR list)
__global__ __launch_bounds__(256) void landmark_reduce_kernel(Problem P, Lin L, Active A, Sys S) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.nL || !A.lm_act[g]) return;
  const int ld = g < P.nq ? 3 : 4;
  double H[16] = {0}, b[4] = {0};
  for (int k = A.lm_off[g]; k < A.lm_off[g + 1]; k++) {
    const int e = A.lm_edges[k];
    for (int i = 0; i < ld * ld; i++) H[i] += L.Hll[16 * e + i];
    for (int i = 0; i < ld; i++) b[i] += L.bl[4 * e + i];
  }
  double mx = 0;
  for (int i = 0; i < 16; i++) S.Hll[16 * g + i] = H[i];
  for (int i = 0; i < 4; i++) S.bl[4 * g + i] = b[i];
  for (int i = 0; i < ld; i++) mx = fmax(mx, fabs(H[i * ld + i]));
  atomic_max_pos(S.out + 2, mx);
}

// pose blocks: Hpp = sum_e Hpp_e, bp = sum_e bp_e over the pose's edges; fixed reduction tree
__global__ __launch_bounds__(128) void pose_reduce_kernel(Problem P, Lin L, Active A, Sys S) {
  __shared__ double red[42][128];
  const int a = blockIdx.x, tid = threadIdx.x;
  double acc[42];
  for (int i = 0; i < 42; i++) acc[i] = 0;
  for (int k = A.ps_off[a] + tid; k < A.ps_off[a + 1]; k += 128) {
    const int e = A.ps_edges[k];
    for (int i = 0; i < 36; i++) acc[i] += L.Hpp[36 * e + i];
    for (int i = 0; i < 6; i++) acc[36 + i] += L.bp[6 * e + i];
  }
  for (int i = 0; i < 42; i++) red[i][tid] = acc[i];
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (tid < s)
      for (int i = 0; i < 42; i++) red[i][tid] += red[i][tid + s];
    __syncthreads();
  }
  if (tid < 36) S.Hpp[36 * a + tid] = red[tid][0];
  if (tid < 6) S.bp[6 * a + tid] = red[36 + tid][0];
  if (tid == 0) {
    double mx = 0;
    for (int i = 0; i < 6; i++) mx = fmax(mx, fabs(red[i * 7][0]));
    atomic_max_pos(S.out + 2, mx);
  }
}

// ---------------------------------------------------------------------------
// Schur complement for damping lambda
// ---------------------------------------------------------------------------
__device__ bool small_inv(const double* A, double* I, int n) {
  double M[4][8];
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      M[i][j] = A[i * n + j];
      M[i][n + j] = (i == j);
    }
  for (int c = 0; c < n; c++) {
    int p = c;
    for (int r = c + 1; r < n; r++)
      if (fabs(M[r][c]) > fabs(M[p][c])) p = r;
    if (M[p][c] == 0) return false;
    if (p != c)
      for (int k = 0; k < 2 * n; k++) {
        const double t = M[c][k];
        M[c][k] = M[p][k];
        M[p][k] = t;
      }
    const double iv = 1.0 / M[c][c];
    for (int k = 0; k < 2 * n; k++) M[c][k] *= iv;
    for (int r = 0; r < n; r++)
      if (r != c) {
        const double f = M[r][c];
        for (int k = 0; k < 2 * n; k++) M[r][k] -= f * M[c][k];
      }
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) I[i * n + j] = M[i][n + j];
  return true;
}

__global__ __launch_bounds__(256) void landmark_schur_kernel(Problem P, Lin L, Active A, Sys S, double lambda) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.nL || !A.lm_act[g]) return;
  const int ld = g < P.nq ? 3 : 4;
  double H[16], D[16];
  for (int i = 0; i < ld * ld; i++) H[i] = S.Hll[16 * g + i];
  for (int i = 0; i < ld; i++) H[i * ld + i] += lambda;
  if (!small_inv(H, D, ld)) {
    atomicOr(S.fail, 1);
    return;
  }
  for (int i = 0; i < ld * ld; i++) S.Dinv[16 * g + i] = D[i];
  for (int k = A.lm_off[g]; k < A.lm_off[g + 1]; k++) {
    const int e = A.lm_edges[k];
    if (A.pidx[P.epose[e]] < 0) continue;
    const double* B = L.Hpl + 24 * e;
    double* Y = L.Y + 24 * e;
    for (int r = 0; r < 6; r++)
      for (int c = 0; c < ld; c++) {
        double s = 0;
        for (int k2 = 0; k2 < ld; k2++) s += B[r * 4 + k2] * D[k2 * ld + c];
        Y[r * 4 + c] = s;
      }
  }
}

// one block per reduced pose pair (a <= b):
//   S_ab = [a==b](Hpp_a + lambda I) - sum_{landmarks seen by both} Y_e1 Hpl_e2^T,  bs_a = bp_a - sum Y_e bl_l
__global__ __launch_bounds__(128) void pair_schur_kernel(Problem P, Lin L, Active A, Sys S, double lambda) {
  __shared__ double red[42][128];
  const int pr = blockIdx.x, tid = threadIdx.x;
  const int a = A.pairs[2 * pr], b = A.pairs[2 * pr + 1];
  const int n = 6 * A.K;
  double acc[42];
  for (int i = 0; i < 42; i++) acc[i] = 0;
  const int b0 = A.ps_off[b], b1 = A.ps_off[b + 1];
  for (int k = A.ps_off[a] + tid; k < A.ps_off[a + 1]; k += 128) {
    const int e1 = A.ps_edges[k], g = A.ps_lm[k];
    const int ld = g < P.nq ? 3 : 4;
    const double* Y = L.Y + 24 * e1;
    // lower_bound of g in the (sorted) landmark list of pose b
    int lo = b0, hi = b1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (A.ps_lm[mid] < g) lo = mid + 1;
      else hi = mid;
    }
    for (int j = lo; j < b1 && A.ps_lm[j] == g; j++) {
      const double* B2 = L.Hpl + 24 * A.ps_edges[j];
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) {
          double s = 0;
          for (int q = 0; q < ld; q++) s += Y[r * 4 + q] * B2[c * 4 + q];
          acc[r * 6 + c] += s;
        }
    }
    if (a == b) {
      const double* bl = S.bl + 4 * g;
      for (int r = 0; r < 6; r++) {
        double s = 0;
        for (int q = 0; q < ld; q++) s += Y[r * 4 + q] * bl[q];
        acc[36 + r] += s;
      }
    }
  }
  for (int i = 0; i < 42; i++) red[i][tid] = acc[i];
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (tid < s)
      for (int i = 0; i < 42; i++) red[i][tid] += red[i][tid + s];
    __syncthreads();
  }
  if (tid < 36) {
    const int r = tid / 6, c = tid % 6;
    double v = -red[tid][0];
    if (a == b) v += S.Hpp[36 * a + tid] + (r == c ? lambda : 0.0);
    S.S[(size_t)(6 * a + r) * n + 6 * b + c] = v;
    if (a != b) S.S[(size_t)(6 * b + c) * n + 6 * a + r] = v;
  }
  if (a == b && tid < 6) S.x[6 * a + tid] = S.bp[6 * a + tid] - red[36 + tid][0];  // bs into x (solved in place)
}

// ---------------------------------------------------------------------------
// Dense Cholesky of the reduced camera system, one workgroup (n = 6K <= 384).
// Right-looking, lower triangle in place; rhs in x[0:n) overwritten by the solution.
// ---------------------------------------------------------------------------
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
  // L y = b
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
  // L^T x = y
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

// xl = Dinv (bl - sum_e Hpl_e^T xp)
__global__ __launch_bounds__(256) void backsub_kernel(Problem P, Lin L, Active A, Sys S) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.nL) return;
  double* xl = S.x + 6 * A.K + 4 * g;
  if (!A.lm_act[g] || *S.fail) {
    for (int i = 0; i < 4; i++) xl[i] = 0;
    return;
  }
  const int ld = g < P.nq ? 3 : 4;
  double c[4];
  for (int i = 0; i < ld; i++) c[i] = S.bl[4 * g + i];
  for (int k = A.lm_off[g]; k < A.lm_off[g + 1]; k++) {
    const int e = A.lm_edges[k];
    const int a = A.pidx[P.epose[e]];
    if (a < 0) continue;
    const double* B = L.Hpl + 24 * e;
    for (int j = 0; j < ld; j++) {
      double s = 0;
      for (int i = 0; i < 6; i++) s += B[i * 4 + j] * S.x[6 * a + i];
      c[j] -= s;
    }
  }
  const double* D = S.Dinv + 16 * g;
  for (int i = 0; i < ld; i++) {
    double s = 0;
    for (int j = 0; j < ld; j++) s += D[i * ld + j] * c[j];
    xl[i] = s;
  }
  for (int i = ld; i < 4; i++) xl[i] = 0;
}

// oplus: poses T <- exp(x) T, points += x, lines oplus(x)
__global__ __launch_bounds__(256) void apply_kernel(Problem P, Active A, Sys S) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (*S.fail) return;
  if (i < A.K) {
    double* Tp = P.T + 8 * A.pose_of[i];
    const SE3 T = load_T(Tp);
    const SE3 r = se3_mul(se3_exp(S.x + 6 * i), T);
    for (int k = 0; k < 4; k++) Tp[k] = r.q[k];
    for (int k = 0; k < 3; k++) Tp[4 + k] = r.t[k];
  } else if (i < A.K + A.nL) {
    const int g = i - A.K;
    if (!A.lm_act[g]) return;
    const double* xl = S.x + 6 * A.K + 4 * g;
    if (g < P.nq) {
      for (int k = 0; k < 3; k++) P.X[3 * g + k] += xl[k];
    } else {
      line_oplus(P.L + 6 * (g - P.nq), xl);
    }
  }
}

// chi2 = sum of block partials (fixed order); scale = x.(lambda x + b) over active vertices
__global__ __launch_bounds__(256) void finish_kernel(Problem P, Active A, Sys S, int nblocks, int with_scale,
                                                     double lambda) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double c = 0;
  for (int i = tid; i < nblocks; i += 256) c += S.partial[i];
  red[tid] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  if (tid == 0) S.out[0] = red[0];
  __syncthreads();
  if (!with_scale) return;
  double sc = 0;
  for (int i = tid; i < 6 * A.K; i += 256) sc += S.x[i] * (lambda * S.x[i] + S.bp[i]);
  for (int g = tid; g < A.nL; g += 256) {
    if (!A.lm_act[g]) continue;
    const int ld = g < P.nq ? 3 : 4;
    for (int k = 0; k < ld; k++) {
      const double xv = S.x[6 * A.K + 4 * g + k];
      sc += xv * (lambda * xv + S.bl[4 * g + k]);
    }
  }
  red[tid] = sc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  if (tid == 0) {
    S.out[1] = red[0];
    S.out[3] = (double)*S.fail;
  }
}

// outlier levels after the first optimize / final inlier flags (g2o_optimization.cc:176-231)
__global__ __launch_bounds__(256) void classify_kernel(Problem P, Lin L, int E, uint8_t* level, uint8_t* inlier,
                                                       int final_pass) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int t = P.etype[e];
  double chi2 = 0;
  for (int k = 0; k < edim(t); k++) chi2 += L.err[4 * e + k] * L.err[4 * e + k];
  chi2 *= einfo(t);
  bool depth_ok = true;
  if (t < 2) {
    const SE3 T = load_T(P.T + 8 * P.epose[e]);
    double R[9], Xc[3];
    q_to_R(T.q, R);
    mat3_vec(R, P.X + 3 * P.elm[e], Xc);
    depth_ok = Xc[2] + T.t[2] > 0.0;
  }
  if (!final_pass) {
    if (chi2 > P.th[t] || !depth_ok) level[e] = 1;
  } else {
    inlier[e] = (chi2 <= P.th[t] && depth_ok) ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
int errors_blocks(int Ea) { return (Ea + 255) / 256; }

hipError_t compute_errors(const Problem& P, const Lin& L, const Active& A, Sys& S, int nblocks, hipStream_t s) {
  if (nblocks > 0) hipLaunchKernelGGL(errors_kernel, dim3(nblocks), dim3(256), 0, s, P, L, A, S.partial);
  hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(256), 0, s, P, A, S, nblocks, 0, 0.0);
  return hipGetLastError();
}

hipError_t linearize(const Problem& P, const Lin& L, const Active& A, hipStream_t s) {
  if (A.Ea > 0) hipLaunchKernelGGL(linearize_kernel, dim3((A.Ea + 127) / 128), dim3(128), 0, s, P, L, A);
  return hipGetLastError();
}

hipError_t reduce_blocks(const Problem& P, const Lin& L, const Active& A, Sys& S, hipStream_t s) {
  if (A.nL > 0) hipLaunchKernelGGL(landmark_reduce_kernel, dim3((A.nL + 255) / 256), dim3(256), 0, s, P, L, A, S);
  if (A.K > 0) hipLaunchKernelGGL(pose_reduce_kernel, dim3(A.K), dim3(128), 0, s, P, L, A, S);
  return hipGetLastError();
}

hipError_t schur(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s) {
  if (A.nL > 0)
    hipLaunchKernelGGL(landmark_schur_kernel, dim3((A.nL + 255) / 256), dim3(256), 0, s, P, L, A, S, lambda);
  if (A.npairs > 0) hipLaunchKernelGGL(pair_schur_kernel, dim3(A.npairs), dim3(128), 0, s, P, L, A, S, lambda);
  return hipGetLastError();
}

hipError_t solve_update(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s) {
  if (A.K > 0) hipLaunchKernelGGL(cholesky_kernel, dim3(1), dim3(256), 0, s, S, 6 * A.K);
  if (A.nL > 0) hipLaunchKernelGGL(backsub_kernel, dim3((A.nL + 255) / 256), dim3(256), 0, s, P, L, A, S);
  const int n = A.K + A.nL;
  if (n > 0) hipLaunchKernelGGL(apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, P, A, S);
  const int nb = errors_blocks(A.Ea);
  if (nb > 0) hipLaunchKernelGGL(errors_kernel, dim3(nb), dim3(256), 0, s, P, L, A, S.partial);
  hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(256), 0, s, P, A, S, nb, 1, lambda);
  return hipGetLastError();
}

hipError_t classify(const Problem& P, const Lin& L, int E, uint8_t* level, uint8_t* inlier, int final_pass,
                    hipStream_t s) {
  if (E > 0) hipLaunchKernelGGL(classify_kernel, dim3((E + 255) / 256), dim3(256), 0, s, P, L, E, level, inlier,
                                final_pass);
  return hipGetLastError();
}

}  // namespace ba
}  // namespace rspl
