// SE3Quat pieces shared by the BA kernels (ba_kernels.hip, frame_kernels.hip): g2o's
// SE3Quat (q w x y z, t), its normalisation, product and exp map (update [omega; upsilon]).
#pragma once
#include <hip/hip_runtime.h>

namespace rspl {
namespace ba {

struct SE3 {
  double q[4];  // w x y z
  double t[3];
};

// x^3 rounded once: the exact product as a double-double (FMA error terms), then one rounding -- the
// correctly rounded cube (0 misses against __float128 over 2e7 arguments in [-1, 1]; glibc's pow(x, 3),
// the CPU restatement's, misses correct rounding by an ulp in 0.08 % of them), in ~6 instructions instead
// of a device pow (log + exp) on the LM decision's chain (OptimizationAlgorithmLevenberg:
// 1 - pow(2 rho - 1, 3))
__device__ __forceinline__ double cube(double x) {
  const double p = x * x, pe = fma(x, x, -p);  // x^2 = p + pe exactly
  const double r = p * x, re = fma(p, x, -r);  // p x = r + re exactly
  return r + fma(pe, x, re);                   // x^3 = r + re + pe x (pe x's own rounding is far below r's ulp)
}

__device__ __forceinline__ void q_to_R(const double* q, double* R) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
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
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  o[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  o[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  o[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
}

__device__ __forceinline__ void se3_normalize(SE3& T) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
  if (T.q[0] < 0)
    for (int i = 0; i < 4; i++) T.q[i] = -T.q[i];
  const double n = sqrt(T.q[0] * T.q[0] + T.q[1] * T.q[1] + T.q[2] * T.q[2] + T.q[3] * T.q[3]);
  for (int i = 0; i < 4; i++) T.q[i] /= n;
}

__device__ __forceinline__ void R_to_q(const double* m, double* q) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
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
    if (m[8] > (i == 0 ? m[0] : m[4])) i = 2;
    // (i, j, k) cyclic; each case spelled out so every index is a constant (no scratch)
    auto branch = [&](int ii, int jj, int kk, double* v) {
      double s = sqrt(m[ii * 3 + ii] - m[jj * 3 + jj] - m[kk * 3 + kk] + 1.0);
      v[ii] = 0.5 * s;
      s = 0.5 / s;
      q[0] = (m[kk * 3 + jj] - m[jj * 3 + kk]) * s;
      v[jj] = (m[jj * 3 + ii] + m[ii * 3 + jj]) * s;
      v[kk] = (m[kk * 3 + ii] + m[ii * 3 + kk]) * s;
    };
    double v[3];
    if (i == 0) branch(0, 1, 2, v);
    else if (i == 1) branch(1, 2, 0, v);
    else branch(2, 0, 1, v);
    q[1] = v[0]; q[2] = v[1]; q[3] = v[2];
  }
}

__device__ __forceinline__ SE3 se3_mul(const SE3& a, const SE3& b) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
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
__device__ inline SE3 se3_exp(const double* u) {
  #pragma clang fp contract(off)  // bit-identical to the CPU restatement (oracle/ba.c, -ffp-contract=off)
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

}  // namespace ba
}  // namespace rspl
