/*
 * ORACLE (test infrastructure only) -- fp64 CPU restatement of SolvePnPWithCV
 * (src/g2o_optimization/g2o_optimization.cc:402-461): cv::solvePnPRansac(object_points,
 * image_points, K, zero distortion, rvec, tvec, false, 100 iterations, 20 px, 0.99) with the
 * default SOLVEPNP_ITERATIVE flags, i.e. RANSAC over 5-point EPnP hypotheses followed by an
 * iterative refinement on the inliers.  OpenCV is a third-party library that is NOT vendored
 * in the reference (version unpinned; absent from this image): the restated pieces are its
 * published algorithms, so parity at the OpenCV boundary is UNPINNED.  Restated:
 *  - cv::RNG (multiply-with-carry, coefficient 4164903690, state seeded with (uint64)-1 by
 *    RANSACPointSetRegistrator::run) and getSubset (5 distinct uniform indices, redraw on a
 *    repeat);
 *  - EPnP (Lepetit et al.; OpenCV's epnp class): PCA control points, barycentric alphas,
 *    M^T M eigenvectors, L_6x10 / rho, beta approximations 1-3 + 5 Gauss-Newton steps,
 *    Procrustes R, t, the solution with the lowest mean reprojection error;
 *  - inliers: squared reprojection error <= reprojection_error^2; adaptive iteration count
 *    RANSACUpdateNumIters(confidence, outlier ratio, 5, niters); a hypothesis replaces the
 *    best only with strictly more inliers than max(best, 4);
 *  - final refinement: Levenberg-Marquardt on the inliers' reprojection error (the optimum
 *    OpenCV's iterative solvePnP converges to), from the best hypothesis;
 *  - the wrapper: < 8 correspondences -> 0 (:433), Twc = [Rcw^T | -Rcw^T tcw] (:448-450).
 * Object / image points are rounded to float first: the reference builds cv::Point3f /
 * cv::Point2f (:425-426).
 */
/* no FMA contraction (the GPU kernel's rule, pnp_kernels.hip): EPnP's 5-point null space is
   degenerate, and the basis the Jacobi leaves in it follows every rounding difference.  The
   Makefile builds with -ffp-contract=off (gcc does not implement the standard pragma; clang does). */
#if defined(__clang__)
#pragma STDC FP_CONTRACT OFF
#endif
#include <float.h>
#include <math.h>

#include "../include/rspl.h"
#include "oracle_common.h"

/* ---------------- cv::RNG / getSubset ---------------- */
static unsigned rng_next(uint64_t* s) {
  *s = (uint64_t)(unsigned)*s * 4164903690u + (unsigned)(*s >> 32);
  return (unsigned)*s;
}

void orc_pnp_subsets(int count, int iters, int32_t* idx /* [iters][5] */) {
  uint64_t s = (uint64_t)-1;
  for (int h = 0; h < iters; h++) {
    int32_t* o = idx + 5 * h;
    for (int i = 0; i < 5; i++) {
      int v;
      for (;;) {
        v = (int)(rng_next(&s) % (unsigned)count);
        int dup = 0;
        for (int j = 0; j < i; j++) dup |= o[j] == v;
        if (!dup) break;
      }
      o[i] = v;
    }
  }
}

/* ---------------- small dense linear algebra ---------------- */
/* cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (n <= 12; used for n = 3): eigenvalues
   descending in d, eigenvectors as ROWS of V (cvSVD's U^T order) */
static void jacobi_eig(int n, const double* A0, double* d, double* V) {
  double A[144], U[144];
  memcpy(A, A0, sizeof(double) * n * n);
  for (int i = 0; i < n * n; i++) U[i] = (i / n == i % n) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0, tot = 0;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) {
        tot += A[i * n + j] * A[i * n + j];
        if (i != j) off += A[i * n + j] * A[i * n + j];
      }
    if (off <= 1e-30 * tot || off == 0.0) break;
    for (int p = 0; p < n - 1; p++)
      for (int q = p + 1; q < n; q++) {
        const double apq = A[p * n + q];
        if (apq == 0.0) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; k++) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; k++) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; k++) {
          const double ukp = U[k * n + p], ukq = U[k * n + q];
          U[k * n + p] = c * ukp - s * ukq;
          U[k * n + q] = s * ukp + c * ukq;
        }
      }
  }
  /* selection sort, descending */
  int ord[12];
  for (int i = 0; i < n; i++) ord[i] = i;
  for (int i = 0; i < n; i++) {
    int b = i;
    for (int j = i + 1; j < n; j++)
      if (A[ord[j] * n + ord[j]] > A[ord[b] * n + ord[b]]) b = j;
    const int t = ord[i];
    ord[i] = ord[b];
    ord[b] = t;
  }
  for (int i = 0; i < n; i++) {
    d[i] = A[ord[i] * n + ord[i]];
    for (int k = 0; k < n; k++) V[i * n + k] = U[k * n + ord[i]];
  }
}

/* Jacobi eigen-decomposition of the symmetric 12 x 12 M^T M in the parallel (round-robin)
   order: a sweep is 11 rounds of 6 disjoint rotations, index 11 fixed and 0..10 on a circle
   (round r: (r, 11) and ((r + k) % 11, (r - k) % 11), k = 1..5).  Each round takes its 6
   angles from the matrix at the round's start, then applies every column rotation, then
   every row rotation, then the eigenvector columns -- the operation order of the GPU's
   wave-cooperative solver (pnp_kernels.hip: one rotation pair per lane group).  The sweep
   test sums the squares in the GPU's order (per-lane partials over elements lane + 64 m,
   then a butterfly over the 64 lanes).  cvSVD's own Jacobi order is OpenCV's (unpinned);
   any converged Jacobi gives the same eigenvectors up to rounding and sign, which EPnP's
   beta solve and solve_for_sign absorb.  Output as jacobi_eig. */
/* the rotation annihilating a_pq from d = a_qq - a_pp, h = 2 a_pq != 0: the classic
   theta = d / h, t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), c = 1 / sqrt(t^2 + 1), s = t c
   rewritten with g = sqrt(d^2 + h^2) as t = sgn(theta) |h| / (|d| + g), c = sqrt((|d| + g) / (2 g))
   -- the same rotation, three dependent sqrt / divide steps instead of five (the GPU's round
   latency); sgn(theta) = +1 for theta = +-0 as in the classic test theta >= 0 */
static void jacobi_cs(double d, double h, double* c, double* s) {
  const double g = sqrt(d * d + h * h);
  const double sg = d == 0.0 ? 1.0 : ((d > 0) == (h > 0) ? 1.0 : -1.0);
  const double t = sg * fabs(h) / (fabs(d) + g);
  *c = sqrt((fabs(d) + g) / (2.0 * g));
  *s = t * *c;
}

static void jacobi12_rounds(const double* A0, double* d, double* V) {
  enum { n = 12 };
  double A[144], U[144];
  memcpy(A, A0, sizeof(A));
  for (int i = 0; i < 144; i++) U[i] = (i / n == i % n) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; sweep++) {
    double po[64], pt[64];
    for (int l = 0; l < 64; l++) {
      po[l] = pt[l] = 0.0;
      for (int e = l; e < 144; e += 64) {
        const double v = A[e] * A[e];
        pt[l] += v;
        if (e / n != e % n) po[l] += v;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {
      double qo[64], qt[64];
      for (int l = 0; l < 64; l++) {
        qo[l] = po[l] + po[l ^ o];
        qt[l] = pt[l] + pt[l ^ o];
      }
      memcpy(po, qo, sizeof(po));
      memcpy(pt, qt, sizeof(pt));
    }
    const double off = po[0], tot = pt[0];
    if (off <= 1e-30 * tot || off == 0.0) break;
    for (int r = 0; r < 11; r++) {
      int pp[6], qq[6], act[6];
      double cc[6], ss[6];
      for (int j = 0; j < 6; j++) {
        int a = j == 0 ? r : (r + j) % 11, b = j == 0 ? 11 : (r - j + 11) % 11;
        pp[j] = a < b ? a : b;
        qq[j] = a < b ? b : a;
        const int p = pp[j], q = qq[j];
        const double apq = A[p * n + q];
        act[j] = apq != 0.0;
        cc[j] = 1.0;
        ss[j] = 0.0;
        if (!act[j]) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        jacobi_cs(aqq - app, 2.0 * apq, &cc[j], &ss[j]);
      }
      for (int j = 0; j < 6; j++) {
        if (!act[j]) continue;
        const int p = pp[j], q = qq[j];
        const double c = cc[j], s = ss[j];
        for (int k = 0; k < n; k++) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
      }
      for (int j = 0; j < 6; j++) {
        if (!act[j]) continue;
        const int p = pp[j], q = qq[j];
        const double c = cc[j], s = ss[j];
        for (int k = 0; k < n; k++) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
      }
      for (int j = 0; j < 6; j++) {
        if (!act[j]) continue;
        const int p = pp[j], q = qq[j];
        const double c = cc[j], s = ss[j];
        for (int k = 0; k < n; k++) {
          const double ukp = U[k * n + p], ukq = U[k * n + q];
          U[k * n + p] = c * ukp - s * ukq;
          U[k * n + q] = s * ukp + c * ukq;
        }
      }
    }
  }
  int ord[12];
  for (int i = 0; i < n; i++) ord[i] = i;
  for (int i = 0; i < n; i++) {
    int b = i;
    for (int j = i + 1; j < n; j++)
      if (A[ord[j] * n + ord[j]] > A[ord[b] * n + ord[b]]) b = j;
    const int t = ord[i];
    ord[i] = ord[b];
    ord[b] = t;
  }
  for (int i = 0; i < n; i++) {
    d[i] = A[ord[i] * n + ord[i]];
    for (int k = 0; k < n; k++) V[i * n + k] = U[k * n + ord[i]];
  }
}

/* least squares min |A x - b| (A m x n, m >= n, row-major) by Householder QR */
static int lsq_qr(int m, int n, const double* A0, const double* b0, double* x) {
  double A[6 * 5], b[6];
  memcpy(A, A0, sizeof(double) * m * n);
  memcpy(b, b0, sizeof(double) * m);
  for (int k = 0; k < n; k++) {
    double nrm = 0;
    for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
    nrm = sqrt(nrm);
    if (nrm == 0.0) return -1;
    const double alpha = A[k * n + k] > 0 ? -nrm : nrm;
    double v[6];
    for (int i = 0; i < m; i++) v[i] = i < k ? 0.0 : A[i * n + k];
    v[k] -= alpha;
    double vv = 0;
    for (int i = k; i < m; i++) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    for (int j = k; j < n; j++) {
      double s = 0;
      for (int i = k; i < m; i++) s += v[i] * A[i * n + j];
      s *= 2.0 / vv;
      for (int i = k; i < m; i++) A[i * n + j] -= s * v[i];
    }
    double s = 0;
    for (int i = k; i < m; i++) s += v[i] * b[i];
    s *= 2.0 / vv;
    for (int i = k; i < m; i++) b[i] -= s * v[i];
  }
  for (int k = n - 1; k >= 0; k--) {
    double s = b[k];
    for (int j = k + 1; j < n; j++) s -= A[k * n + j] * x[j];
    if (A[k * n + k] == 0.0) return -1;
    x[k] = s / A[k * n + k];
  }
  return 0;
}

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* 3x3 SVD via the symmetric eigen-problem of A^T A: A = U diag(s) V^T */
static void svd3(const double* A, double* U, double* V) {
  double AtA[9], d[3], Vt[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += A[k * 3 + i] * A[k * 3 + j];
      AtA[i * 3 + j] = s;
    }
  jacobi_eig(3, AtA, d, Vt); /* rows of Vt = right singular vectors */
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) V[i * 3 + j] = Vt[j * 3 + i];
  for (int c = 0; c < 2; c++) { /* u_c = A v_c / |A v_c| */
    double u[3];
    for (int i = 0; i < 3; i++) u[i] = A[i * 3 + 0] * V[0 * 3 + c] + A[i * 3 + 1] * V[1 * 3 + c] + A[i * 3 + 2] * V[2 * 3 + c];
    const double nu = sqrt(dot3(u, u));
    for (int i = 0; i < 3; i++) U[i * 3 + c] = nu > 0 ? u[i] / nu : (i == c ? 1.0 : 0.0);
  }
  /* u_2 = u_0 x u_1 (orientation fixed below by the determinant check) */
  const double u0[3] = {U[0], U[3], U[6]}, u1[3] = {U[1], U[4], U[7]};
  double u2[3] = {u0[1] * u1[2] - u0[2] * u1[1], u0[2] * u1[0] - u0[0] * u1[2], u0[0] * u1[1] - u0[1] * u1[0]};
  double Av2[3];
  for (int i = 0; i < 3; i++) Av2[i] = A[i * 3 + 0] * V[2] + A[i * 3 + 1] * V[5] + A[i * 3 + 2] * V[8];
  if (dot3(Av2, u2) < 0) for (int i = 0; i < 3; i++) u2[i] = -u2[i];
  for (int i = 0; i < 3; i++) U[i * 3 + 2] = u2[i];
}

/* ---------------- EPnP ---------------- */
typedef struct {
  int n;
  double fu, fv, uc, vc;
  double pws[3 * 8], us[2 * 8], alphas[4 * 8], pcs[3 * 8];
  double cws[4][3], ccs[4][3];
} epnp_t;

static void epnp_control_points(epnp_t* E) {
  for (int j = 0; j < 3; j++) {
    double s = 0;
    for (int i = 0; i < E->n; i++) s += E->pws[3 * i + j];
    E->cws[0][j] = s / E->n;
  }
  double M[9] = {0}, d[3], Vt[9];
  for (int i = 0; i < E->n; i++) {
    double p[3];
    for (int j = 0; j < 3; j++) p[j] = E->pws[3 * i + j] - E->cws[0][j];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) M[a * 3 + b] += p[a] * p[b];
  }
  jacobi_eig(3, M, d, Vt);
  for (int i = 1; i < 4; i++) {
    const double k = sqrt(fmax(d[i - 1], 0.0) / E->n);
    for (int j = 0; j < 3; j++) E->cws[i][j] = E->cws[0][j] + k * Vt[3 * (i - 1) + j];
  }
}

static int inv3(const double* m, double* o) {
  const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8], c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  if (det == 0.0) return -1;
  const double id = 1.0 / det;
  o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  o[3] = c01 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  o[6] = c02 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
  return 0;
}

static int epnp_barycentric(epnp_t* E) {
  double cc[9], ci[9];
  for (int i = 0; i < 3; i++)
    for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = E->cws[j][i] - E->cws[0][i];
  if (inv3(cc, ci)) return -1;
  for (int i = 0; i < E->n; i++) {
    const double* p = E->pws + 3 * i;
    double* a = E->alphas + 4 * i;
    for (int j = 0; j < 3; j++)
      a[1 + j] = ci[3 * j] * (p[0] - E->cws[0][0]) + ci[3 * j + 1] * (p[1] - E->cws[0][1]) + ci[3 * j + 2] * (p[2] - E->cws[0][2]);
    a[0] = 1.0 - a[1] - a[2] - a[3];
  }
  return 0;
}

static void epnp_L(const double* ut, double* L) {
  const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
  double dv[4][6][3];
  for (int i = 0; i < 4; i++) {
    int a = 0, b = 1;
    for (int j = 0; j < 6; j++) {
      for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
      b++;
      if (b > 3) { a++; b = a + 1; }
    }
  }
  for (int i = 0; i < 6; i++) {
    double* r = L + 10 * i;
    r[0] = dot3(dv[0][i], dv[0][i]);
    r[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
    r[2] = dot3(dv[1][i], dv[1][i]);
    r[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
    r[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
    r[5] = dot3(dv[2][i], dv[2][i]);
    r[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
    r[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
    r[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
    r[9] = dot3(dv[3][i], dv[3][i]);
  }
}

static double dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

static void betas_1(const double* L, const double* rho, double* be) {
  double A[24], b4[4] = {0};
  for (int i = 0; i < 6; i++) { A[4 * i] = L[10 * i]; A[4 * i + 1] = L[10 * i + 1]; A[4 * i + 2] = L[10 * i + 3]; A[4 * i + 3] = L[10 * i + 6]; }
  lsq_qr(6, 4, A, rho, b4);
  if (b4[0] < 0) {
    be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
  } else {
    be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
  }
}

static void betas_2(const double* L, const double* rho, double* be) {
  double A[18], b3[3] = {0};
  for (int i = 0; i < 6; i++) { A[3 * i] = L[10 * i]; A[3 * i + 1] = L[10 * i + 1]; A[3 * i + 2] = L[10 * i + 2]; }
  lsq_qr(6, 3, A, rho, b3);
  if (b3[0] < 0) { be[0] = sqrt(-b3[0]); be[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0; }
  else { be[0] = sqrt(b3[0]); be[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0; }
  if (b3[1] < 0) be[0] = -be[0];
  be[2] = 0.0;
  be[3] = 0.0;
}

static void betas_3(const double* L, const double* rho, double* be) {
  double A[30], b5[5] = {0};
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 5; j++) A[5 * i + j] = L[10 * i + j];
  lsq_qr(6, 5, A, rho, b5);
  if (b5[0] < 0) { be[0] = sqrt(-b5[0]); be[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0; }
  else { be[0] = sqrt(b5[0]); be[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0; }
  if (b5[1] < 0) be[0] = -be[0];
  be[2] = b5[3] / be[0];
  be[3] = 0.0;
}

static void gauss_newton(const double* L, const double* rho, double* be) {
  for (int it = 0; it < 5; it++) {
    double A[24], b[6], x[4] = {0, 0, 0, 0};
    for (int i = 0; i < 6; i++) {
      const double* r = L + 10 * i;
      A[4 * i + 0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
      A[4 * i + 1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
      A[4 * i + 2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
      A[4 * i + 3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
      b[i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] + r[3] * be[0] * be[2] +
                       r[4] * be[1] * be[2] + r[5] * be[2] * be[2] + r[6] * be[0] * be[3] + r[7] * be[1] * be[3] +
                       r[8] * be[2] * be[3] + r[9] * be[3] * be[3]);
    }
    if (lsq_qr(6, 4, A, b, x)) return;
    for (int i = 0; i < 4; i++) be[i] += x[i];
  }
}

static double epnp_R_t(epnp_t* E, const double* ut, const double* be, double R[9], double t[3]) {
  for (int j = 0; j < 4; j++)
    for (int k = 0; k < 3; k++) E->ccs[j][k] = 0.0;
  for (int i = 0; i < 4; i++) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; j++)
      for (int k = 0; k < 3; k++) E->ccs[j][k] += be[i] * v[3 * j + k];
  }
  for (int i = 0; i < E->n; i++) {
    const double* a = E->alphas + 4 * i;
    for (int j = 0; j < 3; j++)
      E->pcs[3 * i + j] = a[0] * E->ccs[0][j] + a[1] * E->ccs[1][j] + a[2] * E->ccs[2][j] + a[3] * E->ccs[3][j];
  }
  if (E->pcs[2] < 0.0) { /* solve_for_sign */
    for (int j = 0; j < 4; j++)
      for (int k = 0; k < 3; k++) E->ccs[j][k] = -E->ccs[j][k];
    for (int i = 0; i < 3 * E->n; i++) E->pcs[i] = -E->pcs[i];
  }
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
  for (int i = 0; i < E->n; i++)
    for (int j = 0; j < 3; j++) { pc0[j] += E->pcs[3 * i + j]; pw0[j] += E->pws[3 * i + j]; }
  for (int j = 0; j < 3; j++) { pc0[j] /= E->n; pw0[j] /= E->n; }
  double abt[9] = {0}, U[9], V[9];
  for (int i = 0; i < E->n; i++)
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 3; k++) abt[3 * j + k] += (E->pcs[3 * i + j] - pc0[j]) * (E->pws[3 * i + k] - pw0[k]);
  svd3(abt, U, V);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
  const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                     R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
  for (int i = 0; i < 3; i++) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
  double s2 = 0;
  for (int i = 0; i < E->n; i++) {
    const double* pw = E->pws + 3 * i;
    const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1], iz = 1.0 / (dot3(R + 6, pw) + t[2]);
    const double ue = E->uc + E->fu * Xc * iz, ve = E->vc + E->fv * Yc * iz;
    s2 += sqrt((E->us[2 * i] - ue) * (E->us[2 * i] - ue) + (E->us[2 * i + 1] - ve) * (E->us[2 * i + 1] - ve));
  }
  return s2 / E->n;
}

/* The eigen solver of M^T M: 0 = the GPU kernel's round-robin order (jacobi12_rounds, the GPU's CPU
   mirror: per-hypothesis bit parity), 1 = the classic cyclic Jacobi (jacobi_eig: an independent
   restatement, used by the RANSAC-level parity test -- hypotheses may then differ in the degenerate
   5-point null space, the RANSAC outcome on clean inliers may not). */
static int g_eig_indep = 0;

/* EPnP on n <= 8 correspondences; returns 0 and R (row-major), t on success */
static int epnp(const double* K4, int n, const double* pw, const double* uv, double R[9], double t[3]) {
  epnp_t E;
  memset(&E, 0, sizeof(E));
  E.n = n;
  E.fu = K4[0]; E.fv = K4[1]; E.uc = K4[2]; E.vc = K4[3];
  memcpy(E.pws, pw, sizeof(double) * 3 * n);
  memcpy(E.us, uv, sizeof(double) * 2 * n);
  epnp_control_points(&E);
  if (epnp_barycentric(&E)) return -1;
  double MtM[144] = {0};
  for (int i = 0; i < n; i++) {
    double M1[12], M2[12];
    const double* as = E.alphas + 4 * i;
    for (int k = 0; k < 4; k++) {
      M1[3 * k] = as[k] * E.fu; M1[3 * k + 1] = 0.0; M1[3 * k + 2] = as[k] * (E.uc - uv[2 * i]);
      M2[3 * k] = 0.0; M2[3 * k + 1] = as[k] * E.fv; M2[3 * k + 2] = as[k] * (E.vc - uv[2 * i + 1]);
    }
    for (int a = 0; a < 12; a++)
      for (int b = 0; b < 12; b++) MtM[a * 12 + b] += M1[a] * M1[b] + M2[a] * M2[b];
  }
  double d[12], ut[144];
  if (g_eig_indep) jacobi_eig(12, MtM, d, ut);
  else jacobi12_rounds(MtM, d, ut);
  double L[60], rho[6];
  epnp_L(ut, L);
  rho[0] = dist2(E.cws[0], E.cws[1]); rho[1] = dist2(E.cws[0], E.cws[2]); rho[2] = dist2(E.cws[0], E.cws[3]);
  rho[3] = dist2(E.cws[1], E.cws[2]); rho[4] = dist2(E.cws[1], E.cws[3]); rho[5] = dist2(E.cws[2], E.cws[3]);
  double be[4][4], Rs[4][9], ts[4][3], err[4];
  betas_1(L, rho, be[1]); gauss_newton(L, rho, be[1]); err[1] = epnp_R_t(&E, ut, be[1], Rs[1], ts[1]);
  betas_2(L, rho, be[2]); gauss_newton(L, rho, be[2]); err[2] = epnp_R_t(&E, ut, be[2], Rs[2], ts[2]);
  betas_3(L, rho, be[3]); gauss_newton(L, rho, be[3]); err[3] = epnp_R_t(&E, ut, be[3], Rs[3], ts[3]);
  int N = 1;
  if (err[2] < err[1]) N = 2;
  if (err[3] < err[N]) N = 3;
  if (!isfinite(err[N])) return -1;
  memcpy(R, Rs[N], sizeof(double) * 9);
  memcpy(t, ts[N], sizeof(double) * 3);
  return 0;
}

/* RANSACUpdateNumIters */
static int update_iters(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.), 1.);
  ep = fmin(fmax(ep, 0.), 1.);
  double num = fmax(1. - p, DBL_MIN);
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

static double reproj2(const double* K4, const double R[9], const double t[3], const double* p, const double* uv) {
  const double Xc = dot3(R, p) + t[0], Yc = dot3(R + 3, p) + t[1], Zc = dot3(R + 6, p) + t[2];
  const double iz = 1.0 / Zc;
  const double du = uv[0] - (K4[0] * Xc * iz + K4[2]), dv = uv[1] - (K4[1] * Yc * iz + K4[3]);
  return du * du + dv * dv;
}

/* Levenberg-Marquardt on the inliers' squared reprojection error, pose T_cw (R, t) with the
   left exp-map update; stops after 20 iterations or when a step no longer lowers the cost */
static void refine(const double* K4, int n, const double* pw, const double* uv, const uint8_t* inl, double R[9],
                   double t[3]) {
  double lambda = 1e-3;
  for (int it = 0; it < 20; it++) {
    double H[36] = {0}, g[6] = {0}, cost = 0;
    for (int i = 0; i < n; i++) {
      if (!inl[i]) continue;
      const double* p = pw + 3 * i;
      const double x = dot3(R, p) + t[0], y = dot3(R + 3, p) + t[1], z = dot3(R + 6, p) + t[2];
      const double iz = 1.0 / z, iz2 = iz * iz;
      const double e[2] = {uv[2 * i] - (K4[0] * x * iz + K4[2]), uv[2 * i + 1] - (K4[1] * y * iz + K4[3])};
      cost += e[0] * e[0] + e[1] * e[1];
      const double D[2][3] = {{K4[0] * iz, 0, -K4[0] * x * iz2}, {0, K4[1] * iz, -K4[1] * y * iz2}};
      const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
      double J[2][6];
      for (int r = 0; r < 2; r++)
        for (int c = 0; c < 3; c++) {
          double s = 0;
          for (int k = 0; k < 3; k++) s += D[r][k] * SX[k * 3 + c];
          J[r][c] = s;
          J[r][3 + c] = -D[r][c];
        }
      for (int a = 0; a < 6; a++) {
        g[a] += -(J[0][a] * e[0] + J[1][a] * e[1]);
        for (int b = 0; b < 6; b++) H[a * 6 + b] += J[0][a] * J[0][b] + J[1][a] * J[1][b];
      }
    }
    int accepted = 0;
    for (int trial = 0; trial < 10 && !accepted; trial++) {
      double A[36], x[6];
      memcpy(A, H, sizeof(A));
      for (int a = 0; a < 6; a++) A[a * 7] += lambda * fmax(H[a * 7], 1e-12);
      memcpy(x, g, sizeof(x));
      /* Cholesky */
      int ok = 1;
      for (int j = 0; j < 6 && ok; j++) {
        double s = A[j * 6 + j];
        for (int k = 0; k < j; k++) s -= A[j * 6 + k] * A[j * 6 + k];
        if (!(s > 0)) { ok = 0; break; }
        const double dd = sqrt(s);
        A[j * 6 + j] = dd;
        for (int i = j + 1; i < 6; i++) {
          double v = A[i * 6 + j];
          for (int k = 0; k < j; k++) v -= A[i * 6 + k] * A[j * 6 + k];
          A[i * 6 + j] = v / dd;
        }
      }
      if (!ok) { lambda *= 10; continue; }
      for (int i = 0; i < 6; i++) { double s = x[i]; for (int k = 0; k < i; k++) s -= A[i * 6 + k] * x[k]; x[i] = s / A[i * 7]; }
      for (int i = 5; i >= 0; i--) { double s = x[i]; for (int k = i + 1; k < 6; k++) s -= A[k * 6 + i] * x[k]; x[i] = s / A[i * 7]; }
      /* candidate: R' = exp(w) R, t' = exp(w) t + V v  (SE3 left update) */
      const double* w = x;
      const double th = sqrt(dot3(w, w));
      const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
      double O2[9];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) O2[a * 3 + b] = O[a * 3] * O[b] + O[a * 3 + 1] * O[3 + b] + O[a * 3 + 2] * O[6 + b];
      double ca, cb, cc, cd;
      if (th < 1e-5) { ca = 1.0; cb = 0.5; cc = 0.5; cd = 1.0 / 6.0; }
      else { ca = sin(th) / th; cb = (1 - cos(th)) / (th * th); cc = cb; cd = (th - sin(th)) / (th * th * th); }
      double dR[9], Vm[9], Rn[9], tn[3], dt[3];
      for (int k = 0; k < 9; k++) {
        const double I = (k % 4 == 0) ? 1.0 : 0.0;
        dR[k] = I + ca * O[k] + cb * O2[k];
        Vm[k] = I + cc * O[k] + cd * O2[k];
      }
      for (int a = 0; a < 3; a++) {
        dt[a] = dot3(Vm + 3 * a, x + 3);
        for (int b = 0; b < 3; b++) Rn[a * 3 + b] = dR[a * 3] * R[b] + dR[a * 3 + 1] * R[3 + b] + dR[a * 3 + 2] * R[6 + b];
      }
      for (int a = 0; a < 3; a++) tn[a] = dot3(dR + 3 * a, t) + dt[a];
      double cn = 0;
      for (int i = 0; i < n; i++)
        if (inl[i]) cn += reproj2(K4, Rn, tn, pw + 3 * i, uv + 2 * i);
      if (cn < cost) {
        memcpy(R, Rn, sizeof(Rn));
        memcpy(t, tn, sizeof(tn));
        lambda = fmax(lambda * 0.1, 1e-12);
        accepted = 1;
        if (cost - cn <= 1e-14 * cost) return;
      } else {
        lambda *= 10;
      }
    }
    if (!accepted) return;
  }
}

/* the eigen solver for the following orc_pnp / orc_pnp_hypotheses calls (see g_eig_indep) */
void orc_pnp_set_solver(int independent) { g_eig_indep = independent != 0; }

/* returns the inlier count (0: fewer than 8 correspondences or no model); Twc out */
int orc_pnp(const double* K4, int n, const double* pts3, const double* pts2, int iterations, double reproj_err,
            double confidence, double* Rwc, double* twc, uint8_t* inlier, int* hyps_used) {
  if (hyps_used) *hyps_used = 0;
  for (int i = 0; i < n; i++) inlier[i] = 0;
  if (n < 8) return 0; /* (:433) */
  double* pw = (double*)malloc(sizeof(double) * 3 * n);
  double* uv = (double*)malloc(sizeof(double) * 2 * n);
  for (int i = 0; i < 3 * n; i++) pw[i] = (double)(float)pts3[i]; /* cv::Point3f */
  for (int i = 0; i < 2 * n; i++) uv[i] = (double)(float)pts2[i]; /* cv::Point2f */
  int32_t* sub = (int32_t*)malloc(sizeof(int32_t) * 5 * iterations);
  orc_pnp_subsets(n, iterations, sub);
  const double thr2 = reproj_err * reproj_err;
  int best = -1, best_cnt = 0, niters = iterations, h = 0;
  double bR[9], bt[3];
  for (h = 0; h < niters; h++) {
    double sp[15], su[10], R[9], t[3];
    for (int k = 0; k < 5; k++) {
      memcpy(sp + 3 * k, pw + 3 * sub[5 * h + k], sizeof(double) * 3);
      memcpy(su + 2 * k, uv + 2 * sub[5 * h + k], sizeof(double) * 2);
    }
    if (epnp(K4, 5, sp, su, R, t)) continue;
    int cnt = 0;
    for (int i = 0; i < n; i++) cnt += reproj2(K4, R, t, pw + 3 * i, uv + 2 * i) <= thr2;
    if (cnt > (best_cnt > 4 ? best_cnt : 4)) {
      best = h;
      best_cnt = cnt;
      memcpy(bR, R, sizeof(bR));
      memcpy(bt, t, sizeof(bt));
      niters = update_iters(confidence, (double)(n - cnt) / n, 5, niters);
    }
  }
  if (hyps_used) *hyps_used = h;
  int ninl = 0;
  if (best >= 0) {
    for (int i = 0; i < n; i++) {
      inlier[i] = reproj2(K4, bR, bt, pw + 3 * i, uv + 2 * i) <= thr2;
      ninl += inlier[i];
    }
    refine(K4, n, pw, uv, inlier, bR, bt);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) Rwc[3 * i + j] = bR[3 * j + i];
    for (int i = 0; i < 3; i++) twc[i] = -(Rwc[3 * i] * bt[0] + Rwc[3 * i + 1] * bt[1] + Rwc[3 * i + 2] * bt[2]);
  }
  free(pw); free(uv); free(sub);
  return ninl;
}

/* every hypothesis of orc_pnp's RANSAC (test infrastructure: per-hypothesis parity): the
   inlier count (-1: the minimal solver failed) and R (row-major) | t of each of `iterations`
   subsets, all evaluated (no adaptive stop) */
void orc_pnp_hypotheses(const double* K4, int n, const double* pts3, const double* pts2, int iterations,
                        double reproj_err, int32_t* counts, double* poses) {
  double* pw = (double*)malloc(sizeof(double) * 3 * (n > 0 ? n : 1));
  double* uv = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
  for (int i = 0; i < 3 * n; i++) pw[i] = (double)(float)pts3[i];
  for (int i = 0; i < 2 * n; i++) uv[i] = (double)(float)pts2[i];
  int32_t* sub = (int32_t*)malloc(sizeof(int32_t) * 5 * iterations);
  orc_pnp_subsets(n, iterations, sub);
  const double thr2 = reproj_err * reproj_err;
  for (int h = 0; h < iterations; h++) {
    double sp[15], su[10], R[9] = {0}, t[3] = {0};
    for (int k = 0; k < 5; k++) {
      memcpy(sp + 3 * k, pw + 3 * sub[5 * h + k], sizeof(double) * 3);
      memcpy(su + 2 * k, uv + 2 * sub[5 * h + k], sizeof(double) * 2);
    }
    int cnt = -1;
    if (!epnp(K4, 5, sp, su, R, t)) {
      cnt = 0;
      for (int i = 0; i < n; i++) cnt += reproj2(K4, R, t, pw + 3 * i, uv + 2 * i) <= thr2;
    }
    counts[h] = cnt;
    memcpy(poses + 12 * h, R, sizeof(R));
    memcpy(poses + 12 * h + 9, t, sizeof(t));
  }
  free(pw); free(uv); free(sub);
}
