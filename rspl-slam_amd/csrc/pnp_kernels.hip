// SolvePnPWithCV (src/g2o_optimization/g2o_optimization.cc:402-461) on gfx950: OpenCV's
// solvePnPRansac(100 iterations, 20 px, 0.99, SOLVEPNP_ITERATIVE) for a batch of frames in two
// launches:
//   1. pnp_hyp_kernel: ONE WAVE PER RANSAC HYPOTHESIS (4 per 256-thread workgroup, grid
//      hypotheses/4 x frames): 5-point EPnP -- PCA control points and barycentric alphas
//      (every lane, registers), M^T M built by the lanes into LDS, its 12 x 12 Jacobi
//      eigen-decomposition cooperatively in LDS (round-robin order: 6 disjoint rotations per
//      round, the lanes apply every element's column / row / eigenvector update), beta
//      approximations 1-3 + Gauss-Newton and Procrustes (every lane, registers) -- then the
//      hypothesis' inlier count over the frame's correspondences (lanes strided, wave sum).
//      The 100 minimal solves OpenCV runs one after another run side by side, each on a wave.
//   2. pnp_final_kernel (one wave per frame): RANSAC's sequential acceptance over the
//      hypotheses in order (strictly more inliers than max(best, 4), adaptive iteration count
//      RANSACUpdateNumIters), the best hypothesis' inliers, and the Levenberg-Marquardt
//      refinement on their reprojection error (wave-reduced 6x6 normal equations).
// The hypothesis subsets come from the host's cv::RNG restatement (pnp.cpp).  Same algorithm,
// same Jacobi order, as the CPU restatement orc_pnp (oracle/pnp.c).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "pnp_kernels.hpp"
#include "wave_reduce.hpp"

// No FMA contraction in this file: EPnP on 5 points has a degenerate (>= 2-dimensional) null
// space, so the basis the Jacobi rotations leave there -- and with it the beta approximations --
// changes with any rounding difference.  Hypothesis parity with the oracle (compiled with the
// same rule, oracle/pnp.c) therefore needs the same IEEE operations in the same order.
#pragma clang fp contract(off)

namespace rspl {
namespace pnp {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* ---------------- small dense linear algebra, register resident (static sizes) ---------------- */
/* cyclic Jacobi eigen-decomposition of a symmetric 3 x 3 matrix: eigenvalues descending in d,
   eigenvectors as ROWS of V (oracle jacobi_eig(3, ...)) */
__device__ __forceinline__ void jacobi3(const double (&A0)[9], double (&d)[3], double (&V)[9]) {
  constexpr int n = 3;
  double A[9], U[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    A[i] = A0[i];
    U[i] = (i / n == i % n) ? 1.0 : 0.0;
  }
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
      for (int j = 0; j < n; j++) {
        tot += A[i * n + j] * A[i * n + j];
        if (i != j) off += A[i * n + j] * A[i * n + j];
      }
    if (off <= 1e-30 * tot || off == 0.0) break;
#pragma unroll
    for (int p = 0; p < n - 1; p++)
#pragma unroll
      for (int q = p + 1; q < n; q++) {
        const double apq = A[p * n + q];
        if (apq == 0.0) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
        for (int k = 0; k < n; k++) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
#pragma unroll
        for (int k = 0; k < n; k++) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
#pragma unroll
        for (int k = 0; k < n; k++) {
          const double ukp = U[k * n + p], ukq = U[k * n + q];
          U[k * n + p] = c * ukp - s * ukq;
          U[k * n + q] = s * ukp + c * ukq;
        }
      }
  }
  // descending order (selection sort of the oracle; distinct eigenvalues give the same order)
  double key[3] = {A[0], A[4], A[8]}, col[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) col[i][k] = U[k * n + i];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = i + 1; j < 3; j++) {
      const bool sw = key[j] > key[i];
      const double a = key[i], b = key[j];
      key[i] = sw ? b : a;
      key[j] = sw ? a : b;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const double u = col[i][k], v = col[j][k];
        col[i][k] = sw ? v : u;
        col[j][k] = sw ? u : v;
      }
    }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    d[i] = key[i];
#pragma unroll
    for (int k = 0; k < 3; k++) V[i * 3 + k] = col[i][k];
  }
}

/* least squares min |A x - b| (A m x n, m >= n, row-major) by Householder QR */
template <int m, int n>
__device__ __forceinline__ int lsq_qr(const double (&A0)[m * n], const double (&b0)[m], double (&x)[n]) {
  double A[m * n], b[m];
#pragma unroll
  for (int i = 0; i < m * n; i++) A[i] = A0[i];
#pragma unroll
  for (int i = 0; i < m; i++) b[i] = b0[i];
  bool fail = false;
#pragma unroll
  for (int k = 0; k < n; k++) {
    double nrm = 0;
#pragma unroll
    for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
    nrm = sqrt(nrm);
    fail |= nrm == 0.0;
    const double alpha = A[k * n + k] > 0 ? -nrm : nrm;
    double v[m];
#pragma unroll
    for (int i = 0; i < m; i++) v[i] = i < k ? 0.0 : A[i * n + k];
    v[k] -= alpha;
    double vv = 0;
#pragma unroll
    for (int i = k; i < m; i++) vv += v[i] * v[i];
    if (vv == 0.0 || fail) continue;
#pragma unroll
    for (int j = k; j < n; j++) {
      double s = 0;
#pragma unroll
      for (int i = k; i < m; i++) s += v[i] * A[i * n + j];
      s *= 2.0 / vv;
#pragma unroll
      for (int i = k; i < m; i++) A[i * n + j] -= s * v[i];
    }
    double s = 0;
#pragma unroll
    for (int i = k; i < m; i++) s += v[i] * b[i];
    s *= 2.0 / vv;
#pragma unroll
    for (int i = k; i < m; i++) b[i] -= s * v[i];
  }
  if (fail) return -1;
#pragma unroll
  for (int k = n - 1; k >= 0; k--) {
    double s = b[k];
#pragma unroll
    for (int j = k + 1; j < n; j++) s -= A[k * n + j] * x[j];
    if (A[k * n + k] == 0.0) return -1;
    x[k] = s / A[k * n + k];
  }
  return 0;
}

/* 3x3 SVD via the symmetric eigen-problem of A^T A: A = U diag(s) V^T */
__device__ __forceinline__ void svd3(const double (&A)[9], double (&U)[9], double (&V)[9]) {
  double AtA[9], d[3], Vt[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      double s = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) s += A[k * 3 + i] * A[k * 3 + j];
      AtA[i * 3 + j] = s;
    }
  jacobi3(AtA, d, Vt); /* rows of Vt = right singular vectors */
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) V[i * 3 + j] = Vt[j * 3 + i];
#pragma unroll
  for (int c = 0; c < 2; c++) { /* u_c = A v_c / |A v_c| */
    double u[3];
#pragma unroll
    for (int i = 0; i < 3; i++) u[i] = A[i * 3 + 0] * V[0 * 3 + c] + A[i * 3 + 1] * V[1 * 3 + c] + A[i * 3 + 2] * V[2 * 3 + c];
    const double nu = sqrt(dot3(u, u));
#pragma unroll
    for (int i = 0; i < 3; i++) U[i * 3 + c] = nu > 0 ? u[i] / nu : (i == c ? 1.0 : 0.0);
  }
  /* u_2 = u_0 x u_1 (orientation fixed below by the determinant check) */
  const double u0[3] = {U[0], U[3], U[6]}, u1[3] = {U[1], U[4], U[7]};
  double u2[3] = {u0[1] * u1[2] - u0[2] * u1[1], u0[2] * u1[0] - u0[0] * u1[2], u0[0] * u1[1] - u0[1] * u1[0]};
  double Av2[3];
#pragma unroll
  for (int i = 0; i < 3; i++) Av2[i] = A[i * 3 + 0] * V[2] + A[i * 3 + 1] * V[5] + A[i * 3 + 2] * V[8];
  if (dot3(Av2, u2) < 0)
#pragma unroll
    for (int i = 0; i < 3; i++) u2[i] = -u2[i];
#pragma unroll
  for (int i = 0; i < 3; i++) U[i * 3 + 2] = u2[i];
}

__device__ __forceinline__ int inv3(const double (&m)[9], double (&o)[9]) {
  const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8], c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  if (det == 0.0) return -1;
  const double id = 1.0 / det;
  o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  o[3] = c01 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  o[6] = c02 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
  return 0;
}

__device__ __forceinline__ double dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

/* ---------------- EPnP on one wave (5 correspondences) ---------------- */
constexpr int kN = 5;  // RANSAC's minimal subset (solvePnPRansac with SOLVEPNP_EPNP hypotheses)

struct WaveLds {      // one hypothesis' wave
  double A[2][144], U[2][144];  // M^T M -> diagonalised; eigenvector columns (double-buffered by round)
  double alph[4 * kN];          // barycentric coordinates
  double Vn[4][12];             // eigenvectors of the 4 smallest eigenvalues (ut rows 8..11)
};

/* Jacobi of the 12 x 12 M^T M in w.A[0], the round-robin order of oracle jacobi12_rounds.  A
   round's 6 rotations pair the indices (index 11 with r, r with 11, any other i with (2 r - i) mod 11),
   so A splits into 36 2 x 2 blocks (row pair x column pair): lane < 36 owns one, forms the block's
   row and column rotations itself from the round's start matrix (c, s of the pairs' (p, q), (p, p),
   (q, q)), takes its four elements through the column pass and then the row pass -- the same IEEE
   operations in the same order as the oracle -- and the same block of the eigenvector columns
   through the column pass, into the other buffer -> wave barrier.  One LDS round trip per round
   (it was three: rotations by lanes 0..5 -> LDS -> every element's lane).  Leaves the eigenvectors
   of the 4 smallest eigenvalues in w.Vn (ut row 8 + r). */
/* the rotation annihilating a_pq from d = a_qq - a_pp, h = 2 a_pq != 0 (oracle jacobi_cs):
   t = sgn(theta) |h| / (|d| + g), c = sqrt((|d| + g) / (2 g)), g = sqrt(d^2 + h^2) -- the classic
   Rutishauser rotation with three dependent sqrt / divide steps instead of five */
__device__ __forceinline__ void jacobi_cs(double d, double h, double& c, double& s) {
  const double g = sqrt(d * d + h * h);
  const double sg = d == 0.0 ? 1.0 : ((d > 0) == (h > 0) ? 1.0 : -1.0);
  const double t = sg * fabs(h) / (fabs(d) + g);
  c = sqrt((fabs(d) + g) / (2.0 * g));
  s = t * c;
}
__device__ __forceinline__ int partner(int i, int r) {
  return i == 11 ? r : (i == r ? 11 : (2 * r - i + 22) % 11);
}
__device__ __forceinline__ void jacobi12_wave(WaveLds& w, int lane) {
  constexpr int n = 12;
  int ee[3], ei[3], ej[3];  // this lane's elements and their (row, column)
#pragma unroll
  for (int m = 0; m < 3; m++) {
    ee[m] = lane + 64 * m;
    ei[m] = ee[m] / n;
    ej[m] = ee[m] - n * ei[m];
    if (ee[m] < 144) w.U[0][ee[m]] = (ei[m] == ej[m]) ? 1.0 : 0.0;
  }
  wave_sync();
  int b = 0;
  for (int sweep = 0; sweep < 60; sweep++) {
    double po = 0, pt = 0;
#pragma unroll
    for (int m = 0; m < 3; m++) {
      if (ee[m] < 144) {
        const double v = w.A[b][ee[m]] * w.A[b][ee[m]];
        pt += v;
        if (ei[m] != ej[m]) po += v;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      po += __shfl_xor(po, o);
      pt += __shfl_xor(pt, o);
    }
    if (po <= 1e-30 * pt || po == 0.0) break;  // uniform: identical bits in every lane
    for (int r = 0; r < 11; r++) {
      // lane < 36: the 2 x 2 block (rows of pair rp) x (columns of pair cp) of A and of U -- its two rotations
      // formed in the lane itself from the round's start matrix (no broadcast through LDS), all reads issued
      // together; the same IEEE operations per element as the column pass then row pass (and U's column pass)
      const double* A = w.A[b];
      const double* U = w.U[b];
      if (lane < 36) {
        const int rp = lane / 6, cp = lane - 6 * rp;
        int pi, qi, pj, qj;
        {
          const int a0 = rp == 0 ? r : (r + rp) % 11, b0 = rp == 0 ? 11 : (r - rp + 11) % 11;
          pi = a0 < b0 ? a0 : b0;
          qi = a0 < b0 ? b0 : a0;
          const int a1 = cp == 0 ? r : (r + cp) % 11, b1 = cp == 0 ? 11 : (r - cp + 11) % 11;
          pj = a1 < b1 ? a1 : b1;
          qj = a1 < b1 ? b1 : a1;
        }
        const double rpq = A[pi * n + qi], rpp = A[pi * n + pi], rqq = A[qi * n + qi];
        const double cpq = A[pj * n + qj], cpp = A[pj * n + pj], cqq = A[qj * n + qj];
        const double a_pp = A[pi * n + pj], a_pq = A[pi * n + qj], a_qp = A[qi * n + pj], a_qq = A[qi * n + qj];
        const double u_pp = U[pi * n + pj], u_pq = U[pi * n + qj], u_qp = U[qi * n + pj], u_qq = U[qi * n + qj];
        const bool ai = rpq != 0.0, aj = cpq != 0.0;
        double ci, si, cj, sj;  // both formed unconditionally (two independent chains), an inactive pair's discarded
        jacobi_cs(rqq - rpp, 2.0 * rpq, ci, si);
        jacobi_cs(cqq - cpp, 2.0 * cpq, cj, sj);
        // column pass (index pj takes (c, -s), qj takes (c, s))
        const double x_pp = aj ? cj * a_pp + (-sj) * a_pq : a_pp, x_qp = aj ? cj * a_qp + (-sj) * a_qq : a_qp;
        const double x_pq = aj ? cj * a_pq + sj * a_pp : a_pq, x_qq = aj ? cj * a_qq + sj * a_qp : a_qq;
        double* An = w.A[b ^ 1];
        An[pi * n + pj] = ai ? ci * x_pp + (-si) * x_qp : x_pp;  // row pass
        An[qi * n + pj] = ai ? ci * x_qp + si * x_pp : x_qp;
        An[pi * n + qj] = ai ? ci * x_pq + (-si) * x_qq : x_pq;
        An[qi * n + qj] = ai ? ci * x_qq + si * x_pq : x_qq;
        double* Un = w.U[b ^ 1];
        Un[pi * n + pj] = aj ? cj * u_pp + (-sj) * u_pq : u_pp;
        Un[pi * n + qj] = aj ? cj * u_pq + sj * u_pp : u_pq;
        Un[qi * n + pj] = aj ? cj * u_qp + (-sj) * u_qq : u_qp;
        Un[qi * n + qj] = aj ? cj * u_qq + sj * u_qp : u_qq;
      }
      wave_sync();
      b ^= 1;
    }
  }
  // descending eigenvalue order: lane i < 12 finds its rank (ties by index, as a stable
  // selection sort); ranks 8..11 hold the null-space candidates
  if (lane < n) {
    const double di = w.A[b][lane * n + lane];
    int rank = 0;
    for (int j = 0; j < n; j++) {
      const double dj = w.A[b][j * n + j];
      rank += (dj > di) || (dj == di && j < lane);
    }
    if (rank >= 8)
      for (int k = 0; k < n; k++) w.Vn[rank - 8][k] = w.U[b][k * n + lane];
  }
  wave_sync();
}

struct Epnp {
  double fu, fv, uc, vc;
  double pws[3 * kN], us[2 * kN], alphas[4 * kN];
  double cws[4][3];
};

__device__ __forceinline__ void epnp_control_points(Epnp& E) {
#pragma unroll
  for (int j = 0; j < 3; j++) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < kN; i++) s += E.pws[3 * i + j];
    E.cws[0][j] = s / kN;
  }
  double M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, d[3], Vt[9];
#pragma unroll
  for (int i = 0; i < kN; i++) {
    double p[3];
#pragma unroll
    for (int j = 0; j < 3; j++) p[j] = E.pws[3 * i + j] - E.cws[0][j];
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int b = 0; b < 3; b++) M[a * 3 + b] += p[a] * p[b];
  }
  jacobi3(M, d, Vt);
#pragma unroll
  for (int i = 1; i < 4; i++) {
    const double k = sqrt(fmax(d[i - 1], 0.0) / kN);
#pragma unroll
    for (int j = 0; j < 3; j++) E.cws[i][j] = E.cws[0][j] + k * Vt[3 * (i - 1) + j];
  }
}

__device__ __forceinline__ int epnp_barycentric(Epnp& E) {
  double cc[9], ci[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = E.cws[j][i] - E.cws[0][i];
  if (inv3(cc, ci)) return -1;
#pragma unroll
  for (int i = 0; i < kN; i++) {
    const double* p = E.pws + 3 * i;
    double* a = E.alphas + 4 * i;
#pragma unroll
    for (int j = 0; j < 3; j++)
      a[1 + j] = ci[3 * j] * (p[0] - E.cws[0][0]) + ci[3 * j + 1] * (p[1] - E.cws[0][1]) + ci[3 * j + 2] * (p[2] - E.cws[0][2]);
    a[0] = 1.0 - a[1] - a[2] - a[3];
  }
  return 0;
}

/* L_6x10 from the null-space vectors v[i] = ut row 11 - i (Vn[3 - i]) */
__device__ __forceinline__ void epnp_L(const double (&Vn)[4][12], double (&L)[60]) {
  double dv[4][6][3];
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int j = 0, a = 0, b = 1; j < 6; j++) {
#pragma unroll
      for (int k = 0; k < 3; k++) dv[i][j][k] = Vn[3 - i][3 * a + k] - Vn[3 - i][3 * b + k];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
#pragma unroll
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

__device__ __forceinline__ void betas_1(const double (&L)[60], const double (&rho)[6], double (&be)[4]) {
  double A[24], b4[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 6; i++) { A[4 * i] = L[10 * i]; A[4 * i + 1] = L[10 * i + 1]; A[4 * i + 2] = L[10 * i + 3]; A[4 * i + 3] = L[10 * i + 6]; }
  lsq_qr<6, 4>(A, rho, b4);
  if (b4[0] < 0) {
    be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
  } else {
    be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
  }
}

__device__ __forceinline__ void betas_2(const double (&L)[60], const double (&rho)[6], double (&be)[4]) {
  double A[18], b3[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 6; i++) { A[3 * i] = L[10 * i]; A[3 * i + 1] = L[10 * i + 1]; A[3 * i + 2] = L[10 * i + 2]; }
  lsq_qr<6, 3>(A, rho, b3);
  if (b3[0] < 0) { be[0] = sqrt(-b3[0]); be[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0; }
  else { be[0] = sqrt(b3[0]); be[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0; }
  if (b3[1] < 0) be[0] = -be[0];
  be[2] = 0.0;
  be[3] = 0.0;
}

__device__ __forceinline__ void betas_3(const double (&L)[60], const double (&rho)[6], double (&be)[4]) {
  double A[30], b5[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) A[5 * i + j] = L[10 * i + j];
  lsq_qr<6, 5>(A, rho, b5);
  if (b5[0] < 0) { be[0] = sqrt(-b5[0]); be[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0; }
  else { be[0] = sqrt(b5[0]); be[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0; }
  if (b5[1] < 0) be[0] = -be[0];
  be[2] = b5[3] / be[0];
  be[3] = 0.0;
}

__device__ __forceinline__ void gauss_newton(const double (&L)[60], const double (&rho)[6], double (&be)[4]) {
#pragma unroll 1
  for (int it = 0; it < 5; it++) {
    double A[24], b[6], x[4] = {0, 0, 0, 0};
#pragma unroll
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
    if (lsq_qr<6, 4>(A, b, x)) return;
#pragma unroll
    for (int i = 0; i < 4; i++) be[i] += x[i];
  }
}

__device__ __forceinline__ double epnp_R_t(const Epnp& E, const double (&Vn)[4][12], const double (&be)[4],
                                           double (&R)[9], double (&t)[3]) {
  double ccs[4][3];
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int k = 0; k < 3; k++) ccs[j][k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int k = 0; k < 3; k++) ccs[j][k] += be[i] * Vn[3 - i][3 * j + k];
  double pcs[3 * kN];
#pragma unroll
  for (int i = 0; i < kN; i++) {
    const double* a = E.alphas + 4 * i;
#pragma unroll
    for (int j = 0; j < 3; j++) pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
  }
  if (pcs[2] < 0.0) { /* solve_for_sign */
#pragma unroll
    for (int i = 0; i < 3 * kN; i++) pcs[i] = -pcs[i];
  }
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < kN; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) { pc0[j] += pcs[3 * i + j]; pw0[j] += E.pws[3 * i + j]; }
#pragma unroll
  for (int j = 0; j < 3; j++) { pc0[j] /= kN; pw0[j] /= kN; }
  double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, U[9], V[9];
#pragma unroll
  for (int i = 0; i < kN; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
      for (int k = 0; k < 3; k++) abt[3 * j + k] += (pcs[3 * i + j] - pc0[j]) * (E.pws[3 * i + k] - pw0[k]);
  svd3(abt, U, V);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) R[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
  const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                     R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
#pragma unroll
  for (int i = 0; i < 3; i++) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
  double s2 = 0;
#pragma unroll
  for (int i = 0; i < kN; i++) {
    const double* pw = E.pws + 3 * i;
    const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1], iz = 1.0 / (dot3(R + 6, pw) + t[2]);
    const double ue = E.uc + E.fu * Xc * iz, ve = E.vc + E.fv * Yc * iz;
    s2 += sqrt((E.us[2 * i] - ue) * (E.us[2 * i] - ue) + (E.us[2 * i + 1] - ve) * (E.us[2 * i + 1] - ve));
  }
  return s2 / kN;
}

/* EPnP of one 5-point subset on one wave (every lane returns the same R, t): 0 on success */
__device__ __forceinline__ void pstamp(unsigned long long* pf, int i) {
  if (pf) pf[i] = wall_clock64();
}
__device__ int epnp_wave(const double* K4, const double (&pw)[3 * kN], const double (&uv)[2 * kN], WaveLds& w,
                         int lane, double (&R)[9], double (&t)[3], unsigned long long* pf) {
  Epnp E;
  E.fu = K4[0]; E.fv = K4[1]; E.uc = K4[2]; E.vc = K4[3];
#pragma unroll
  for (int i = 0; i < 3 * kN; i++) E.pws[i] = pw[i];
#pragma unroll
  for (int i = 0; i < 2 * kN; i++) E.us[i] = uv[i];
  epnp_control_points(E);
  pstamp(pf, 1);
  if (epnp_barycentric(E)) return -1;  // uniform
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 4 * kN; i++) w.alph[i] = E.alphas[i];
  wave_sync();
  // M^T M: element (a, b) = sum_i M1_ia M1_ib + M2_ia M2_ib, i in order (oracle loop order)
#pragma unroll
  for (int m = 0; m < 3; m++) {
    const int e = lane + 64 * m;
    if (e >= 144) continue;
    const int a = e / 12, b = e - 12 * a;
    const int ka = a / 3, ca = a - 3 * ka, kb = b / 3, cb = b - 3 * kb;
    double s = 0;
#pragma unroll
    for (int i = 0; i < kN; i++) {
      const double aa = w.alph[4 * i + ka], ab = w.alph[4 * i + kb];
      const double du = E.uc - uv[2 * i], dv = E.vc - uv[2 * i + 1];
      const double m1a = ca == 0 ? aa * E.fu : ca == 1 ? 0.0 : aa * du;
      const double m1b = cb == 0 ? ab * E.fu : cb == 1 ? 0.0 : ab * du;
      const double m2a = ca == 0 ? 0.0 : ca == 1 ? aa * E.fv : aa * dv;
      const double m2b = cb == 0 ? 0.0 : cb == 1 ? ab * E.fv : ab * dv;
      s += m1a * m1b + m2a * m2b;
    }
    w.A[0][e] = s;
  }
  wave_sync();
  pstamp(pf, 2);
  jacobi12_wave(w, lane);
  pstamp(pf, 3);
  const double(&Vn)[4][12] = w.Vn;  // LDS broadcast reads
  double L[60], rho[6];
  epnp_L(Vn, L);
  rho[0] = dist2(E.cws[0], E.cws[1]); rho[1] = dist2(E.cws[0], E.cws[2]); rho[2] = dist2(E.cws[0], E.cws[3]);
  rho[3] = dist2(E.cws[1], E.cws[2]); rho[4] = dist2(E.cws[1], E.cws[3]); rho[5] = dist2(E.cws[2], E.cws[3]);
  // the three beta approximations side by side: lane 0 approximation 1, lane 1 approximation 2,
  // the other lanes 3 (betas_k diverge; Gauss-Newton and R, t run converged on the lanes' own
  // betas), then the oracle's choice (strictly lower mean reprojection error, 1 first)
  const int k = lane < 2 ? lane + 1 : 3;
  double be[4], Rk[9], tk[3];
  if (k == 1) betas_1(L, rho, be);
  else if (k == 2) betas_2(L, rho, be);
  else betas_3(L, rho, be);
  pstamp(pf, 4);
  gauss_newton(L, rho, be);
  pstamp(pf, 5);
  const double ek = epnp_R_t(E, Vn, be, Rk, tk);
  pstamp(pf, 6);
  const double e1 = wave::rdlaned(ek, 0), e2 = wave::rdlaned(ek, 1), e3 = wave::rdlaned(ek, 2);
  int N = 1;
  if (e2 < e1) N = 2;
  if (e3 < (N == 2 ? e2 : e1)) N = 3;
  const double eb = N == 1 ? e1 : (N == 2 ? e2 : e3);
  double Rb[9], tb[3];
#pragma unroll
  for (int q = 0; q < 9; q++) Rb[q] = wave::rdlaned(Rk[q], N - 1);
#pragma unroll
  for (int q = 0; q < 3; q++) tb[q] = wave::rdlaned(tk[q], N - 1);
  if (!isfinite(eb)) return -1;
#pragma unroll
  for (int q = 0; q < 9; q++) R[q] = Rb[q];
#pragma unroll
  for (int q = 0; q < 3; q++) t[q] = tb[q];
  return 0;
}

/* RANSACUpdateNumIters */
__device__ int update_iters(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.), 1.);
  ep = fmin(fmax(ep, 0.), 1.);
  double num = fmax(1. - p, DBL_MIN);
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

__device__ double reproj2(const double* K4, const double R[9], const double t[3], const double* p, const double* uv) {
  const double Xc = dot3(R, p) + t[0], Yc = dot3(R + 3, p) + t[1], Zc = dot3(R + 6, p) + t[2];
  const double iz = 1.0 / Zc;
  const double du = uv[0] - (K4[0] * Xc * iz + K4[2]), dv = uv[1] - (K4[1] * Yc * iz + K4[3]);
  return du * du + dv * dv;
}


// Levenberg-Marquardt on the inliers' squared reprojection error (orc_pnp's refine, oracle/pnp.c):
// pose T_cw (R, t) with the left exp-map update; the NW waves' threads own strided correspondences, the
// 6x6 normal equations and the costs are wave-reduced and then added over the waves in wave order
// (wave::block_allreduce28), so every thread takes the same decisions
template <int NW>
__device__ void refine(const double* K4, int n, const double* pw, const double* uv, const uint8_t* inl, int tid,
                       double R[9], double t[3]) {
#pragma clang fp contract(fast)  // the refinement is held to a tolerance, not to bits
  const int lane = tid & 63;
  double lambda = 1e-3;
  for (int it = 0; it < 20; it++) {
    double acc[wave::kNV];
    for (int k = 0; k < wave::kNV; k++) acc[k] = 0.0;
    for (int i = tid; i < n; i += 64 * NW) {
      if (!inl[i]) continue;
      const double* p = pw + 3 * i;
      const double x = dot3(R, p) + t[0], y = dot3(R + 3, p) + t[1], z = dot3(R + 6, p) + t[2];
      const double iz = 1.0 / z, iz2 = iz * iz;
      const double e0 = uv[2 * i] - (K4[0] * x * iz + K4[2]), e1 = uv[2 * i + 1] - (K4[1] * y * iz + K4[3]);
      acc[27] += e0 * e0 + e1 * e1;
      const double Dm[2][3] = {{K4[0] * iz, 0, -K4[0] * x * iz2}, {0, K4[1] * iz, -K4[1] * y * iz2}};
      const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
      double J[2][6];
      for (int r = 0; r < 2; r++)
        for (int c = 0; c < 3; c++) {
          double s = 0;
          for (int k = 0; k < 3; k++) s += Dm[r][k] * SX[k * 3 + c];
          J[r][c] = s;
          J[r][3 + c] = -Dm[r][c];
        }
      for (int a = 0; a < 6; a++) {
        acc[21 + a] += -(J[0][a] * e0 + J[1][a] * e1);
        for (int b = a; b < 6; b++) acc[a * 6 - a * (a - 1) / 2 + (b - a)] += J[0][a] * J[0][b] + J[1][a] * J[1][b];
      }
    }
    wave::block_allreduce28<NW>(acc, lane);
    const double cost = acc[27];
    auto H = [&](int a, int b) { return a <= b ? acc[a * 6 - a * (a - 1) / 2 + (b - a)] : acc[b * 6 - b * (b - 1) / 2 + (a - b)]; };
    bool accepted = false;
    for (int trial = 0; trial < 10 && !accepted; trial++) {
      double A[6][6], x[6];
      for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) A[i][j] = H(i, j);
      for (int i = 0; i < 6; i++) A[i][i] += lambda * fmax(H(i, i), 1e-12);
      for (int i = 0; i < 6; i++) x[i] = acc[21 + i];
      // Cholesky with the pivots' reciprocals on the diagonal: one v_rcp_f64 + Newton per
      // column instead of a divide per entry (the refined optimum agrees with the oracle's
      // divides to rounding; the tests hold it to 1e-9)
      bool ok = true;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        double s = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) s -= A[j][k] * A[j][k];
        ok = ok && s > 0;
        const double r = wave::rcp64(sqrt(s));
        A[j][j] = r;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
          double v = A[i][j];
#pragma unroll
          for (int k = 0; k < j; k++) v -= A[i][k] * A[j][k];
          A[i][j] = v * r;
        }
      }
      if (!ok) {
        lambda *= 10;
        continue;
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
        double s = x[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= A[i][k] * x[k];
        x[i] = s * A[i][i];
      }
#pragma unroll
      for (int i = 5; i >= 0; i--) {
        double s = x[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= A[k][i] * x[k];
        x[i] = s * A[i][i];
      }
      const double* w = x;
      const double th = sqrt(dot3(w, w));
      const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
      double O2[9];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) O2[a * 3 + b] = O[a * 3] * O[b] + O[a * 3 + 1] * O[3 + b] + O[a * 3 + 2] * O[6 + b];
      double ca, cb, cc, cd;
      if (th < 1e-5) {
        ca = 1.0; cb = 0.5; cc = 0.5; cd = 1.0 / 6.0;
      } else {
        ca = sin(th) / th; cb = (1 - cos(th)) / (th * th); cc = cb; cd = (th - sin(th)) / (th * th * th);
      }
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
      double cn[1] = {0};
      for (int i = tid; i < n; i += 64 * NW)
        if (inl[i]) cn[0] += reproj2(K4, Rn, tn, pw + 3 * i, uv + 2 * i);
      cn[0] = wave::wsum(cn[0]);
      wave::block_combine<NW>(cn);
      if (cn[0] < cost) {
        for (int k = 0; k < 9; k++) R[k] = Rn[k];
        for (int k = 0; k < 3; k++) t[k] = tn[k];
        lambda = fmax(lambda * 0.1, 1e-12);
        accepted = true;
        if (cost - cn[0] <= 1e-14 * cost) return;
      } else {
        lambda *= 10;
      }
    }
    if (!accepted) return;
  }
}

// squared reprojection error of world point p (pixels), pinhole K4 = (fx, fy, cx, cy)
__device__ __forceinline__ double proj_err2(const double* K4, const double* R, const double* t, const double* p,
                                            const double* uv) {
  return reproj2(K4, R, t, p, uv);
}

// stage 1: wave w of workgroup (bx, frame) solves hypothesis 4 bx + w and counts its inliers
__global__ __launch_bounds__(256) void pnp_hyp_kernel(Args a) {
  __shared__ WaveLds wl[kHypWaves];
  const int f = blockIdx.y, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x * kHypWaves + wv;
  const Desc D = a.frames[f];
  if (h >= D.iters || D.n < 8) return;  // wave-uniform
  const double* pw = a.pts + 3 * (size_t)D.p0;
  const double* uv = a.kps + 2 * (size_t)D.p0;
  const int32_t* sub = a.subsets + 5 * ((size_t)D.s0 + h);
  double sp[3 * kN], su[2 * kN], R[9], t[3];
#pragma unroll
  for (int k = 0; k < kN; k++) {
    const int s = sub[k];
#pragma unroll
    for (int j = 0; j < 3; j++) sp[3 * k + j] = pw[3 * s + j];
#pragma unroll
    for (int j = 0; j < 2; j++) su[2 * k + j] = uv[2 * s + j];
  }
  int cnt = -1;
  unsigned long long* pf = (a.prof && f == 0 && h == 0 && lane == 0) ? a.prof : nullptr;
  pstamp(pf, 0);
  if (epnp_wave(D.K, sp, su, wl[wv], lane, R, t, pf) == 0) {
    int c = 0;
    for (int i = lane; i < D.n; i += 64) c += reproj2(D.K, R, t, pw + 3 * i, uv + 2 * i) <= D.thr2;
    cnt = wave::wsum_int(c);
  }
  pstamp(pf, 7);
  if (lane == 0) {
    double* hr = a.hyp + ((size_t)f * kMaxIters + h) * 12;
#pragma unroll
    for (int k = 0; k < 9; k++) hr[k] = R[k];
#pragma unroll
    for (int k = 0; k < 3; k++) hr[9 + k] = t[k];
    a.hcnt[(size_t)f * kMaxIters + h] = cnt;
  }
}

// stage 2: one workgroup of kFinalWaves waves per frame -- RANSAC's acceptance in hypothesis order (replayed
// by every thread), inliers, refinement (its sums over the four waves: 52 us on one wave, r05_experiments.md)
constexpr int kFinalWaves = 4;
__global__ __launch_bounds__(64 * kFinalWaves) void pnp_final_kernel(Args a) {
  const int f = blockIdx.x, tid = threadIdx.x;
  constexpr int T = 64 * kFinalWaves;
  unsigned long long* pf = (a.prof && f == 0 && tid == 0) ? a.prof : nullptr;
  pstamp(pf, 8);
  const Desc D = a.frames[f];
  const int n = D.n;
  const int* hc = a.hcnt + (size_t)f * kMaxIters;
  int best = -1, used = 0;
  if (n >= 8) {  // uniform: every lane replays the same sequence (counts read as broadcasts)
    int best_cnt = 0, niters = D.iters, h = 0;
    for (h = 0; h < niters; h++) {
      const int c = hc[h];
      if (c < 0) continue;  // the minimal solver failed (runKernel returned no model)
      if (c > (best_cnt > 4 ? best_cnt : 4)) {
        best = h;
        best_cnt = c;
        niters = update_iters(D.confidence, (double)(n - c) / n, 5, niters);
      }
    }
    used = h;
  }
  Out* o = a.out + f;
  uint8_t* inl = a.inl + D.p0;
  if (best < 0) {
    for (int i = tid; i < n; i += T) inl[i] = 0;
    if (tid == 0) {
      o->n_inliers = 0;
      o->hyps = used;
    }
    return;
  }
  const double* pw = a.pts + 3 * (size_t)D.p0;
  const double* uv = a.kps + 2 * (size_t)D.p0;
  const double* hr = a.hyp + ((size_t)f * kMaxIters + best) * 12;
  double R[9], t[3];
#pragma unroll
  for (int k = 0; k < 9; k++) R[k] = hr[k];
#pragma unroll
  for (int k = 0; k < 3; k++) t[k] = hr[9 + k];
  int ninl = 0;
  for (int i = tid; i < n; i += T) {
    const uint8_t in = reproj2(D.K, R, t, pw + 3 * i, uv + 2 * i) <= D.thr2;
    inl[i] = in;
    ninl += in;
  }
  ninl = wave::block_sum_int<kFinalWaves>(ninl);  // (its barriers order the inlier flags before the refinement)
  pstamp(pf, 9);
  refine<kFinalWaves>(D.K, n, pw, uv, inl, tid, R, t);
  pstamp(pf, 10);
  if (tid == 0) {
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) o->Rwc[3 * i + j] = R[3 * j + i];
    for (int i = 0; i < 3; i++) o->twc[i] = -(R[i] * t[0] + R[3 + i] * t[1] + R[6 + i] * t[2]);
    o->n_inliers = ninl;
    o->hyps = used;
  }
}

hipError_t solve(const Args& a, int batch, int max_iters, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  if (max_iters > 0) pnp_hyp_kernel<<<dim3((max_iters + kHypWaves - 1) / kHypWaves, batch), 256, 0, s>>>(a);
  pnp_final_kernel<<<batch, 64 * kFinalWaves, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace pnp
}  // namespace rspl
