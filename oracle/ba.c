/*
 * ORACLE (test infrastructure only) -- fp64 CPU restatement of the reference's
 * local bundle adjustment, LocalmapOptimization
 * (src/g2o_optimization/g2o_optimization.cc:21-252), and of the parts of g2o it
 * relies on.  g2o is a third-party library NOT vendored in the reference
 * (CMakeLists.txt:32, version unpinned); the restated g2o semantics are its
 * published algorithms -- parity at the g2o boundary is therefore UNPINNED and
 * is checked against independent optima (scipy least_squares) and known answers.
 *
 * Restated pieces:
 *  - VertexSE3Expmap (estimate T_cw = SE3Quat(q,p).inverse(), :42) with the
 *    left-multiplicative exp-map update  T <- exp([w; v]) * T
 *  - VertexPointXYZ (p += dx), VertexLine3D (g2o::Line3D::oplus, orthonormal
 *    4-DoF update; include/g2o_optimization/vertex_line3d.h:26-29)
 *  - EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ: e = obs - proj(T p),
 *    analytic Jacobians (:81-118)
 *  - EdgeSE3ProjectLine / EdgeStereoSE3ProjectLine computeError
 *    (src/g2o_optimization/edge_project_line.cc:21-42,
 *     edge_project_stereo_line.cc:22-51) with g2o's default numeric central
 *    difference Jacobian (delta 1e-9) because they do not override linearizeOplus
 *  - Huber kernel with delta = (float)sqrt(threshold) (:77-78, 125-126); robust
 *    information = rho'(chi2) * Omega
 *  - OptimizationAlgorithmLevenberg (tau 1e-5, good-step scale in [1/3, 2/3],
 *    ni doubling, 10 trials) over BlockSolver<-1,-1> Schur complement on
 *    marginalised points and lines
 *  - two-phase schedule: optimize(10) -> chi2/depth outlier levels, drop
 *    kernels -> initializeOptimization(0), optimize(5) -> inlier flags (:172-231);
 *    an edge's chi2 is that of its last computed error (g2o keeps _error), which
 *    for level-1 edges is the phase-1 value.
 */
#include <float.h>
#include <math.h>

#include "../include/rspl.h"
#include "oracle_common.h"

typedef struct {
  double q[4]; /* w, x, y, z */
  double t[3];
} se3;

static void q_norm(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int i = 0; i < 4; i++) q[i] /= n;
}

static void q_to_R(const double q[4], double R[9]) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

static void R_to_q(const double m[9], double q[4]) {
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

static void q_mul(const double a[4], const double b[4], double o[4]) {
  o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  o[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  o[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  o[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}

static void se3_normalize(se3* T) { /* SE3Quat::normalizeRotation */
  if (T->q[0] < 0)
    for (int i = 0; i < 4; i++) T->q[i] = -T->q[i];
  q_norm(T->q);
}

static void mat3_vec(const double R[9], const double v[3], double o[3]) {
  o[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  o[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  o[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
}

static void se3_map(const se3* T, const double p[3], double o[3]) {
  double R[9];
  q_to_R(T->q, R);
  mat3_vec(R, p, o);
  for (int i = 0; i < 3; i++) o[i] += T->t[i];
}

static se3 se3_inverse(const se3* T) {
  se3 r;
  r.q[0] = T->q[0]; r.q[1] = -T->q[1]; r.q[2] = -T->q[2]; r.q[3] = -T->q[3];
  double R[9], t[3];
  q_to_R(r.q, R);
  mat3_vec(R, T->t, t);
  for (int i = 0; i < 3; i++) r.t[i] = -t[i];
  se3_normalize(&r);
  return r;
}

static se3 se3_mul(const se3* a, const se3* b) {
  se3 r;
  double R[9], t[3];
  q_to_R(a->q, R);
  mat3_vec(R, b->t, t);
  for (int i = 0; i < 3; i++) r.t[i] = a->t[i] + t[i];
  q_mul(a->q, b->q, r.q);
  se3_normalize(&r);
  return r;
}

/* SE3Quat::exp (update = [omega; upsilon]) */
static se3 se3_exp(const double u[6]) {
  const double* w = u;
  const double* v = u + 3;
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
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
    c = (1 - cos(th)) / (th * th);
    d = (th - sin(th)) / (th * th * th);
  }
  double R[9], V[9];
  for (int i = 0; i < 9; i++) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    R[i] = I + a * O[i] + b * O2[i];
    V[i] = I + c * O[i] + d * O2[i];
  }
  se3 r;
  R_to_q(R, r.q);
  mat3_vec(V, v, r.t);
  se3_normalize(&r);
  return r;
}

/* ---------------- g2o::Line3D (slam3d_addons/line3d.h) ---------------- */
static double n3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

static void line_oplus(double L[6], const double v[4]) {
  const double* w = L;
  const double* d = L + 3;
  /* toOrthonormal */
  const double mx = n3(d), my = n3(w);
  const double wn = 1.0 / sqrt(mx * mx + my * my);
  double Wm[4] = {my * wn, -mx * wn, mx * wn, my * wn};
  const double mn = 1.0 / my, dn = 1.0 / mx;
  double mdc[3];
  cross3(w, d, mdc);
  const double mdn = 1.0 / n3(mdc);
  double U[9] = {w[0] * mn, d[0] * dn, mdc[0] * mdn,
                 w[1] * mn, d[1] * dn, mdc[1] * mdn,
                 w[2] * mn, d[2] * dn, mdc[2] * mdn};
  /* update */
  const double cs = cos(v[3]), sn = sin(v[3]);
  double Wu[4] = {cs, -sn, sn, cs};
  double q[4] = {sqrt(1 - (v[0] * v[0] + v[1] * v[1] + v[2] * v[2])), v[0], v[1], v[2]};
  q_norm(q);
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
  /* fromOrthonormal + normalize (twice: fromOrthonormal and oplus) */
  double out[6];
  for (int i = 0; i < 3; i++) {
    out[i] = W2[0] * U2[i * 3 + 0];
    out[3 + i] = W2[2] * U2[i * 3 + 1];
  }
  for (int rep = 0; rep < 2; rep++) {
    const double s = 1.0 / n3(out + 3);
    for (int i = 0; i < 6; i++) out[i] *= s;
  }
  memcpy(L, out, sizeof(out));
}

/* T * L for an isometry T (operator*(Isometry3, Line3D)) */
static void line_transform(const double R[9], const double t[3], const double L[6], double o[6]) {
  double Rw[3], Rd[3], tx[3];
  mat3_vec(R, L, Rw);
  mat3_vec(R, L + 3, Rd);
  cross3(t, Rd, tx);
  for (int i = 0; i < 3; i++) {
    o[i] = Rw[i] + tx[i];
    o[3 + i] = Rd[i];
  }
}

/* ---------------- problem state ---------------- */
typedef struct {
  const rspl_ba_problem* P;
  int np, nq, nl; /* poses, points, lines */
  se3* T;          /* T_cw */
  double* X;       /* points [nq][3] */
  double* L;       /* lines [nl][6] */
  double dmp, dsp, dml, dsl; /* Huber deltas */
  /* per-edge state (types: 0 mono, 1 stereo, 2 mono line, 3 stereo line) */
  int ne[4];
  double* err[4]; /* last computed error */
  unsigned char* level[4];
  int robust;
} ba_t;

static const int EDIM[4] = {2, 3, 2, 4};
static const int LDIM[4] = {3, 3, 4, 4};

static const double* cam_of(const ba_t* b, const int32_t* ids, int e) {
  const int c = ids ? ids[e] : 0;
  return b->P->cameras + 5 * c;
}

static int edge_pose(const ba_t* b, int t, int e) {
  const rspl_ba_problem* P = b->P;
  return t == 0 ? P->mono_pose[e] : t == 1 ? P->stereo_pose[e] : t == 2 ? P->mono_line_pose[e] : P->stereo_line_pose[e];
}
static int edge_lm(const ba_t* b, int t, int e) {
  const rspl_ba_problem* P = b->P;
  return t == 0 ? P->mono_point[e] : t == 1 ? P->stereo_point[e] : t == 2 ? P->mono_line_line[e] : P->stereo_line_line[e];
}
static double edge_info(int t) { return t < 2 ? 1.0 : 0.1; }
static double edge_delta(const ba_t* b, int t) { return t == 0 ? b->dmp : t == 1 ? b->dsp : t == 2 ? b->dml : b->dsl; }

static void line_err(const double* cam, const se3* T, const double* L, const double* obs, int stereo, double* e) {
  const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3], bf = cam[4];
  const double Kv[3] = {-fy * cx, -fx * cy, fx * fy};
  double R[9], Lc[6];
  q_to_R(T->q, R);
  for (int side = 0; side < (stereo ? 2 : 1); side++) {
    double t[3] = {T->t[0], T->t[1], T->t[2]};
    if (side == 1) t[0] -= bf / fx; /* T_right(0,3) -= b, b = bf/fx (g2o_optimization.cc:165) */
    line_transform(R, t, L, Lc);
    const double l0 = fy * Lc[0], l1 = fx * Lc[1], l2 = Kv[0] * Lc[0] + Kv[1] * Lc[1] + Kv[2] * Lc[2];
    const double nrm = sqrt(l0 * l0 + l1 * l1);
    const double* o = obs + 4 * side;
    e[2 * side + 0] = (o[0] * l0 + o[1] * l1 + l2) / nrm;
    e[2 * side + 1] = (o[2] * l0 + o[3] * l1 + l2) / nrm;
  }
}

static void compute_error(const ba_t* b, int t, int e, double* out) {
  const rspl_ba_problem* P = b->P;
  const se3* T = &b->T[edge_pose(b, t, e)];
  const int l = edge_lm(b, t, e);
  if (t < 2) {
    const double* cam = cam_of(b, t == 0 ? P->mono_camera : P->stereo_camera, e);
    double Xc[3];
    se3_map(T, b->X + 3 * l, Xc);
    const double iz = 1.0 / Xc[2];
    const double u = cam[0] * Xc[0] * iz + cam[2];
    const double v = cam[1] * Xc[1] * iz + cam[3];
    const double* obs = t == 0 ? P->mono_obs + 2 * e : P->stereo_obs + 3 * e;
    out[0] = obs[0] - u;
    out[1] = obs[1] - v;
    if (t == 1) out[2] = obs[2] - (u - cam[4] * iz);
  } else if (t == 2) {
    line_err(cam_of(b, P->mono_line_camera, e), T, b->L + 6 * l, P->mono_line_obs + 4 * e, 0, out);
  } else {
    line_err(cam_of(b, P->stereo_line_camera, e), T, b->L + 6 * l, P->stereo_line_obs + 8 * e, 1, out);
  }
}

static double chi2_of(int t, const double* e) {
  double s = 0;
  for (int i = 0; i < EDIM[t]; i++) s += e[i] * e[i];
  return s * edge_info(t);
}

/* Huber rho (g2o RobustKernelHuber::robustify) */
static void huber(double e2, double delta, double rho[2]) {
  const double dsqr = delta * delta;
  if (e2 <= dsqr) {
    rho[0] = e2;
    rho[1] = 1.0;
  } else {
    const double s = sqrt(e2);
    rho[0] = 2 * s * delta - dsqr;
    rho[1] = delta / s;
  }
}

static int depth_positive(const ba_t* b, int t, int e) {
  double Xc[3];
  se3_map(&b->T[edge_pose(b, t, e)], b->X + 3 * edge_lm(b, t, e), Xc);
  return Xc[2] > 0.0;
}

/* Line-edge Jacobians, analytic: the delta -> 0 limit of g2o's central difference below (its O(delta^2)
 * truncation is ~1e-18 relative at delta 1e-9; the quotient's cancellation noise, ~1e-7 relative, is what
 * this removes).  Restated from the same definitions:
 *  - pose: VertexSE3Expmap::oplusImpl T' = exp(u) T, u = [omega; upsilon]; with a = R w, b = R d and
 *    wc = a + t x b (operator*(Isometry3, Line3D)): d wc / d omega = -[wc]x, d wc / d upsilon = -[b]x; the
 *    right camera of a stereo edge (t_x -= bf / fx after the perturbation, g2o_optimization.cc:165) adds
 *    [b]x [c]x with c = (bf / fx, 0, 0);
 *  - line: Line3D::oplus (line_oplus above) at v = 0, after its normalisation to |d| = 1: with u1 = w / |w|,
 *    u2 = d / |d|, u3 = (w x d) / |w x d|, rho = |w| / |d|: d w'' / dv = [0, -2 rho u3, 2 rho u2, -(1 + rho^2) u1],
 *    d d'' / dv = [2 u3, 0, -2 u1, 0] (the quaternion part rotates U by 2 [v]x, the angle part rotates W);
 *  - error (edge_project_line.cc:21-42): l = [fy wc0, fx wc1, Kv . wc], e_k = (o_k . l01 + l2) / |l01|.
 * The error is homogeneous of degree 0 in the line, so everything is evaluated at L / |d|. */
static int g_line_jac_analytic = 0;
/* LM trials (accepted + rejected) of the last orc_ba_local's two optimize() calls (test hook) */
static int g_trials[2] = {0, 0};
void orc_ba_last_trials(int* out) {
  out[0] = g_trials[0];
  out[1] = g_trials[1];
}
void orc_ba_set_line_jacobian(int analytic) { g_line_jac_analytic = analytic != 0; }

static void skew(const double* v, double* S) { /* S x = v x x */
  S[0] = 0; S[1] = -v[2]; S[2] = v[1];
  S[3] = v[2]; S[4] = 0; S[5] = -v[0];
  S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

/* g2o's numeric central difference of one line edge (BaseBinaryEdge::linearizeOplus, delta 1e-9): the pose by
 * the left exp-map increment, the line by Line3D::oplus, each +-delta, the quotient (e+ - e-) / (2 delta) --
 * used by linearize() and by the orc_line_jacobian test hook alike */
static void line_jac_numeric(const double* cam, const se3* T0, const double* L, const double* obs, int stereo,
                             double* Jp, double* Jl) {
  const se3 T = *T0;
  const double delta = 1e-9, scal = 1.0 / (2 * delta);
  const int rows = stereo ? 4 : 2;
  double ep[4], em[4], Lp[6];
  for (int d = 0; d < 4; d++) {
    double v[4] = {0, 0, 0, 0};
    v[d] = delta;
    memcpy(Lp, L, sizeof(Lp));
    line_oplus(Lp, v);
    line_err(cam, &T, Lp, obs, stereo, ep);
    v[d] = -delta;
    memcpy(Lp, L, sizeof(Lp));
    line_oplus(Lp, v);
    line_err(cam, &T, Lp, obs, stereo, em);
    for (int r = 0; r < rows; r++) Jl[r * 4 + d] = scal * (ep[r] - em[r]);
  }
  for (int d = 0; d < 6; d++) {
    double u[6] = {0, 0, 0, 0, 0, 0};
    u[d] = delta;
    se3 dT = se3_exp(u), Tp = se3_mul(&dT, &T);
    line_err(cam, &Tp, L, obs, stereo, ep);
    u[d] = -delta;
    dT = se3_exp(u);
    Tp = se3_mul(&dT, &T);
    line_err(cam, &Tp, L, obs, stereo, em);
    for (int r = 0; r < rows; r++) Jp[r * 6 + d] = scal * (ep[r] - em[r]);
  }
}

static void line_jac_analytic(const double* cam, const se3* T, const double* L, const double* obs, int stereo,
                              double* Jp, double* Jl) {
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
  /* d w / dv_k, d d / dv_k (columns k = 0..3) */
  double dw[4][3], dd[4][3];
  for (int i = 0; i < 3; i++) {
    dw[0][i] = 0;                dd[0][i] = 2 * u3[i];
    dw[1][i] = -2 * rho * u3[i]; dd[1][i] = 0;
    dw[2][i] = 2 * rho * d[i];   dd[2][i] = -2 * u1[i];
    dw[3][i] = -(1 + rho * rho) * u1[i]; dd[3][i] = 0;
  }
  double R[9], a[3], bb[3];
  q_to_R(T->q, R);
  mat3_vec(R, w, a);
  mat3_vec(R, d, bb);
  double Sb[9];
  skew(bb, Sb);
  for (int side = 0; side < (stereo ? 2 : 1); side++) {
    double t[3] = {T->t[0], T->t[1], T->t[2]};
    const double c[3] = {side == 1 ? bf / fx : 0.0, 0.0, 0.0};
    t[0] -= c[0];
    double txb[3], wc[3];
    cross3(t, bb, txb);
    for (int i = 0; i < 3; i++) wc[i] = a[i] + txb[i];
    double l[3];
    mat3_vec(M, wc, l);
    const double n = sqrt(l[0] * l[0] + l[1] * l[1]);
    /* d wc / d pose [3][6] */
    double Sw[9], Sc[9], BC[9];
    skew(wc, Sw);
    skew(c, Sc);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += Sb[i * 3 + k] * Sc[k * 3 + j];
        BC[i * 3 + j] = s;
      }
    double Gp[3][6];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        Gp[i][j] = -Sw[i * 3 + j] + BC[i * 3 + j];
        Gp[i][3 + j] = -Sb[i * 3 + j];
      }
    /* d wc / dv [3][4] = R dw + t x (R dd) */
    double Gl[3][4];
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

/* Jacobians: Jp [edim][6] wrt pose update, Jl [edim][ldim] wrt landmark update. */
static void linearize(ba_t* b, int t, int e, double* Jp, double* Jl) {
  const rspl_ba_problem* P = b->P;
  const int pi = edge_pose(b, t, e), l = edge_lm(b, t, e);
  if (t < 2) {
    const double* cam = cam_of(b, t == 0 ? P->mono_camera : P->stereo_camera, e);
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    double R[9], Xc[3];
    q_to_R(b->T[pi].q, R);
    se3_map(&b->T[pi], b->X + 3 * l, Xc);
    const double x = Xc[0], y = Xc[1], z = Xc[2], iz = 1.0 / z, iz2 = iz * iz;
    /* d proj / d Xc */
    double D[3][3] = {{fx * iz, 0, -fx * x * iz2}, {0, fy * iz, -fy * y * iz2}, {fx * iz, 0, -fx * x * iz2 + bf * iz2}};
    const int rows = EDIM[t];
    /* dXc/dw = -[Xc]x, dXc/dv = I, dXc/dp = R; e = obs - proj -> J = -D * dXc */
    const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int r = 0; r < rows; r++) {
      for (int c = 0; c < 3; c++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += D[r][k] * SX[k * 3 + c];
        Jp[r * 6 + c] = s;                /* -D * (-[Xc]x) */
        Jp[r * 6 + 3 + c] = -D[r][c];     /* -D * I */
        double sl = 0;
        for (int k = 0; k < 3; k++) sl += D[r][k] * R[k * 3 + c];
        Jl[r * 3 + c] = -sl;
      }
    }
  } else if (g_line_jac_analytic) {
    if (t == 2)
      line_jac_analytic(cam_of(b, P->mono_line_camera, e), &b->T[pi], b->L + 6 * l, P->mono_line_obs + 4 * e, 0, Jp, Jl);
    else
      line_jac_analytic(cam_of(b, P->stereo_line_camera, e), &b->T[pi], b->L + 6 * l, P->stereo_line_obs + 8 * e, 1, Jp,
                        Jl);
  } else if (t == 2) {
    line_jac_numeric(cam_of(b, P->mono_line_camera, e), &b->T[pi], b->L + 6 * l, P->mono_line_obs + 4 * e, 0, Jp, Jl);
  } else {
    line_jac_numeric(cam_of(b, P->stereo_line_camera, e), &b->T[pi], b->L + 6 * l, P->stereo_line_obs + 8 * e, 1, Jp,
                     Jl);
  }
}

/* Cholesky solve of dense SPD system (n x n, row-major), in place. returns 0 ok */
static int chol_solve(double* A, double* x, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (!(s > 0)) return -1;
    const double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  for (int i = 0; i < n; i++) {
    double s = x[i];
    for (int k = 0; k < i; k++) s -= A[i * n + k] * x[k];
    x[i] = s / A[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++) s -= A[k * n + i] * x[k];
    x[i] = s / A[i * n + i];
  }
  return 0;
}

/* small dense inverse via Gauss-Jordan (landmark blocks 3x3 / 4x4) */
static int small_inv(const double* A, double* I, int n) {
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
    if (M[p][c] == 0) return -1;
    if (p != c)
      for (int k = 0; k < 2 * n; k++) {
        double t = M[c][k]; M[c][k] = M[p][k]; M[p][k] = t;
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
  return 0;
}

typedef struct {
  int pose_idx_count;
  int* pidx;          /* pose -> reduced index or -1 */
  unsigned char* qact, *lact; /* active landmarks */
  /* linear system */
  double* Hpp;        /* [6K][6K] */
  double* bp;         /* [6K] */
  double* Hqq;        /* [nq][9] */
  double* bq;         /* [nq][3] */
  double* Hll;        /* [nl][16] */
  double* bl;         /* [nl][4] */
  double* Hpl[4];     /* per edge [6][ldim] */
  double* x;          /* [6K + 3nq + 4nl] */
} sys_t;

static int edge_active(const ba_t* b, int t, int e, int phase) { return phase == 1 || b->level[t][e] == 0; }

static double active_chi2(ba_t* b, int phase, int robust) {
  double s = 0;
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b->ne[t]; e++) {
      if (!edge_active(b, t, e, phase)) continue;
      compute_error(b, t, e, b->err[t] + 4 * e);
      const double c2 = chi2_of(t, b->err[t] + 4 * e);
      if (robust) {
        double rho[2];
        huber(c2, edge_delta(b, t), rho);
        s += rho[0];
      } else {
        s += c2;
      }
    }
  return s;
}

static void build_system(ba_t* b, sys_t* S, int phase, int robust) {
  const int K = S->pose_idx_count, nq = b->nq, nl = b->nl;
  memset(S->Hpp, 0, sizeof(double) * 36 * K * K);
  memset(S->bp, 0, sizeof(double) * 6 * K);
  memset(S->Hqq, 0, sizeof(double) * 9 * nq);
  memset(S->bq, 0, sizeof(double) * 3 * nq);
  memset(S->Hll, 0, sizeof(double) * 16 * nl);
  memset(S->bl, 0, sizeof(double) * 4 * nl);
  double Jp[4 * 6], Jl[4 * 4];
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b->ne[t]; e++) {
      if (!edge_active(b, t, e, phase)) continue;
      const int rows = EDIM[t], ld = LDIM[t];
      linearize(b, t, e, Jp, Jl);
      const double* er = b->err[t] + 4 * e;
      double w = edge_info(t);
      if (robust) {
        double rho[2];
        huber(chi2_of(t, er), edge_delta(b, t), rho);
        w *= rho[1];
      }
      const int pi = S->pidx[edge_pose(b, t, e)];
      const int l = edge_lm(b, t, e);
      double* Hl = t < 2 ? S->Hqq + 9 * l : S->Hll + 16 * l;
      double* blv = t < 2 ? S->bq + 3 * l : S->bl + 4 * l;
      for (int i = 0; i < ld; i++) {
        double s = 0;
        for (int r = 0; r < rows; r++) s += Jl[r * ld + i] * er[r];
        blv[i] += -w * s;
        for (int j = 0; j < ld; j++) {
          double h = 0;
          for (int r = 0; r < rows; r++) h += Jl[r * ld + i] * Jl[r * ld + j];
          Hl[i * ld + j] += w * h;
        }
      }
      double* Hpl = S->Hpl[t] + 24 * e;
      if (pi >= 0) {
        for (int i = 0; i < 6; i++) {
          double s = 0;
          for (int r = 0; r < rows; r++) s += Jp[r * 6 + i] * er[r];
          S->bp[6 * pi + i] += -w * s;
          for (int j = 0; j < 6; j++) {
            double h = 0;
            for (int r = 0; r < rows; r++) h += Jp[r * 6 + i] * Jp[r * 6 + j];
            S->Hpp[(6 * pi + i) * 6 * K + 6 * pi + j] += w * h;
          }
          for (int j = 0; j < ld; j++) {
            double h = 0;
            for (int r = 0; r < rows; r++) h += Jp[r * 6 + i] * Jl[r * ld + j];
            Hpl[i * ld + j] = w * h;
          }
        }
      }
    }
}

/* solve with lambda; x layout [6K | 3 nq | 4 nl].  returns 0 ok */
static int solve_system(ba_t* b, sys_t* S, int phase, double lambda, int** lm_edges, int* lm_off) {
  const int K = S->pose_idx_count, nq = b->nq, nl = b->nl, n6 = 6 * K;
  double* A = (double*)malloc(sizeof(double) * (n6 ? n6 * n6 : 1));
  double* bs = (double*)malloc(sizeof(double) * (n6 ? n6 : 1));
  memcpy(A, S->Hpp, sizeof(double) * n6 * n6);
  memcpy(bs, S->bp, sizeof(double) * n6);
  for (int i = 0; i < n6; i++) A[i * n6 + i] += lambda;
  int ok = 0;
  const int nlm = nq + nl;
  double* Dinv = (double*)malloc(sizeof(double) * 16 * (nlm ? nlm : 1));
  for (int g = 0; g < nlm; g++) {
    const int isq = g < nq, l = isq ? g : g - nq, ld = isq ? 3 : 4;
    if (!(isq ? S->qact[l] : S->lact[l])) continue;
    double H[16];
    memcpy(H, isq ? S->Hqq + 9 * l : S->Hll + 16 * l, sizeof(double) * ld * ld);
    for (int i = 0; i < ld; i++) H[i * ld + i] += lambda;
    if (small_inv(H, Dinv + 16 * g, ld)) { ok = -1; continue; }
    const double* blv = isq ? S->bq + 3 * l : S->bl + 4 * l;
    double db[4];
    for (int i = 0; i < ld; i++) {
      double s = 0;
      for (int j = 0; j < ld; j++) s += Dinv[16 * g + i * ld + j] * blv[j];
      db[i] = s;
    }
    for (int a = lm_off[g]; a < lm_off[g + 1]; a++) {
      const int t1 = lm_edges[0][a], e1 = lm_edges[1][a];
      if (!edge_active(b, t1, e1, phase)) continue;
      const int p1 = S->pidx[edge_pose(b, t1, e1)];
      if (p1 < 0) continue;
      const double* B1 = S->Hpl[t1] + 24 * e1;
      double BD[6][4];
      for (int i = 0; i < 6; i++) {
        double s = 0;
        for (int j = 0; j < ld; j++) {
          double t = 0;
          for (int k = 0; k < ld; k++) t += B1[i * ld + k] * Dinv[16 * g + k * ld + j];
          BD[i][j] = t;
          s += B1[i * ld + j] * db[j];
        }
        bs[6 * p1 + i] -= s;
      }
      for (int c = lm_off[g]; c < lm_off[g + 1]; c++) {
        const int t2 = lm_edges[0][c], e2 = lm_edges[1][c];
        if (!edge_active(b, t2, e2, phase)) continue;
        const int p2 = S->pidx[edge_pose(b, t2, e2)];
        if (p2 < 0) continue;
        const double* B2 = S->Hpl[t2] + 24 * e2;
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 6; j++) {
            double s = 0;
            for (int k = 0; k < ld; k++) s += BD[i][k] * B2[j * ld + k];
            A[(6 * p1 + i) * n6 + 6 * p2 + j] -= s;
          }
      }
    }
  }
  if (!ok && n6) ok = chol_solve(A, bs, n6);
  if (!ok) {
    memcpy(S->x, bs, sizeof(double) * n6);
    for (int g = 0; g < nlm; g++) {
      const int isq = g < nq, l = isq ? g : g - nq, ld = isq ? 3 : 4;
      double* xl = S->x + n6 + (isq ? 3 * l : 3 * nq + 4 * l);
      if (!(isq ? S->qact[l] : S->lact[l])) {
        for (int i = 0; i < ld; i++) xl[i] = 0;
        continue;
      }
      double c[4];
      const double* blv = isq ? S->bq + 3 * l : S->bl + 4 * l;
      for (int i = 0; i < ld; i++) c[i] = blv[i];
      for (int a = lm_off[g]; a < lm_off[g + 1]; a++) {
        const int t1 = lm_edges[0][a], e1 = lm_edges[1][a];
        if (!edge_active(b, t1, e1, phase)) continue;
        const int p1 = S->pidx[edge_pose(b, t1, e1)];
        if (p1 < 0) continue;
        const double* B1 = S->Hpl[t1] + 24 * e1;
        for (int j = 0; j < ld; j++) {
          double s = 0;
          for (int i = 0; i < 6; i++) s += B1[i * ld + j] * bs[6 * p1 + i];
          c[j] -= s;
        }
      }
      for (int i = 0; i < ld; i++) {
        double s = 0;
        for (int j = 0; j < ld; j++) s += Dinv[16 * g + i * ld + j] * c[j];
        xl[i] = s;
      }
    }
  }
  free(A); free(bs); free(Dinv);
  return ok;
}

static double compute_scale(const ba_t* b, const sys_t* S, double lambda) {
  const int n6 = 6 * S->pose_idx_count;
  double s = 0;
  for (int i = 0; i < n6; i++) s += S->x[i] * (lambda * S->x[i] + S->bp[i]);
  for (int l = 0; l < b->nq; l++)
    if (S->qact[l])
      for (int i = 0; i < 3; i++) s += S->x[n6 + 3 * l + i] * (lambda * S->x[n6 + 3 * l + i] + S->bq[3 * l + i]);
  for (int l = 0; l < b->nl; l++)
    if (S->lact[l])
      for (int i = 0; i < 4; i++) {
        const double xv = S->x[n6 + 3 * b->nq + 4 * l + i];
        s += xv * (lambda * xv + S->bl[4 * l + i]);
      }
  return s;
}

static void apply_update(ba_t* b, const sys_t* S) {
  const int n6 = 6 * S->pose_idx_count;
  for (int p = 0; p < b->np; p++)
    if (S->pidx[p] >= 0) {
      se3 dT = se3_exp(S->x + 6 * S->pidx[p]);
      b->T[p] = se3_mul(&dT, &b->T[p]);
    }
  for (int l = 0; l < b->nq; l++)
    if (S->qact[l])
      for (int i = 0; i < 3; i++) b->X[3 * l + i] += S->x[n6 + 3 * l + i];
  for (int l = 0; l < b->nl; l++)
    if (S->lact[l]) line_oplus(b->L + 6 * l, S->x + n6 + 3 * b->nq + 4 * l);
}

/* one g2o optimize(iters) run; returns iterations done, *chi2 = current chi2 */
static int optimize(ba_t* b, int phase, int iters, double* chi2_out) {
  sys_t S;
  memset(&S, 0, sizeof(S));
  const int np = b->np, nq = b->nq, nl = b->nl;
  /* active vertices */
  S.pidx = (int*)malloc(sizeof(int) * (np ? np : 1));
  S.qact = (unsigned char*)calloc(nq ? nq : 1, 1);
  S.lact = (unsigned char*)calloc(nl ? nl : 1, 1);
  unsigned char* pact = (unsigned char*)calloc(np ? np : 1, 1);
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b->ne[t]; e++) {
      if (!edge_active(b, t, e, phase)) continue;
      pact[edge_pose(b, t, e)] = 1;
      if (t < 2) S.qact[edge_lm(b, t, e)] = 1;
      else S.lact[edge_lm(b, t, e)] = 1;
    }
  int K = 0;
  for (int p = 0; p < np; p++) S.pidx[p] = (pact[p] && !b->P->pose_fixed[p]) ? K++ : -1;
  S.pose_idx_count = K;
  S.Hpp = (double*)malloc(sizeof(double) * (36 * K * K + 1));
  S.bp = (double*)malloc(sizeof(double) * (6 * K + 1));
  S.Hqq = (double*)malloc(sizeof(double) * (9 * nq + 1));
  S.bq = (double*)malloc(sizeof(double) * (3 * nq + 1));
  S.Hll = (double*)malloc(sizeof(double) * (16 * nl + 1));
  S.bl = (double*)malloc(sizeof(double) * (4 * nl + 1));
  for (int t = 0; t < 4; t++) S.Hpl[t] = (double*)calloc(24 * (size_t)b->ne[t] + 1, sizeof(double));
  S.x = (double*)calloc(6 * K + 3 * nq + 4 * nl + 1, sizeof(double));
  /* landmark -> edges CSR (points first, then lines) */
  const int nlm = nq + nl;
  int* lm_off = (int*)calloc(nlm + 1, sizeof(int));
  int tot = 0;
  for (int t = 0; t < 4; t++) tot += b->ne[t];
  int* lm_e[2] = {(int*)malloc(sizeof(int) * (tot + 1)), (int*)malloc(sizeof(int) * (tot + 1))};
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b->ne[t]; e++) lm_off[(t < 2 ? 0 : nq) + edge_lm(b, t, e) + 1]++;
  for (int g = 0; g < nlm; g++) lm_off[g + 1] += lm_off[g];
  int* fill = (int*)calloc(nlm + 1, sizeof(int));
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b->ne[t]; e++) {
      const int g = (t < 2 ? 0 : nq) + edge_lm(b, t, e);
      const int pos = lm_off[g] + fill[g]++;
      lm_e[0][pos] = t;
      lm_e[1][pos] = e;
    }
  /* backups */
  se3* Tb = (se3*)malloc(sizeof(se3) * (np + 1));
  double* Xb = (double*)malloc(sizeof(double) * (3 * nq + 1));
  double* Lb = (double*)malloc(sizeof(double) * (6 * nl + 1));

  const int robust = b->robust;
  double lambda = 0, ni = 2;
  int done = 0;
  double currentChi = 0;
  for (int it = 0; it < iters; it++) {
    currentChi = active_chi2(b, phase, robust);
    const double iniChi = currentChi;
    (void)iniChi;
    build_system(b, &S, phase, robust);
    if (it == 0) {
      double mx = 0;
      for (int i = 0; i < 6 * K; i++) mx = fmax(mx, fabs(S.Hpp[i * 6 * K + i]));
      for (int l = 0; l < nq; l++)
        if (S.qact[l])
          for (int i = 0; i < 3; i++) mx = fmax(mx, fabs(S.Hqq[9 * l + 4 * i]));
      for (int l = 0; l < nl; l++)
        if (S.lact[l])
          for (int i = 0; i < 4; i++) mx = fmax(mx, fabs(S.Hll[16 * l + 5 * i]));
      lambda = 1e-5 * mx;
      ni = 2;
    }
    double rho = 0;
    int qmax = 0;
    do {
      memcpy(Tb, b->T, sizeof(se3) * np);
      memcpy(Xb, b->X, sizeof(double) * 3 * nq);
      memcpy(Lb, b->L, sizeof(double) * 6 * nl);
      const int ok = solve_system(b, &S, phase, lambda, lm_e, lm_off) == 0;
      if (ok) apply_update(b, &S);
      double tempChi = active_chi2(b, phase, robust);
      if (!ok) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      const double scale = ok ? compute_scale(b, &S, lambda) + 1e-3 : 1.0;
      rho /= scale;
      if (rho > 0 && isfinite(tempChi) && ok) {
        double alpha = 1. - pow(2 * rho - 1, 3);
        alpha = fmin(alpha, 2. / 3.);
        const double sf = fmax(1. / 3., alpha);
        lambda *= sf;
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        memcpy(b->T, Tb, sizeof(se3) * np);
        memcpy(b->X, Xb, sizeof(double) * 3 * nq);
        memcpy(b->L, Lb, sizeof(double) * 6 * nl);
        if (!isfinite(lambda)) break;
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    done++;
    g_trials[phase - 1] += qmax;
    if (qmax == 10 || rho == 0 || !isfinite(lambda)) break;
  }
  *chi2_out = currentChi;
  free(S.pidx); free(S.qact); free(S.lact); free(pact);
  free(S.Hpp); free(S.bp); free(S.Hqq); free(S.bq); free(S.Hll); free(S.bl);
  for (int t = 0; t < 4; t++) free(S.Hpl[t]);
  free(S.x); free(lm_off); free(lm_e[0]); free(lm_e[1]); free(fill); free(Tb); free(Xb); free(Lb);
  return done;
}

int orc_ba_local(const rspl_ba_problem* P, rspl_ba_result* R) {
  ba_t b;
  memset(&b, 0, sizeof(b));
  b.P = P;
  b.np = P->n_poses;
  b.nq = P->n_points;
  b.nl = P->n_lines;
  b.ne[0] = P->n_mono;
  b.ne[1] = P->n_stereo;
  b.ne[2] = P->n_mono_line;
  b.ne[3] = P->n_stereo_line;
  b.T = (se3*)malloc(sizeof(se3) * (b.np + 1));
  for (int p = 0; p < b.np; p++) {
    se3 Twc;
    Twc.q[0] = P->pose_q[4 * p + 3];
    Twc.q[1] = P->pose_q[4 * p + 0];
    Twc.q[2] = P->pose_q[4 * p + 1];
    Twc.q[3] = P->pose_q[4 * p + 2];
    memcpy(Twc.t, P->pose_p + 3 * p, sizeof(Twc.t));
    se3_normalize(&Twc);
    b.T[p] = se3_inverse(&Twc);
  }
  b.X = (double*)malloc(sizeof(double) * (3 * b.nq + 1));
  memcpy(b.X, P->points, sizeof(double) * 3 * b.nq);
  b.L = (double*)malloc(sizeof(double) * (6 * b.nl + 1));
  memcpy(b.L, P->lines, sizeof(double) * 6 * b.nl);
  b.dmp = (double)(float)sqrt(P->th_mono_point);
  b.dsp = (double)(float)sqrt(P->th_stereo_point);
  b.dml = (double)(float)sqrt(P->th_mono_line);
  b.dsl = (double)(float)sqrt(P->th_stereo_line);
  for (int t = 0; t < 4; t++) {
    b.err[t] = (double*)calloc(4 * (size_t)b.ne[t] + 1, sizeof(double));
    b.level[t] = (unsigned char*)calloc(b.ne[t] + 1, 1);
  }
  const double th[4] = {P->th_mono_point, P->th_stereo_point, P->th_mono_line, P->th_stereo_line};
  /* phase 1: all edges, Huber */
  b.robust = 1;
  g_trials[0] = g_trials[1] = 0;
  R->iterations_done_first = optimize(&b, 1, P->iterations_first, &R->chi2_first);
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b.ne[t]; e++) {
      const double c2 = chi2_of(t, b.err[t] + 4 * e);
      int out = c2 > th[t];
      if (t < 2 && !depth_positive(&b, t, e)) out = 1;
      if (out) b.level[t][e] = 1;
    }
  /* phase 2: level-0 edges, no kernel */
  b.robust = 0;
  R->iterations_done_second = optimize(&b, 2, P->iterations_second, &R->chi2_second);
  uint8_t* inl[4] = {R->mono_inlier, R->stereo_inlier, R->mono_line_inlier, R->stereo_line_inlier};
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < b.ne[t]; e++) {
      int ok = chi2_of(t, b.err[t] + 4 * e) <= th[t];
      if (t < 2) ok = ok && depth_positive(&b, t, e);
      if (inl[t]) inl[t][e] = (uint8_t)ok;
    }
  for (int p = 0; p < b.np; p++) {
    se3 Twc = se3_inverse(&b.T[p]);
    R->pose_q[4 * p + 0] = Twc.q[1];
    R->pose_q[4 * p + 1] = Twc.q[2];
    R->pose_q[4 * p + 2] = Twc.q[3];
    R->pose_q[4 * p + 3] = Twc.q[0];
    memcpy(R->pose_p + 3 * p, Twc.t, sizeof(Twc.t));
  }
  memcpy(R->points, b.X, sizeof(double) * 3 * b.nq);
  memcpy(R->lines, b.L, sizeof(double) * 6 * b.nl);
  free(b.T); free(b.X); free(b.L);
  for (int t = 0; t < 4; t++) { free(b.err[t]); free(b.level[t]); }
  return 0;
}

/* exported helpers for tests: single-edge residual / line oplus */
void orc_line_oplus(double* L, const double* v) { line_oplus(L, v); }

/* one line edge's Jacobians at T_cw = (q w x y z, t): Jp [rows][6], Jl [rows][4] (rows 2 mono, 4 stereo),
 * analytic or g2o's central difference (test hook) */
void orc_line_jacobian(const double* cam, const double* q, const double* t, const double* L, const double* obs,
                       int stereo, int analytic, double* Jp, double* Jl) {
  se3 T;
  memcpy(T.q, q, sizeof(T.q));
  memcpy(T.t, t, sizeof(T.t));
  if (analytic) {
    line_jac_analytic(cam, &T, L, obs, stereo, Jp, Jl);
    return;
  }
  line_jac_numeric(cam, &T, L, obs, stereo, Jp, Jl);
}

/* ====================================================================== */
/* FrameOptimization (src/g2o_optimization/g2o_optimization.cc:256-398):   */
/* one VertexSE3Expmap (T_cw = SE3Quat(q,p).inverse(), :265), unary        */
/* EdgeSE3ProjectXYZOnlyPose (I2) / EdgeStereoSE3ProjectXYZOnlyPose (I3)   */
/* with Huber delta (float)sqrt(th) (:279-282); 4 rounds (:336-392): reset */
/* the estimate to the input pose, initializeOptimization(0), optimize(10);*/
/* then chi2 per edge -- re-computed at the current estimate only for      */
/* edges whose inlier flag is false (:345-347), otherwise the last error   */
/* the optimizer computed -- cast to float and compared with the threshold */
/* (:350-351) to set inlier / level; kernels dropped after round 2 (:363); */
/* stop after the first round when the graph holds < 10 edges (:383).      */
/* ====================================================================== */
typedef struct {
  const rspl_frame_problem* P;
  int n;          /* edges: mono [0, n_mono), stereo [n_mono, n) */
  double* err;    /* [n][3] last computed error */
  unsigned char* level;
  unsigned char* inl;
} fo_t;

static void fo_edge(const fo_t* f, int e, int* stereo, const double** X, const double** obs, const double** cam) {
  const rspl_frame_problem* P = f->P;
  const int s = e >= P->n_mono, i = s ? e - P->n_mono : e;
  const int32_t* cid = s ? P->stereo_camera : P->mono_camera;
  *stereo = s;
  *X = P->points + 3 * (s ? P->stereo_point[i] : P->mono_point[i]);
  *obs = s ? P->stereo_obs + 3 * i : P->mono_obs + 2 * i;
  *cam = P->cameras + 5 * (cid ? cid[i] : 0);
}

static void fo_error(const fo_t* f, const se3* T, int e, double* out) {
  int s;
  const double *X, *obs, *cam;
  fo_edge(f, e, &s, &X, &obs, &cam);
  double Xc[3];
  se3_map(T, X, Xc);
  const double iz = 1.0 / Xc[2];
  const double u = cam[0] * Xc[0] * iz + cam[2], v = cam[1] * Xc[1] * iz + cam[3];
  out[0] = obs[0] - u;
  out[1] = obs[1] - v;
  out[2] = s ? obs[2] - (u - cam[4] * iz) : 0.0;
}

static double fo_chi2(const double* e) { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }

static double fo_delta(const fo_t* f, int e) {
  return (double)(float)sqrt(e >= f->P->n_mono ? f->P->th_stereo_point : f->P->th_mono_point);
}

/* computeActiveErrors + activeRobustChi2 */
static double fo_active_chi2(fo_t* f, const se3* T, int robust) {
  double s = 0;
  for (int e = 0; e < f->n; e++) {
    if (f->level[e]) continue;
    fo_error(f, T, e, f->err + 3 * e);
    const double c2 = fo_chi2(f->err + 3 * e);
    if (robust) {
      double rho[2];
      huber(c2, fo_delta(f, e), rho);
      s += rho[0];
    } else {
      s += c2;
    }
  }
  return s;
}

/* H (6x6) and b = -J^T W e over the active edges at T, from the errors in f->err */
static void fo_build(fo_t* f, const se3* T, int robust, double* H, double* b) {
  memset(H, 0, sizeof(double) * 36);
  memset(b, 0, sizeof(double) * 6);
  for (int e = 0; e < f->n; e++) {
    if (f->level[e]) continue;
    int s;
    const double *X, *obs, *cam;
    fo_edge(f, e, &s, &X, &obs, &cam);
    double Xc[3];
    se3_map(T, X, Xc);
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    const double x = Xc[0], y = Xc[1], z = Xc[2], iz = 1.0 / z, iz2 = iz * iz;
    const double D[3][3] = {{fx * iz, 0, -fx * x * iz2}, {0, fy * iz, -fy * y * iz2}, {fx * iz, 0, -fx * x * iz2 + bf * iz2}};
    const double SX[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    double J[3][6];
    const int rows = s ? 3 : 2;
    for (int r = 0; r < rows; r++)
      for (int c = 0; c < 3; c++) {
        double a = 0;
        for (int k = 0; k < 3; k++) a += D[r][k] * SX[k * 3 + c];
        J[r][c] = a;
        J[r][3 + c] = -D[r][c];
      }
    const double* er = f->err + 3 * e;
    double w = 1.0;
    if (robust) {
      double rho[2];
      huber(fo_chi2(er), fo_delta(f, e), rho);
      w = rho[1];
    }
    for (int i = 0; i < 6; i++) {
      double g = 0;
      for (int r = 0; r < rows; r++) g += J[r][i] * er[r];
      b[i] += -w * g;
      for (int j = 0; j < 6; j++) {
        double h = 0;
        for (int r = 0; r < rows; r++) h += J[r][i] * J[r][j];
        H[i * 6 + j] += w * h;
      }
    }
  }
}

/* SparseOptimizer::optimize(iters) with OptimizationAlgorithmLevenberg on the pose vertex */
static int fo_optimize(fo_t* f, se3* T, int iters, int robust, double* chi2_out) {
  double H[36], b[36], A[36], x[6];
  double lambda = 0, ni = 2, currentChi = 0;
  int done = 0;
  for (int it = 0; it < iters; it++) {
    currentChi = fo_active_chi2(f, T, robust);
    fo_build(f, T, robust, H, b);
    if (it == 0) {
      double mx = 0;
      for (int i = 0; i < 6; i++) mx = fmax(mx, fabs(H[i * 7]));
      lambda = 1e-5 * mx;
      ni = 2;
    }
    double rho = 0;
    int qmax = 0;
    do {
      memcpy(A, H, sizeof(A));
      for (int i = 0; i < 6; i++) A[i * 7] += lambda;
      memcpy(x, b, sizeof(x));
      const int ok = chol_solve(A, x, 6) == 0;
      const se3 Tb = *T;
      if (ok) {
        se3 dT = se3_exp(x);
        *T = se3_mul(&dT, &Tb);
      }
      double tempChi = fo_active_chi2(f, T, robust);
      if (!ok) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 1.0;
      if (ok) {
        scale = 0;
        for (int i = 0; i < 6; i++) scale += x[i] * (lambda * x[i] + b[i]);
        scale += 1e-3;
      }
      rho /= scale;
      if (rho > 0 && isfinite(tempChi) && ok) {
        double alpha = 1. - pow(2 * rho - 1, 3);
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        *T = Tb;
        if (!isfinite(lambda)) break;
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    done++;
    if (qmax == 10 || rho == 0 || !isfinite(lambda)) break;
  }
  *chi2_out = currentChi;
  return done;
}

int orc_frame_opt(const rspl_frame_problem* P, rspl_frame_result* R) {
  fo_t f;
  memset(&f, 0, sizeof(f));
  f.P = P;
  f.n = P->n_mono + P->n_stereo;
  f.err = (double*)calloc(3 * (size_t)f.n + 1, sizeof(double));
  f.level = (unsigned char*)calloc(f.n + 1, 1);
  f.inl = (unsigned char*)calloc(f.n + 1, 1);
  for (int e = 0; e < f.n; e++) {
    const uint8_t* src = e < P->n_mono ? P->mono_inlier_in : P->stereo_inlier_in;
    f.inl[e] = src ? src[e < P->n_mono ? e : e - P->n_mono] : 1;
  }
  se3 Twc;
  Twc.q[0] = P->pose_q[3]; Twc.q[1] = P->pose_q[0]; Twc.q[2] = P->pose_q[1]; Twc.q[3] = P->pose_q[2];
  memcpy(Twc.t, P->pose_p, sizeof(Twc.t));
  se3_normalize(&Twc);
  const se3 T0 = se3_inverse(&Twc);
  se3 T = T0;
  int num_outlier = 0;
  R->rounds = 0;
  for (int r = 0; r < 4; r++) {
    T = T0;
    const int robust = r < 3;
    int active = 0;
    for (int e = 0; e < f.n; e++) active += !f.level[e];
    R->iterations[r] = 0;
    R->chi2[r] = 0;
    if (active) R->iterations[r] = fo_optimize(&f, &T, 10, robust, &R->chi2[r]);
    num_outlier = 0;
    for (int e = 0; e < f.n; e++) {
      double ev[3];
      if (!f.inl[e]) fo_error(&f, &T, e, f.err + 3 * e);
      memcpy(ev, f.err + 3 * e, sizeof(ev));
      const float c2 = (float)fo_chi2(ev);
      const double th = e < P->n_mono ? P->th_mono_point : P->th_stereo_point;
      if (c2 > th) {
        f.inl[e] = 0;
        f.level[e] = 1;
        num_outlier++;
      } else {
        f.inl[e] = 1;
        f.level[e] = 0;
      }
    }
    R->rounds = r + 1;
    if (f.n < 10) break;
  }
  const se3 W = se3_inverse(&T);
  R->pose_q[0] = W.q[1]; R->pose_q[1] = W.q[2]; R->pose_q[2] = W.q[3]; R->pose_q[3] = W.q[0];
  memcpy(R->pose_p, W.t, sizeof(W.t));
  for (int e = 0; e < f.n; e++) {
    uint8_t* dst = e < P->n_mono ? R->mono_inlier : R->stereo_inlier;
    if (dst) dst[e < P->n_mono ? e : e - P->n_mono] = f.inl[e];
  }
  R->n_inliers = f.n - num_outlier;
  free(f.err); free(f.level); free(f.inl);
  return 0;
}
